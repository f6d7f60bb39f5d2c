// tpl_runtime.cpp — operator lifetime, SpMV schedule, and the device-resident
// Lanczos drivers behind the C ABI (include/tpl.h).
//
// The Lanczos loops of the reference (src/algorithms/lanczos.rs:86-128,
// src/algorithms/lanczos_two_pass.rs:84-102 and :266-309) run entirely on the GPU:
// the per-step launches are captured once per (variant, k) into a hipGraph and
// replayed, alpha/beta never leave HBM during a pass, and breakdown is handled
// on the device (a stop flag turns the remaining launches into no-ops). The only
// host round trip of a solve is the f(T_k) call between the passes, exactly
// where the reference calls its closure (src/solvers.rs:71-75, :155-156).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "tpl_device.h"
#include "tpl_internal.h"
#include "tpl_layout.h"

#ifndef TPL_LAB
#define TPL_LAB 0  // lab builds only (scripts/build_variants.sh): runtime layout knobs
#endif

namespace tpl {
namespace launch {
hipError_t spmv(const CsrDev& A, const double* x, double* y, hipStream_t s);
hipError_t p1_init(const CsrDev& A, const DevState& S, const double* b, hipStream_t s);
// stamp: workgroup 0 records the launch's start there (live timing), or nullptr
hipError_t p1_spmv(const CsrDev& A, const DevState& S, const double* xsrc, const double* r_cur,
                   const double* r_prev, double* W, double* Vcol, int j, hipStream_t s,
                   unsigned long long* stamp = nullptr);
// elim: one more workgroup eliminates row j - 3 of T_k's LU (one-graph inv)
hipError_t p1_axpy(const CsrDev& A, const DevState& S, const double* W, const double* r_cur,
                   double* r_next, int j, int k, int elim, hipStream_t s,
                   unsigned long long* stamp = nullptr);
hipError_t p2_tail(int64_t n, const DevState& S, double* x, double* const V[3], hipStream_t s);
hipError_t permute(int64_t n, int cols, double* out, int64_t ldo, const double* in, int64_t ldi,
                   const int32_t* idx, hipStream_t s);
hipError_t ftk_inv(const DevState& S, int kcap, int scale, hipStream_t s);
hipError_t ftk_exp(const DevState& S, int kcap, int scale, hipStream_t s);
hipError_t p2_init(int64_t n, const DevState& S, const double* b, double* v1, double* x,
                   double* Vcol, int dyn, hipStream_t s);
// nflush: x terms the step applies (tpl::p2_flush: every third step and the last)
hipError_t p2_spmv(const CsrDev& A, const DevState& S, const double* xsrc, const double* v_cur,
                   const double* v_prev, double* v_next, double* x, double* Vcol, int j,
                   int nflush, hipStream_t s);
// pass-two step records (EpiPass2R) for steps 1 .. k-1; dyn: activity from the device count
hipError_t p2_coefs(const DevState& S, int k, int dyn, hipStream_t s);
hipError_t gemv_recon(int64_t n, int steps, const DevState& S, const double* V, double* x,
                      hipStream_t s);
hipError_t long_epi_p1(const CsrDev& A, const DevState& S, const double* yall, int R,
                       const double* r_cur, const double* r_prev, double* W, double* Vcol,
                       double* Pa_long, int j, hipStream_t s);
hipError_t long_epi_p2(const CsrDev& A, const DevState& S, const double* yall, int R,
                       const double* v_cur, const double* v_prev, double* v_next, double* x,
                       double* Vcol, int j, int nflush, hipStream_t s);
hipError_t long_epi_y(const CsrDev& A, const double* yall, int R, double* y, hipStream_t s);
hipError_t reorth_decide(const DevState& S, const double* Pb1, int G2, int* skip, int* rec,
                         hipStream_t s);
hipError_t reorth_dot(int64_t n, int cols, const double* V, const double* r, double* P, int G,
                      int64_t E, const int* skip, hipStream_t s);
hipError_t reorth_reduce(int cols, const double* P, int G, double* h, const int* skip, hipStream_t s);
hipError_t reorth_update(int64_t n, int cols, const double* V, double* r, const double* h,
                         double* Pnorm, int G, int64_t E, const int* skip, hipStream_t s);
} // namespace launch

#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      ::tpl::fail(e_ == hipErrorOutOfMemory ? TPL_ERR_OUT_OF_MEMORY : TPL_ERR_DEVICE,       \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                       \
  } while (0)

template <class F>
static tpl_status guarded(F&& f) {
  try {
    f();
    set_last_error("");
    return TPL_OK;
  } catch (const Error& e) {
    // a failed HIP call leaves its status as the runtime's "last error", which the next
    // launch's hipGetLastError() check would report as its own: clear it here
    if (e.code == TPL_ERR_DEVICE || e.code == TPL_ERR_OUT_OF_MEMORY) (void)hipGetLastError();
    set_last_error(e.code, e.msg, e.det);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error(TPL_ERR_OUT_OF_MEMORY, "host allocation failed", {});
    return TPL_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    set_last_error(TPL_ERR_INVALID_ARGUMENT, e.what(), {});
    return TPL_ERR_INVALID_ARGUMENT;
  }
}

} // namespace tpl

using namespace tpl;

// ---------------------------------------------------------------- objects
struct tpl_ctx_s {
  int device = 0;
  hipStream_t stream = nullptr;
};

// A rank of a row-partitioned operator (tpl_dist_create*): its GPU and stream, and the
// transport of the per-step exchanges — RCCL over xGMI, or (tests) a host callback.
struct tpl_dist_s {
  tpl_ctx_s ctx;
  int rank = 0, nranks = 1;
  ncclComm_t comm = nullptr;
  tpl_allgather_fn host_fn = nullptr;
  void* host_user = nullptr;
};

namespace {
enum GraphKind {
  kGPass1 = 0, kGStandard = 1, kGPass2 = 2, kGPass2Steps = 3,
  kGTwoPassDev = 4,   // one-graph solve: pass one, device f(T_k), pass two
  kGDevFtk = 5,       // (timed variant) device f(T_k) + pass-two prologue
  kGPass2Dyn = 6,     // (timed variant) the k - 1 step launches of a one-graph solve
  kGPass1Elim = 7,    // (timed variant) pass one eliminating T_k's LU as it goes
  kGStandardElim = 8, // the standard pass eliminating T_k's LU as it goes (one-pass inv)
  kGPass1Stamped = 9, // (timed variant) pass one with start stamps on kStampSteps steps
  kGPass1ElimStamped = 10,
};
// Live timing of pass one's kernels (tpl_op_step_samples): in a timed solve, workgroup 0
// of the k_p1_spmv and k_p1_axpy launches of kStampSteps consecutive middle steps (and of
// the next step's k_p1_spmv) records its start on the 100 MHz real-time clock; a kernel's
// launch time is the start-to-start interval, boundary included (as pass two's figure).
constexpr int kStampSteps = 8;
// Callback polling (tpl_lanczos_standard with a step callback): largest batch of steps
// run ahead of the host callback.
constexpr int kCbBatchMax = 32;
// One-graph solves keep the device f(T_k)'s working rows in LDS (k_ftk_inv: 11 k doubles,
// 120 KB at this k; gfx950 has 160 KiB of LDS per workgroup).
constexpr size_t kDevFtkMaxK = 1365;
// Auto mode: the device inv up to k = 500, the largest k at which it was measured no
// slower than the host round trip it replaces. Its elimination runs during pass one
// (k_p1_axpy's extra workgroup) and its back substitution with Markstein divisions (round
// 4, same box, profiles/r04_ftk_timing.txt: 0.574 vs 0.583 ms at 5k arcs k = 50, 2.390 vs
// 2.412 at 50k k = 200, 9.312 vs 9.315 ms at the 500k headline k = 500); past that the
// serial back substitution grows longer than the round trip (round 5, same box,
// profiles/r05_ftk_timing.txt: 10.36 vs 10.24 ms at 5k arcs k = 1000, 14.16 vs 13.84 at
// k = 1365; 11.18 vs 10.99 and 15.62 vs 15.05 ms at 50k arcs). Mode 1 still takes the
// device inv up to kDevFtkMaxK.
constexpr size_t kDevFtkAutoK = 500;
// The device exp (k_ftk_exp, a Chebyshev expansion: parallel over the rows of T_k) keeps
// 4 k + 4 doubles of dynamic LDS plus 8.2 KB of static arrays: 65.8 KB at this k, which
// gfx950's 160 KiB of LDS per workgroup holds (a 64 KiB part would need k <= 1790).
constexpr size_t kDevExpMaxK = 1800;
// Which built-in f(T_k) a one-graph solve evaluates on the device.
enum DevF { kDevInv = 0, kDevExp = 1 };
// Locality order, auto mode: on up to this many rows. Measured k_p2_spmv (KKT, D = 0;
// profiles/r02_order_lab.txt): 500k arcs 8.76 -> 6.91 us, 1M arcs 12.8 -> 11.8 us,
// 50k / 5k arcs flat; 2M arcs 20.5 -> 21.8 us and 5M arcs 54 -> 58 us (the gathered
// vector, 16-40 MB, no longer fits the XCDs' L2s).
constexpr int64_t kReorderAutoMaxRows = 1 << 20;
}

struct tpl_op_s {
  tpl_ctx_s* ctx = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t n = 0, nnz = 0;           // this operator's rows (the rank's block) and nonzeros
  // row partition (tpl_dist_op_create_csr); single GPU: dist == nullptr, n_glob == n
  tpl_dist_s* dist = nullptr;
  int64_t n_glob = 0;
  std::vector<int64_t> starts;
  bool eager = false;               // launch without graphs (host transport / no capture)
  // replicated-long-row partition ("hybrid"): local vector = [own short rows | all long
  // rows]; g2l maps global rows/columns to local indices (-1: not local), local_rows back
  bool hybrid = false;
  int64_t ns_local = 0;
  std::vector<int32_t> g2l;
  std::vector<int64_t> local_rows;
  double* d_yall = nullptr;         // nranks x y_ld1 (pass one: long-row partials + the
                                    // rank's short-chunk alpha partials, all-gathered
                                    // together); pass two: nranks x (n_long + 1)
  int32_t y_ld1 = 0;                // n_long + the most chunks of any rank
  std::vector<int32_t> nch;         // chunks (alpha partials) of every rank
  std::vector<int32_t> g2s;         // norm partials (element-wise blocks) of every rank
  int32_t pb_ld = 0;                // > 0: every rank's norm partials all-gathered (CsrDev::pb_ld)
  double* d_pball = nullptr;        // [nranks x pb_ld] gathered norm partials (pb_ld > 0)
  int32_t* d_nch = nullptr;
  // halo-exchange row blocks (tpl_dist_op_create_halo): the gathered vector is
  // [own block (ld) | nranks x hH halo slots]; rank q's slot holds the hH_q <= hH rows of
  // its block that some other rank's rows reference (halo_send: their local indices),
  // packed before each all-gather; halo_map: global column -> device position
  bool halo = false;
  int64_t hH = 0;
  std::vector<int32_t> halo_send, halo_map;
  int32_t* d_halo_send = nullptr;
  std::vector<int32_t> h_rowptr;
  std::vector<int32_t> h_col;
  std::vector<double> h_val;
  SchedParams sp;
  Layout lay;
  void* d_bcol = nullptr;
  int32_t* d_bcbase = nullptr;
  int32_t* d_bhdr = nullptr;
  int32_t* d_scbase = nullptr;
  void* d_bval = nullptr;
  BinSeg* d_bseg = nullptr;
  double* d_P = nullptr;
  unsigned int* d_Pcnt = nullptr;
  int32_t* d_srows = nullptr;
  void* d_scol = nullptr;
  void* d_sval = nullptr;
  int32_t* d_cbase = nullptr;
  int32_t* d_cwidth = nullptr;
  // vectors: b, R0..R2, W, x, V2_0..V2_2, tmp (n each, padded)
  double* d_vecs = nullptr;
  int64_t ld = 0;
  double *b = nullptr, *R[3] = {nullptr, nullptr, nullptr}, *W = nullptr, *x = nullptr,
         *V2[3] = {nullptr, nullptr, nullptr}, *tmp = nullptr;
  // gather sources of the SpMV: the same buffers on one GPU; with a partition, the
  // all-gathered vectors (nranks x ld) whose rank-th slice the local pointers view
  double *bG = nullptr, *RG[3] = {nullptr, nullptr, nullptr}, *V2G[3] = {nullptr, nullptr, nullptr},
         *tmpG = nullptr;
  double* d_rsum = nullptr;         // [nranks alpha totals][nranks norm totals] (partition)
  // solver state
  size_t kcap = 0;
  void* d_state = nullptr;  // flags | norms | alphas | betas | y | Pa | Pb | Pr
  void* h_state = nullptr;  // pinned mirror of flags | norms | alphas | betas
  DevState S{};
  double* d_Pr = nullptr;   // reorthogonalisation partials (G * kcap)
  double* d_V = nullptr;    // standard-variant basis (n x vcols, ld = n)
  size_t vcols = 0;
  std::map<std::pair<int, size_t>, hipGraphExec_t> graphs;
  // device allocations of this operator (pointer -> bytes): tpl_op_device_bytes
  std::map<const void*, size_t> allocs;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // live timing (tpl_op_enable_timing): events recorded inside the captured passes
  bool timing = false;
  int device_ftk = 2;               // built-in inv on the device (one graph): 0 off, 1 on, 2 auto
  bool last_one_graph = false;      // the last tpl_lanczos_two_pass ran as one device graph
  int64_t reorth_second = 0;        // second Gram-Schmidt passes of the last reorth solve
  // locality order (single GPU, tpl_op_set_reorder): the device works on P A P^T; vectors
  // cross the boundary through a gather (internal i <- caller's perm[i], back via iperm).
  // h_rowptr / h_col / h_val keep the caller's order.
  int reorder = 2;                  // 0 off, 1 on, 2 auto (n <= kReorderAutoMaxRows)
  bool local_order = false;         // replicated partition: own short rows in locality order
  std::vector<int32_t> perm, iperm;
  int32_t* d_perm = nullptr;
  int32_t* d_iperm = nullptr;
  double* d_stage = nullptr;        // one host-order vector (host uploads / downloads)
  double* d_Vext = nullptr;         // the callback's V_k view in the caller's order
  size_t vext_cols = 0;
  hipEvent_t tev[4] = {nullptr, nullptr, nullptr, nullptr};
  int64_t p2_launches = 0;
  // live timing of pass one's kernels: start stamps of the last timed solve's sampled
  // launches (2 kStampSteps + 1), tpl_op_step_samples
  unsigned long long* d_stamps = nullptr;
  int32_t p1_samples = 0;
  // tpl_plan_create: the host half of an operator only (rows, order, layout), for the
  // oracle's reduction order without a GPU; every device entry point refuses it
  bool plan_only = false;
  std::unique_ptr<tpl_dist_s> plan_dist;  // a plan's rank and rank count (no transport)
};

namespace {

bool use_graphs() {
  const char* e = std::getenv("TPL_NO_GRAPH");
  return !(e && e[0] == '1');
}

int long_epi_blocks(const tpl_op_s* op) {
  return (int)((op->lay.lrows.size() + kLongEpiRows - 1) / kLongEpiRows);
}

CsrDev csr_dev(const tpl_op_s* op, bool pass1 = false) {
  const Layout& L = op->lay;
  CsrDev A;
  A.srows = op->d_srows;
  A.s_col = op->d_scol;
  A.s_val = op->d_sval;
  A.val_i8 = L.val_i8 ? 1 : 0;
  A.s_col16 = L.s_col16 ? 1 : 0;
  A.b_col16 = L.b_col16 ? 1 : 0;
  A.s_cbase = op->d_scbase;
  A.b_cbase = op->d_bcbase;
  A.c_base = op->d_cbase;
  A.c_width = op->d_cwidth;
  A.b_col = op->d_bcol;
  A.b_val = op->d_bval;
  A.b_seg = op->d_bseg;
  A.b_hdr = op->d_bhdr;
  A.P = op->d_P;
  A.Pcnt = op->d_Pcnt;
  A.s_width = L.s_width;
  A.s_identity = L.s_identity;
  A.n_short = (int32_t)L.srows.size();
  A.n_chunks = (int32_t)L.c_base.size();
  A.n_long = (int32_t)L.lrows.size();
  A.bin_cap = L.bin_cap;
  A.n_slices = L.nslices;
  A.n_slice_blocks = L.nslices * L.M;
  A.G2 = L.G2;
  A.NA = A.n_chunks + A.n_long;
  A.NA_r = op->dist ? op->dist->nranks + (op->hybrid ? long_epi_blocks(op) : 0) : A.NA;
  A.G2_r = op->dist ? op->dist->nranks : A.G2;
  A.pb_ld = op->pb_ld;
  A.long_defer = op->hybrid ? 1 : 0;
  A.y_ld = pass1 && op->hybrid ? op->y_ld1 : (int32_t)L.lrows.size() + 1;
  A.ypart = op->hybrid ? op->d_yall + (size_t)op->dist->rank * A.y_ld : nullptr;
  A.nch = op->d_nch;
  A.norm_n = op->hybrid && op->dist->rank != 0 ? op->ns_local : op->n;
  A.s_win = L.s_win;
  A.s_win_max = L.s_win_max;
  A.n = op->n;
  A.E = L.E;
  return A;
}

void drop_graphs(tpl_op_s* op) {
  for (auto& kv : op->graphs) hipGraphExecDestroy(kv.second);
  op->graphs.clear();
}

// Device memory of an operator, accounted per allocation (tpl_op_device_bytes).
template <class T>
void dev_alloc(tpl_op_s* op, T** p, size_t bytes) {
  HIPCHK(hipMalloc(p, bytes));
  op->allocs[*p] = bytes;
}
template <class T>
void dev_free(tpl_op_s* op, T*& p) {
  if (!p) return;
  op->allocs.erase(p);
  hipFree(p);
  p = nullptr;
}

template <class T>
void upload(tpl_op_s* op, T** dst, const std::vector<T>& src) {
  dev_free(op, *dst);
  if (src.empty()) return;
  dev_alloc(op, dst, src.size() * sizeof(T));
  HIPCHK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
}

void rebuild_schedule(tpl_op_s* op) {
  ColMap cmap;
  if (op->halo) {
    cmap.table = &op->halo_map;
  } else if (op->dist && !op->hybrid) {
    cmap.starts = &op->starts;
    cmap.ld = op->ld;
  }
  op->perm.clear();
  op->iperm.clear();
  const bool want = op->reorder == 1 || (op->reorder == 2 && op->n <= kReorderAutoMaxRows);
  if (want && !op->dist) op->perm = locality_order(op->n, op->h_rowptr, op->h_col, op->sp);
  std::vector<int32_t> prp, pcol;
  std::vector<double> pval;
  if (!op->perm.empty()) {
    op->iperm.resize(op->n);
    for (int64_t i = 0; i < op->n; ++i) op->iperm[op->perm[i]] = (int32_t)i;
    permute_csr(op->n, op->h_rowptr, op->h_col, op->h_val, op->perm, op->iperm, prp, pcol, pval);
  }
  const bool p = !op->perm.empty();
  // In the locality order a chunk's rows share their hub columns, so its gathers hit
  // few lines and the LDS window costs more than it saves (measured +0.4 us per SpMV at
  // 500k): window only in the caller's order.
  SchedParams sp = op->sp;
  sp.window = !p && !op->local_order;
#if TPL_LAB
  // layout knobs of the lab builds (scripts/build_variants.sh -DTPL_LAB=1), never in the
  // product library: the measured alternatives of DESIGN.md §3/§4
  if (const char* e = std::getenv("TPL_WINDOW")) sp.window = std::atoi(e) != 0;
  if (const char* e = std::getenv("TPL_ELEM_ROWS")) sp.elem_rows = std::atoi(e);
  if (const char* e = std::getenv("TPL_BIN_LINES")) sp.bin_lines = std::atoi(e);
  if (const char* e = std::getenv("TPL_BIN_SEGS")) sp.bin_segs = std::atoi(e);
  if (const char* e = std::getenv("TPL_BIN_BIG")) sp.bin_big = std::atoi(e);
  if (const char* e = std::getenv("TPL_BIN_SMALL")) sp.bin_small = std::atoi(e);
  if (const char* e = std::getenv("TPL_BIN_BALANCE")) sp.bin_balance = std::atoi(e);
  if (const char* e = std::getenv("TPL_BIN_CROWD")) sp.bin_crowd = std::atof(e);
  if (const char* e = std::getenv("TPL_SLICES")) {  // auto slice count only; the values
    const int s = std::atoi(e);                     // tpl_op_set_slices accepts
    if (sp.slices <= 0 && s > 0 && s <= kSlices && (s & (s - 1)) == 0) sp.slices = s;
  }
#endif
  // slice bounds over global columns — or, replicated-long-row partition, over this
  // rank's local columns (its CSR is stored in local indices)
  op->lay = build_layout(op->n, op->hybrid ? op->n : op->n_glob, p ? prp : op->h_rowptr,
                         p ? pcol : op->h_col, p ? pval : op->h_val, sp, cmap);
  // the replicated partition's ranks agree on every rank's element-wise block count (the
  // gathered norm partials, the alpha partial counts): a layout that changed it is refused
  if (op->hybrid && !op->g2s.empty() && op->lay.G2 != op->g2s[op->dist->rank])
    fail(TPL_ERR_UNSUPPORTED, "replicated partition: the element-wise blocks must stay those "
                              "every rank computed from the split");
  if (op->plan_only) return;  // tpl_plan_create: the layout is all a plan holds
  const Layout& L = op->lay;
  upload(op, &op->d_perm, op->perm);
  upload(op, &op->d_iperm, op->iperm);
  dev_free(op, op->d_stage);
  dev_free(op, op->d_Vext);
  op->vext_cols = 0;
  if (p) dev_alloc(op, &op->d_stage, (size_t)op->n * sizeof(double));
  upload(op, &op->d_srows, L.srows);
  // entries in the device order (tpl_device.h kPackedEntries; positions unchanged)
  const bool pack_s = packed_chunk_width(L.s_width);
  auto sidx = [&](int64_t i) { return pack_s ? packed_chunk_index(i, L.s_width) : i; };
  auto bidx = [&](int64_t i) { return kPackedEntries ? packed_bin_index(i, L.bin_cap) : i; };
  if (L.s_col16)
    upload(op, reinterpret_cast<uint16_t**>(&op->d_scol), to_device_order(L.s_col16v, sidx));
  else
    upload(op, reinterpret_cast<int32_t**>(&op->d_scol), to_device_order(L.s_col, sidx));
  upload(op, &op->d_scbase, L.s_cbase);
  if (L.val_i8)
    upload(op, reinterpret_cast<int8_t**>(&op->d_sval), to_device_order(L.s_val8, sidx));
  else
    upload(op, reinterpret_cast<double**>(&op->d_sval), to_device_order(L.s_val, sidx));
  upload(op, &op->d_cbase, L.c_base);
  upload(op, &op->d_cwidth, L.c_width);
  if (L.b_col16)
    upload(op, reinterpret_cast<uint16_t**>(&op->d_bcol), to_device_order(L.b_col16v, bidx));
  else
    upload(op, reinterpret_cast<int32_t**>(&op->d_bcol), to_device_order(L.b_col, bidx));
  upload(op, &op->d_bcbase, L.b_cbase);
  if (L.val_i8)
    upload(op, reinterpret_cast<int8_t**>(&op->d_bval), to_device_order(L.b_val8, bidx));
  else
    upload(op, reinterpret_cast<double**>(&op->d_bval), to_device_order(L.b_val, bidx));
  upload(op, &op->d_bseg, L.b_seg);
  upload(op, &op->d_bhdr, L.b_hdr);
  // piece slots, and the arrival counters of the sliced long rows (zero; each wraps at
  // its row's packed-piece count, BinSeg::pad + 1, so it runs on across launches)
  upload(op, &op->d_P, std::vector<double>(std::max<size_t>(L.lrows.size() * kSlotStride, 1), 0.0));
  upload(op, &op->d_Pcnt,
         std::vector<unsigned int>(std::max<size_t>(L.lrows.size() * kCntStride, 1), 0u));
  drop_graphs(op);
  // partial buffers depend on the layout: force state reallocation
  op->kcap = 0;
}

// state layout: [flags: 8 int32 (kFlagBytes)] [norms kcap+1] [alphas kcap] [betas kcap] [y kcap]
// [Pa NA] [Pb G2] [p2c 8 kcap] [lu 4 kcap + 3]; reorthogonalisation partials separately (d_Pr)
void ensure_state(tpl_op_s* op, size_t k, bool reorth = false) {
  if (k > op->kcap) {
    const size_t kc = std::max<size_t>(k, 16);
    drop_graphs(op);
    dev_free(op, op->d_state);
    if (op->h_state) HIPCHK(hipHostFree(op->h_state));
    dev_free(op, op->d_Pr);
    op->d_state = nullptr;
    op->h_state = nullptr;
    op->d_Pr = nullptr;
    const CsrDev A = csr_dev(op);
    // [.. | Pb G2 | pad to 64 B | p2c: 8 kc step records | lu: 4 kc + 3]
    const size_t head = kFlagBytes / sizeof(double) + (kc + 1) + 3 * kc +
                        (size_t)std::max(A.NA, 1) + (size_t)A.G2;
    const size_t p2c_off = (head + 7) / 8 * 8;  // in doubles from the base (64-B aligned)
    const size_t doubles = p2c_off - kFlagBytes / sizeof(double) + 8 * kc + 4 * kc + 3;
    const size_t bytes = kFlagBytes + doubles * sizeof(double);
    dev_alloc(op, &op->d_state, bytes);
    HIPCHK(hipMemset(op->d_state, 0, bytes));
    HIPCHK(hipHostMalloc(&op->h_state, kFlagBytes + (4 * kc + 1) * sizeof(double),
                         hipHostMallocDefault));
    char* base = (char*)op->d_state;
    op->S.flags = (int32_t*)base;
    op->S.norms = (double*)(base + kFlagBytes);
    op->S.alphas = op->S.norms + (kc + 1);
    op->S.betas = op->S.alphas + kc;
    op->S.y = op->S.betas + kc;
    op->S.Pa = op->S.y + kc;
    op->S.Pb = op->S.Pa + std::max(A.NA, 1);
    op->S.p2c = reinterpret_cast<double*>(base) + p2c_off;
    op->S.lu = op->S.p2c + 8 * kc;
    op->S.kcap = (int32_t)kc;
    // hybrid: the chunks' alpha partials go straight into this rank's pass-one segment of
    // the all-gather (k_long_epi_p1 reduces every rank's after the exchange)
    if (op->hybrid)
      op->S.Pa = op->d_yall + (size_t)op->dist->rank * op->y_ld1 + op->lay.lrows.size();
    op->S.Pa_r = op->dist ? op->d_rsum : op->S.Pa;
    op->S.Pb_r = op->dist ? op->d_rsum + A.NA_r : op->S.Pb;
    if (op->pb_ld > 0) {  // the norm partials go straight into this rank's gathered segment
      op->S.Pb = op->d_pball + (size_t)op->dist->rank * op->pb_ld;
      op->S.Pb_r = op->d_pball;
    }
    op->kcap = kc;
  }
  if (reorth && !op->d_Pr) {
    // [cols x G partials][cols coefficients][G norm partials after the first pass][skip flag]
    // [kcap per-step second-pass records (int)]
    dev_alloc(op, &op->d_Pr,
              (((size_t)op->lay.G2 + 2) * op->kcap + (size_t)op->lay.G2 + 1) * sizeof(double));
  }
}

void ensure_basis(tpl_op_s* op, size_t cols) {
  if (cols <= op->vcols && op->d_V) return;
  drop_graphs(op);
  dev_free(op, op->d_V);
  op->d_V = nullptr;
  op->vcols = 0;
  const size_t c = std::max<size_t>(cols, 1);
  dev_alloc(op, &op->d_V, (size_t)op->n * c * sizeof(double) + 64);
  op->vcols = c;
}

void set_device(const tpl_op_s* op) {
  if (op->plan_only)
    fail(TPL_ERR_INVALID_ARGUMENT, "a host-only plan (tpl_plan_create) holds no device data");
  HIPCHK(hipSetDevice(op->device));
}

void check_b(const tpl_op_s* op, const double* b, int64_t b_len) {
  if (!b && op->n > 0) fail(TPL_ERR_INVALID_ARGUMENT, "b is NULL");
  if (b_len != op->n) fail_dimension(op->n, b_len);
}

// A caller-order vector into a device vector (internal order).
void upload_vec(tpl_op_s* op, double* dst, const double* src, int mem) {
  if (op->n == 0) return;
  const size_t bytes = op->n * sizeof(double);
  if (!op->d_perm) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes,
                          mem == TPL_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                          op->stream));
    return;
  }
  const double* from = src;
  if (mem != TPL_MEM_DEVICE) {
    HIPCHK(hipMemcpyAsync(op->d_stage, src, bytes, hipMemcpyHostToDevice, op->stream));
    from = op->d_stage;
  }
  HIPCHK(launch::permute(op->n, 1, dst, op->n, from, op->n, op->d_perm, op->stream));
}
// `cols` device columns (internal order, ld = n) out to the caller, in the caller's order.
void download_vec(tpl_op_s* op, double* dst, const double* src, int64_t cols, int mem) {
  if (cols == 0 || op->n == 0) return;
  // one vector, or columns of the basis: nothing else is ever this wide
  if (cols < 0 || (cols > 1 && (src != op->d_V || (size_t)cols > op->vcols)))
    fail(TPL_ERR_INVALID_ARGUMENT, "download_vec: column count exceeds its source");
  if (!op->d_perm) {
    HIPCHK(hipMemcpyAsync(dst, src, cols * op->n * sizeof(double),
                          mem == TPL_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                          op->stream));
    return;
  }
  if (mem == TPL_MEM_DEVICE) {
    HIPCHK(launch::permute(op->n, (int)cols, dst, op->n, src, op->n, op->d_iperm, op->stream));
    return;
  }
  for (int64_t c = 0; c < cols; ++c) {  // through the staging vector, a column at a time
    HIPCHK(launch::permute(op->n, 1, op->d_stage, op->n, src + c * op->n, op->n, op->d_iperm,
                           op->stream));
    HIPCHK(hipMemcpyAsync(dst + c * op->n, op->d_stage, op->n * sizeof(double),
                          hipMemcpyDeviceToHost, op->stream));
  }
}

// r_j buffer of pass one: r_1 = b, then R[j % 3] (local view, and gather source).
inline double* r_of(const tpl_op_s* op, int j) { return j == 1 ? op->b : op->R[j % 3]; }
inline double* rG_of(const tpl_op_s* op, int j) { return j == 1 ? op->bG : op->RG[j % 3]; }

// ---- exchanges of a row-partitioned operator -------------------------------------
#define NCCLCHK(expr)                                                                       \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess)                                                                  \
      ::tpl::fail(TPL_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(r_));     \
  } while (0)

// In-place all-gather of `count` doubles per rank: rank r's part sits at base + r*count.
void dist_allgather(tpl_op_s* op, double* base, size_t count) {
  tpl_dist_s* d = op->dist;
  if (d->comm && std::getenv("TPL_TEST_REFUSE_CAPTURE")) {
    // test hook: behave like a transport that cannot be captured into a graph
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(op->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) fail(TPL_ERR_DEVICE, "exchange refused stream capture (test hook)");
  }
  if (d->comm) {
    NCCLCHK(ncclAllGather(base + (size_t)d->rank * count, base, count, ncclDouble, d->comm,
                          op->stream));
    return;
  }
  // host transport (tests): stage through host memory around the callback
  std::vector<double> send(count), recv(count * (size_t)d->nranks);
  HIPCHK(hipMemcpyAsync(send.data(), base + (size_t)d->rank * count, count * sizeof(double),
                        hipMemcpyDeviceToHost, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  if (d->host_fn(send.data(), recv.data(), count * sizeof(double), d->host_user) != 0)
    fail(TPL_ERR_DEVICE, "host all-gather callback failed");
  HIPCHK(hipMemcpyAsync(base, recv.data(), recv.size() * sizeof(double), hipMemcpyHostToDevice,
                        op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
}
// Row blocks: complete the gather source G of this rank's SpMV. Plain row blocks
// all-gather every rank's whole block (ld doubles each, in place); halo blocks first pack
// the rows other ranks reference into this rank's halo slot (halo_pack, k_permute — issued
// before the collective group) and all-gather the slots only (hH doubles each).
void halo_pack(tpl_op_s* op, double* G) {
  if (!op->halo || op->halo_send.empty()) return;
  HIPCHK(launch::permute((int64_t)op->halo_send.size(), 1,
                         G + op->ld + (size_t)op->dist->rank * op->hH, 0, G, 0,
                         op->d_halo_send, op->stream));
}
void gather_vec(tpl_op_s* op, double* G) {
  if (!op->halo) dist_allgather(op, G, (size_t)op->ld);
  else if (op->hH > 0) dist_allgather(op, G + op->ld, (size_t)op->hH);
}
void dist_group(tpl_op_s* op, bool begin) {
  if (op->dist && op->dist->comm) NCCLCHK(begin ? ncclGroupStart() : ncclGroupEnd());
}
// This rank's total of a partial array, in the single-GPU canonical order, into
// its slot of the all-gathered totals.
void dist_total(tpl_op_s* op, const double* P, int N, double* slot) {
  HIPCHK(launch::reorth_reduce(1, P, N, slot, nullptr, op->stream));
}

// Per-step second-pass records of the selective re-orthogonalisation (slot j - 1: step j).
int* reorth_records(const tpl_op_s* op) {
  return reinterpret_cast<int*>(op->d_Pr + ((size_t)op->lay.G2 + 1) * op->kcap + op->lay.G2 + 1);
}

// ---- reorthogonalisation (extension, not in the reference): classical Gram-Schmidt of
// r_{j+1} against the stored columns V[:, 0..j) before beta_j. mode 1 (CGS2): two
// passes, always. mode 2 (selective, Kahan–Parlett "twice is enough"): the second pass
// runs only when the first removed more than half of ||r||^2 (k_reorth_decide; its
// kernels see the device flag and return at once otherwise).
void enqueue_reorth(tpl_op_s* op, int j, int mode) {
  if (op->dist) fail(TPL_ERR_UNSUPPORTED, "re-orthogonalisation of a partitioned operator");
  const int cols = j; // v_1 .. v_j are stored in V[:, 0..j)
  const int G2 = op->lay.G2;
  const int64_t E = op->lay.E;
  double* P = op->d_Pr;                             // cols x G2 partials
  double* h = op->d_Pr + (size_t)G2 * op->kcap;    // cols coefficients
  double* Pb1 = h + op->kcap;                      // ||r'||^2 partials (selective)
  int* skip = reinterpret_cast<int*>(Pb1 + G2);
  int* rec = reorth_records(op) + (j - 1);
  double* r = op->R[(j + 1) % 3];
  for (int pass = 0; pass < 2; ++pass) {
    const int* sk = (mode == 2 && pass == 1) ? skip : nullptr;
    HIPCHK(launch::reorth_dot(op->n, cols, op->d_V, r, P, G2, E, sk, op->stream));
    HIPCHK(launch::reorth_reduce(cols, P, G2, h, sk, op->stream));
    // the last update rewrites the ||r||^2 partials that k_p1_spmv(j+1) reduces; in the
    // selective mode the first one writes its own partials for the decision
    double* pn = pass == 1 ? op->S.Pb : (mode == 2 ? Pb1 : nullptr);
    HIPCHK(launch::reorth_update(op->n, cols, op->d_V, r, h, pn, G2, E, sk, op->stream));
    if (mode == 2 && pass == 0)
      HIPCHK(launch::reorth_decide(op->S, Pb1, G2, skip, rec, op->stream));
  }
}

// Pass one prologue: ||b||^2 partials; with a partition, b and the per-rank
// totals are all-gathered (step 1 gathers from b).
void enqueue_p1_prologue(tpl_op_s* op) {
  const CsrDev A = csr_dev(op);
  HIPCHK(launch::p1_init(A, op->S, op->b, op->stream));
  if (op->hybrid) {  // every column this rank gathers is local: only the norm partials move
    if (op->pb_ld > 0) {
      dist_allgather(op, op->d_pball, (size_t)op->pb_ld);
    } else {
      dist_total(op, op->S.Pb, A.G2, const_cast<double*>(op->S.Pb_r) + op->dist->rank);
      dist_allgather(op, const_cast<double*>(op->S.Pb_r), 1);
    }
  } else if (op->dist) {
    const int R = op->dist->nranks;
    dist_total(op, op->S.Pb, A.G2, op->d_rsum + R + op->dist->rank);
    halo_pack(op, op->bG);
    dist_group(op, true);
    dist_allgather(op, op->d_rsum + R, 1);
    gather_vec(op, op->bG);
    dist_group(op, false);
  }
}

// The exchanges of a pass-one step of a partitioned operator: (a) after the SpMV launch
// (the alpha total; with replicated long rows their partials travel with it), (b) after
// the AXPY (the beta total; with row blocks r_{j+1} travels with it).
void enqueue_p1_exchange_a(tpl_op_s* op, const CsrDev& A) {
  if (op->hybrid) {
    // ONE all-gather: each rank's long-row partials and its short-chunk alpha partials
    // travel in one segment (one collective's latency per SpMV); every rank then finishes
    // the long rows itself (replicated), reduces each rank's alpha partials to its total
    // and adds the long rows' alpha once (k_long_epi_p1). No rank-total launch sits
    // between the SpMV and the collective.
    dist_allgather(op, op->d_yall, (size_t)op->y_ld1);
  } else {
    dist_total(op, op->S.Pa, A.NA, op->d_rsum + op->dist->rank);
    dist_allgather(op, op->d_rsum, 1);
  }
}
void enqueue_p1_exchange_b(tpl_op_s* op, const CsrDev& A, int j) {
  if (op->hybrid) {
    if (op->pb_ld > 0) {
      // round 6: every rank's norm partials travel (pb_ld doubles per rank) and the next
      // k_p1_spmv reduces each rank's itself — no rank-total launch between k_p1_axpy and
      // the collective
      dist_allgather(op, op->d_pball, (size_t)op->pb_ld);
    } else {
      // the rank's beta total: its own one-workgroup launch (folding it into k_p1_axpy's
      // last arriver measured slower, round 5: DESIGN.md §6.3)
      dist_total(op, op->S.Pb, A.G2, const_cast<double*>(op->S.Pb_r) + op->dist->rank);
      dist_allgather(op, const_cast<double*>(op->S.Pb_r), 1);
    }
  } else {
    const int R = op->dist->nranks;
    dist_total(op, op->S.Pb, A.G2, op->d_rsum + R + op->dist->rank);
    halo_pack(op, op->RG[(j + 1) % 3]);
    dist_group(op, true);
    dist_allgather(op, op->d_rsum + R, 1);
    gather_vec(op, op->RG[(j + 1) % 3]);
    dist_group(op, false);
  }
}
// The exchange after pass-two step j's SpMV launch.
void enqueue_p2_exchange(tpl_op_s* op, int j) {
  if (op->hybrid) {
    const size_t nl = op->lay.lrows.size();
    if (nl) dist_allgather(op, op->d_yall, nl + 1);
  } else {
    halo_pack(op, op->V2G[(j + 1) % 3]);
    gather_vec(op, op->V2G[(j + 1) % 3]);
  }
}

// Pass one, step j (k = requested steps). elim: also eliminate row j - 3 of T_k's LU
// (the one-graph inv, k_p1_axpy).
// st1 / st2: start stamps of the step's k_p1_spmv / k_p1_axpy launch (live timing), or nullptr.
void enqueue_p1_step(tpl_op_s* op, int j, int k, double* Vcol, bool elim = false,
                     unsigned long long* st1 = nullptr, unsigned long long* st2 = nullptr) {
  const CsrDev A = csr_dev(op, true);
  HIPCHK(launch::p1_spmv(A, op->S, rG_of(op, j), r_of(op, j), j >= 2 ? r_of(op, j - 1) : nullptr,
                         op->W, Vcol, j, op->stream, st1));
  if (op->dist) enqueue_p1_exchange_a(op, A);
  if (op->hybrid)
    HIPCHK(launch::long_epi_p1(A, op->S, op->d_yall, op->dist->nranks, r_of(op, j),
                               j >= 2 ? r_of(op, j - 1) : nullptr, op->W, Vcol,
                               op->d_rsum + op->dist->nranks, j, op->stream));
  HIPCHK(launch::p1_axpy(A, op->S, op->W, r_of(op, j), op->R[(j + 1) % 3], j, k,
                         elim ? 1 : 0, op->stream, st2));
  if (op->dist && j < k) enqueue_p1_exchange_b(op, A, j);
}

// First stamped step of a k-step pass one (steps js .. js + kStampSteps - 1, and the
// k_p1_spmv of the step after), or 0: the pass is too short to sample.
int stamp_first(size_t k) {
  return k >= (size_t)kStampSteps + 3 ? (int)(k - kStampSteps) / 2 + 1 : 0;
}

void enqueue_pass1(tpl_op_s* op, size_t k, bool storeV, int reorth, bool elim = false,
                   bool stamped = false) {
  enqueue_p1_prologue(op);
  const int js = stamped ? stamp_first(k) : 0;
  for (int j = 1; j <= (int)k; ++j) {
    double* Vcol = storeV ? op->d_V + (size_t)(j - 1) * op->n : nullptr;
    const int i = j - js;  // stamp slots: spmv of step js + i at 2i, its axpy at 2i + 1
    unsigned long long* st1 = js && i >= 0 && i <= kStampSteps ? op->d_stamps + 2 * i : nullptr;
    unsigned long long* st2 = js && i >= 0 && i < kStampSteps ? op->d_stamps + 2 * i + 1 : nullptr;
    enqueue_p1_step(op, j, (int)k, Vcol, elim, st1, st2);
    if (reorth && j < (int)k) enqueue_reorth(op, j, reorth);
  }
}

void enqueue_pass2_init(tpl_op_s* op, size_t steps, double* Vout) {
  HIPCHK(launch::p2_init(op->n, op->S, op->b, op->V2[1], op->x, Vout, 0, op->stream));
  HIPCHK(launch::p2_coefs(op->S, (int)steps, 0, op->stream));
  if (op->dist && !op->hybrid) {
    halo_pack(op, op->V2G[1]);
    gather_vec(op, op->V2G[1]);
  }
}
void enqueue_pass2_steps(tpl_op_s* op, size_t steps, double* Vout) {
  const CsrDev A = csr_dev(op);
  for (int j = 1; j < (int)steps; ++j) {
    double* Vcol = Vout ? Vout + (size_t)j * op->n : nullptr;
    const int nflush = p2_flush(j, (int)steps - 1);
    HIPCHK(launch::p2_spmv(A, op->S, op->V2G[j % 3], op->V2[j % 3],
                           j >= 2 ? op->V2[(j - 1) % 3] : nullptr, op->V2[(j + 1) % 3], op->x,
                           Vcol, j, nflush, op->stream));
    if (op->hybrid) {
      enqueue_p2_exchange(op, j);
      HIPCHK(launch::long_epi_p2(A, op->S, op->d_yall, op->dist->nranks, op->V2[j % 3],
                                 j >= 2 ? op->V2[(j - 1) % 3] : nullptr, op->V2[(j + 1) % 3],
                                 op->x, Vcol, j, nflush, op->stream));
    } else if (op->dist && j + 1 < (int)steps) {
      enqueue_p2_exchange(op, j);
    }
  }
}
void enqueue_pass2(tpl_op_s* op, size_t steps, double* Vout) {
  enqueue_pass2_init(op, steps, Vout);
  enqueue_pass2_steps(op, steps, Vout);
}

// ---- one-graph two-pass solve (built-in f = inv, single GPU): steps_taken stays on the
// device. Pass one as usual; k_ftk_inv forms y = ||b|| T^{-1} e_1 from the device alpha /
// beta (bitwise the host solver's result); pass two is the k - 1 step launches, those at
// or past steps_taken doing nothing, with x flushed at multiples of 3 only and the
// pending terms of the last step added by k_p2_tail (the same sums as the host schedule).
// y = f(T_k) e_1 from the device alpha / beta, times ||b|| (scale: the two-pass y_k) or not
// (the one-pass y').
void enqueue_ftk_only(tpl_op_s* op, size_t k, int f, int scale) {
  if (f == kDevExp)
    HIPCHK(launch::ftk_exp(op->S, (int)k, scale, op->stream));
  else
    HIPCHK(launch::ftk_inv(op->S, (int)k, scale, op->stream));
}
void enqueue_ftk_dev(tpl_op_s* op, size_t k, int f) {
  enqueue_ftk_only(op, k, f, 1);
  HIPCHK(launch::p2_init(op->n, op->S, op->b, op->V2[1], op->x, nullptr, 1, op->stream));
  HIPCHK(launch::p2_coefs(op->S, (int)k, 1, op->stream));
}
void enqueue_pass2_dyn_steps(tpl_op_s* op, size_t k) {
  const CsrDev A = csr_dev(op);
  for (int j = 1; j < (int)k; ++j)
    HIPCHK(launch::p2_spmv(A, op->S, op->V2G[j % 3], op->V2[j % 3],
                           j >= 2 ? op->V2[(j - 1) % 3] : nullptr, op->V2[(j + 1) % 3], op->x,
                           nullptr, j, j % 3 == 0 ? 3 : 0, op->stream));
}
void enqueue_pass2_tail(tpl_op_s* op) {
  HIPCHK(launch::p2_tail(op->n, op->S, op->x, op->V2, op->stream));
}

template <class Enq>
void run_graph(tpl_op_s* op, int kind, size_t key, Enq&& enqueue) {
  if (!use_graphs() || op->eager) {
    enqueue();
    return;
  }
  auto it = op->graphs.find({kind, key});
  if (it == op->graphs.end()) {
    HIPCHK(hipStreamBeginCapture(op->stream, hipStreamCaptureModeThreadLocal));
    try {
      enqueue();
    } catch (...) {
      hipGraph_t g = nullptr;
      hipStreamEndCapture(op->stream, &g);
      if (g) hipGraphDestroy(g);
      if (!op->dist) throw;
      op->eager = true;  // the transport refused capture: launch eagerly from now on
      hipGetLastError();
      enqueue();
      return;
    }
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(op->stream, &g);
    hipGraphExec_t ge = nullptr;
    if (e == hipSuccess) e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (g) hipGraphDestroy(g);
    if (e != hipSuccess && op->dist) {
      op->eager = true;
      hipGetLastError();
      enqueue();
      return;
    }
    HIPCHK(e);
    it = op->graphs.emplace(std::make_pair(kind, key), ge).first;
  }
  HIPCHK(hipGraphLaunch(it->second, op->stream));
}

// Pass two without a basis. With live timing on, the prologue is launched on its own
// and events bracket the graph of the steps - 1 step launches (tpl_op_pass_timing).
void run_pass2(tpl_op_s* op, size_t steps) {
  if (!op->timing) {
    run_graph(op, kGPass2, steps, [&] { enqueue_pass2(op, steps, nullptr); });
    return;
  }
  enqueue_pass2_init(op, steps, nullptr);
  HIPCHK(hipEventRecord(op->tev[2], op->stream));
  run_graph(op, kGPass2Steps, steps, [&] { enqueue_pass2_steps(op, steps, nullptr); });
  HIPCHK(hipEventRecord(op->tev[3], op->stream));
  op->p2_launches = (int64_t)steps - 1;
}

struct HostDecomp {
  int32_t flags[kFlagBytes / 4];
  double b_norm;
  const double* alphas;
  const double* betas;
  size_t steps;
};

// Copy flags | norms[0] | alphas | betas back (one D2H), synchronise.
void sync_checked(tpl_op_s* op) { HIPCHK(hipStreamSynchronize(op->stream)); }

HostDecomp fetch_decomp(tpl_op_s* op, size_t k) {
  const size_t kc = op->kcap;
  char* h = (char*)op->h_state;
  const size_t bytes = kFlagBytes + ((kc + 1) + 2 * kc) * sizeof(double);
  (void)k;
  HIPCHK(hipMemcpyAsync(h, op->d_state, bytes, hipMemcpyDeviceToHost, op->stream));
  sync_checked(op);
  HostDecomp d;
  std::memcpy(d.flags, h, kFlagBytes);
  const double* norms = (const double*)(h + kFlagBytes);
  d.b_norm = norms[0];
  d.alphas = norms + (kc + 1);
  d.betas = d.alphas + kc;
  d.steps = (size_t)d.flags[2];
  return d;
}

// The whole two-pass solve as one graph (or, with live timing on, as several graphs with
// the events between them); no host round trip between the passes.
void run_two_pass_dev(tpl_op_s* op, size_t k, int f) {
  const size_t key = 2 * k + (size_t)f;  // one graph per (k, f)
  const bool elim = f == kDevInv;  // T_k's LU eliminated during pass one
  if (!op->timing) {
    op->p1_samples = 0;  // the untimed graph records no launch stamps
    run_graph(op, kGTwoPassDev, key, [&] {
      enqueue_pass1(op, k, false, false, elim);
      enqueue_ftk_dev(op, k, f);
      enqueue_pass2_dyn_steps(op, k);
      enqueue_pass2_tail(op);
    });
    return;
  }
  HIPCHK(hipEventRecord(op->tev[0], op->stream));
  const bool stamped = !op->dist && stamp_first(k) > 0;
  if (stamped && !op->d_stamps) {
    dev_alloc(op, &op->d_stamps, 32 * sizeof(unsigned long long));
    HIPCHK(hipMemset(op->d_stamps, 0, 32 * sizeof(unsigned long long)));
  }
  run_graph(op, stamped ? (elim ? kGPass1ElimStamped : kGPass1Stamped) : (elim ? kGPass1Elim : kGPass1),
            k, [&] { enqueue_pass1(op, k, false, false, elim, stamped); });
  op->p1_samples = stamped ? kStampSteps : 0;
  HIPCHK(hipEventRecord(op->tev[1], op->stream));
  run_graph(op, kGDevFtk, key, [&] { enqueue_ftk_dev(op, k, f); });
  HIPCHK(hipEventRecord(op->tev[2], op->stream));
  run_graph(op, kGPass2Dyn, k, [&] { enqueue_pass2_dyn_steps(op, k); });
  HIPCHK(hipEventRecord(op->tev[3], op->stream));
  enqueue_pass2_tail(op);
  op->p2_launches = (int64_t)k - 1;
}

// elim: eliminate T_k's LU during the pass (a device inv follows: k_ftk_inv)
void run_pass_one(tpl_op_s* op, const double* b, size_t k, int mem, bool storeV, int reorth,
                  bool elim = false) {
  ensure_state(op, k, reorth);
  if (storeV) ensure_basis(op, k);
  upload_vec(op, op->b, b, mem);
  op->p1_samples = 0;  // no pass run here records launch stamps (tpl_op_step_samples)
  if (reorth) {
    enqueue_pass1(op, k, true, reorth); // eager: reorth launch counts vary with j
  } else {
    if (op->timing) HIPCHK(hipEventRecord(op->tev[0], op->stream));
    const int kind = storeV ? (elim ? kGStandardElim : kGStandard) : (elim ? kGPass1Elim : kGPass1);
    run_graph(op, kind, k, [&] { enqueue_pass1(op, k, storeV, false, elim); });
    if (op->timing) HIPCHK(hipEventRecord(op->tev[1], op->stream));
  }
}

void check_k(size_t k) {
  // The reference panics at k = 0 (Vec::with_capacity(k - 1) underflow,
  // src/algorithms/lanczos.rs:75); the C ABI reports it instead.
  if (k == 0) fail_input("The number of iterations `k` must be at least 1.");
  if (k > (size_t)INT32_MAX / 2) fail(TPL_ERR_INVALID_ARGUMENT, "k too large");
}

void call_ftk(tpl_ftk_fn f, void* user, const HostDecomp& d, std::vector<double>& y) {
  if (!f) fail(TPL_ERR_INVALID_ARGUMENT, "f_tk_solver is NULL");
  y.assign(d.steps, 0.0);
  size_t ylen = d.steps;
  char err[1024];
  err[0] = '\0';
  const int rc = f(d.alphas, d.steps, d.betas, d.steps > 0 ? d.steps - 1 : 0, y.data(), d.steps,
                   &ylen, err, sizeof(err), user);
  err[sizeof(err) - 1] = '\0';
  if (rc != 0) fail_solver(err);
  if (ylen != d.steps)
    fail_param_mismatch("y_k_prime", d.steps, ylen);
}

void zero_out(tpl_op_s* op, double* x_out, int mem) {
  if (op->n == 0) return;
  if (mem == TPL_MEM_DEVICE) {
    HIPCHK(hipMemsetAsync(x_out, 0, op->n * sizeof(double), op->stream));
    sync_checked(op);
  } else {
    std::memset(x_out, 0, op->n * sizeof(double));
  }
}

// Layout, vectors and events of a freshly filled operator (single GPU or one rank
// of a partition; the vector stride ld is common to all ranks).
// Vector stride ld, common to all ranks (the gathered vector holds rank r's block at r * ld).
void set_stride(tpl_op_s* op) {
  if (op->halo) {  // [own block | nranks x hH halo slots]; fill_halo sized and checked it
    op->ld = ((std::max<int64_t>(op->n, 1) + 63) / 64) * 64;
    return;
  }
  const int R = op->dist && !op->hybrid ? op->dist->nranks : 1;  // gathered vector copies
  int64_t widest = op->n;
  if (op->dist && !op->hybrid)
    for (int r = 0; r < R; ++r) widest = std::max(widest, op->starts[r + 1] - op->starts[r]);
  op->ld = ((std::max<int64_t>(widest, 1) + 63) / 64) * 64;
  // gathered column indices (ColMap: r * ld + local) are int32 on the device
  if ((int64_t)R * op->ld >= (int64_t)INT32_MAX)
    fail(TPL_ERR_UNSUPPORTED, "row blocks too unbalanced: nranks x widest block >= 2^31");
}

void init_op(tpl_op_s* op) {
  const int R = op->dist && !op->hybrid ? op->dist->nranks : 1;  // gathered vector copies
  set_stride(op);
  rebuild_schedule(op);
  // gathered: b, R0..2, V2_0..2, tmp (R x ld each; halo: ld + R x hH); local: W, x (ld each)
  const size_t gl = op->halo ? (size_t)op->ld + (size_t)R * op->hH : (size_t)R * op->ld;
  const size_t gathered = 8 * gl, local = 2 * (size_t)op->ld;
  dev_alloc(op, &op->d_vecs, (gathered + local) * sizeof(double));
  HIPCHK(hipMemset(op->d_vecs, 0, (gathered + local) * sizeof(double)));
  double* p = op->d_vecs;
  const size_t own = (size_t)(op->dist && !op->hybrid && !op->halo ? op->dist->rank : 0) * op->ld;
  upload(op, &op->d_halo_send, op->halo_send);
  op->bG = p;
  p += gl;
  for (int i = 0; i < 3; ++i, p += gl) op->RG[i] = p;
  for (int i = 0; i < 3; ++i, p += gl) op->V2G[i] = p;
  op->tmpG = p;
  p += gl;
  op->W = p;
  p += op->ld;
  op->x = p;
  op->b = op->bG + own;
  for (int i = 0; i < 3; ++i) op->R[i] = op->RG[i] + own;
  for (int i = 0; i < 3; ++i) op->V2[i] = op->V2G[i] + own;
  op->tmp = op->tmpG + own;
  if (op->dist) {
    // [nranks alpha totals | long-row alpha partials (hybrid) | nranks norm totals]
    const size_t nr = (size_t)op->dist->nranks;
    const size_t cnt = 2 * nr + (op->hybrid ? (size_t)long_epi_blocks(op) : 0);
    dev_alloc(op, &op->d_rsum, cnt * sizeof(double));
    HIPCHK(hipMemset(op->d_rsum, 0, cnt * sizeof(double)));
    if (op->hybrid) {
      // every rank's chunk count (each rank's short rows are a contiguous block of the
      // global split, chunked by kChunkRows: every rank computes all counts alike)
      if ((int)op->nch.size() != op->dist->nranks ||
          op->nch[op->dist->rank] != (int32_t)op->lay.c_base.size())
        fail(TPL_ERR_UNSUPPORTED, "replicated partition: chunk counts disagree with the layout");
      const int32_t nmax = *std::max_element(op->nch.begin(), op->nch.end());
      op->y_ld1 = (int32_t)op->lay.lrows.size() + nmax;
      upload(op, &op->d_nch, op->nch);
      // pass one strides the all-gather by y_ld1, pass two and tpl_op_apply by n_long + 1
      const size_t ya = nr * (size_t)std::max<int64_t>(op->y_ld1, (int64_t)op->lay.lrows.size() + 1);
      dev_alloc(op, &op->d_yall, ya * sizeof(double));
      HIPCHK(hipMemset(op->d_yall, 0, ya * sizeof(double)));
      // the β stage all-gathers every rank's norm partials (each rank computes all ranks'
      // counts from the global split) and k_p1_spmv reduces each rank's with the tree the
      // rank-total launch applied — one launch less per pass-one step, the same bits —
      // while they fit one load per lane and rank (≤ kPbRanks ranks, ≤ kTPB partials)
      if ((int)op->g2s.size() != op->dist->nranks ||
          op->g2s[op->dist->rank] != op->lay.G2)
        fail(TPL_ERR_UNSUPPORTED, "replicated partition: block counts disagree with the layout");
      const int32_t g2max = *std::max_element(op->g2s.begin(), op->g2s.end());
      if (op->dist->nranks <= kPbRanks && g2max <= kTPB) {
        op->pb_ld = g2max;
        dev_alloc(op, &op->d_pball, nr * (size_t)g2max * sizeof(double));
        HIPCHK(hipMemset(op->d_pball, 0, nr * (size_t)g2max * sizeof(double)));
      }
    }
  }
  HIPCHK(hipEventCreate(&op->ev0));
  HIPCHK(hipEventCreate(&op->ev1));
  for (hipEvent_t& e : op->tev) HIPCHK(hipEventCreate(&e));
}

// Contiguous blocks over items 0..m-1 with cost prefix[m+1]: cut where the prefix
// crosses r/nranks of the total; every block keeps at least one item.
void balanced_cuts(const std::vector<double>& prefix, int nranks, int64_t* starts) {
  const int64_t m = (int64_t)prefix.size() - 1;
  const double total = prefix[m];
  starts[0] = 0;
  int64_t i = 0;
  for (int r = 1; r < nranks; ++r) {
    const double target = total * r / nranks;
    while (i < m && prefix[i] < target) ++i;
    starts[r] = std::min<int64_t>(std::max<int64_t>(i, starts[r - 1] + 1), m - (nranks - r));
    i = starts[r];
  }
  starts[nranks] = m;
}

// Host half of tpl_dist_op_create_replicated (and of its tpl_plan_create): the short-row
// split, this rank's rows in their order and its local CSR. op->n .. op->nch.
void fill_replicated(tpl_op_s* op, int R, int me, int64_t n, const int64_t* row_ptr,
                     const int32_t* col_idx, const double* vals) {
  const int64_t nnz = row_ptr[n];
  if (n < 1 || n >= INT32_MAX / 2 || nnz >= INT32_MAX || row_ptr[0] != 0)
    fail(TPL_ERR_INVALID_ARGUMENT, "bad CSR sizes");
  if (nnz > 0 && !vals) fail(TPL_ERR_INVALID_ARGUMENT, "col_idx/vals is NULL");
  check_csr(n, n, row_ptr, col_idx);
  std::vector<int32_t> rp32(n + 1);
  for (int64_t i = 0; i <= n; ++i) rp32[i] = (int32_t)row_ptr[i];
  // short / long rows by the global rule; long rows are replicated on every rank
  const int32_t T = short_row_threshold(n, rp32, -1);
  std::vector<int64_t> S, Lr;
  std::vector<int32_t> lidx(n, -1);
  for (int64_t i = 0; i < n; ++i) {
    if (rp32[i + 1] - rp32[i] > T) {
      lidx[i] = (int32_t)Lr.size();
      Lr.push_back(i);
    } else {
      S.push_back(i);
    }
  }
  if ((int64_t)S.size() < R) fail(TPL_ERR_UNSUPPORTED, "fewer short rows than ranks");
  // short rows in contiguous blocks balanced by bytes: the row itself plus the
  // long-row entries in its column, which the owner of that column computes
  std::vector<int32_t> longcnt(n, 0);
  for (int64_t l : Lr)
    for (int64_t q = row_ptr[l]; q < row_ptr[l + 1]; ++q) longcnt[col_idx[q]]++;
  std::vector<double> prefix(S.size() + 1, 0.0);
  for (size_t p = 0; p < S.size(); ++p) {
    const int64_t i = S[p];
    prefix[p + 1] = prefix[p] + 12.0 * (double)(rp32[i + 1] - rp32[i] + longcnt[i]) + 40.0;
  }
  std::vector<int64_t> cut(R + 1);
  balanced_cuts(prefix, R, cut.data());
  std::vector<int32_t> owner(n, -1);
  for (int r = 0; r < R; ++r)
    for (int64_t p = cut[r]; p < cut[r + 1]; ++p) owner[S[p]] = r;
  // halo-free check (all ranks decide alike: they all see the whole matrix)
  for (int64_t i : S)
    for (int64_t q = row_ptr[i]; q < row_ptr[i + 1]; ++q) {
      const int32_t c = col_idx[q];
      if (lidx[c] < 0 && owner[c] != owner[i])
        fail(TPL_ERR_UNSUPPORTED, "a short row references a short row of another rank "
                                  "(use the row-partitioned operator)");
    }
  op->hybrid = true;
  op->n_glob = n;
  const int64_t ns = cut[me + 1] - cut[me], nl = (int64_t)Lr.size();
  op->ns_local = ns;
  op->n = ns + nl;
  // this rank's short rows; in the locality order (tpl_layout.h locality_order, the
  // same key over the replicated long rows' ranks) when the rank's rows fit the auto
  // rule. The local order is the caller's to follow through tpl_op_local_rows, so no
  // vector is permuted on the device.
  std::vector<int64_t> mine(S.begin() + cut[me], S.begin() + cut[me + 1]);
  if (nl > 0 && op->n <= kReorderAutoMaxRows) {
    // lidx is each long row's rank among the long rows, as locality_order ranks them
    locality_sort(mine, row_ptr, col_idx, lidx.data(), (int32_t)nl, op->sp.order_groups);
    op->local_order = true;
  }
  op->g2l.assign(n, -1);
  op->local_rows.resize(op->n);
  for (int64_t p = 0; p < ns; ++p) {
    op->g2l[mine[p]] = (int32_t)p;
    op->local_rows[p] = mine[p];
  }
  for (int64_t l = 0; l < nl; ++l) {
    op->g2l[Lr[l]] = (int32_t)(ns + l);
    op->local_rows[ns + l] = Lr[l];
  }
  // local CSR in local column indices, each row ascending: own short rows whole; long
  // rows restricted to the columns this rank owns (long-row columns: rank 0). The
  // long rows' 8 column slices then split this rank's own columns, so every XCD
  // gets a share of the long-row work.
  op->h_rowptr.assign(1, 0);
  std::vector<std::pair<int32_t, double>> row;
  for (int64_t p = 0; p < op->n; ++p) {
    const int64_t i = op->local_rows[p];
    const bool is_long = p >= ns;
    row.clear();
    for (int64_t q = row_ptr[i]; q < row_ptr[i + 1]; ++q) {
      const int32_t c = col_idx[q];
      if (is_long && !(lidx[c] < 0 ? owner[c] == me : me == 0)) continue;
      row.emplace_back(op->g2l[c], vals[q]);
    }
    std::sort(row.begin(), row.end(),
              [](const std::pair<int32_t, double>& a, const std::pair<int32_t, double>& b) {
                return a.first < b.first;
              });
    for (const auto& e : row) {
      op->h_col.push_back(e.first);
      op->h_val.push_back(e.second);
    }
    op->h_rowptr.push_back((int32_t)op->h_col.size());
  }
  op->nnz = (int64_t)op->h_col.size();
  op->sp.long_from = ns;
  op->nch.resize(R);
  op->g2s.resize(R);
  for (int r = 0; r < R; ++r) {
    op->nch[r] = (int32_t)((cut[r + 1] - cut[r] + kChunkRows - 1) / kChunkRows);
    int64_t E = 0;
    elem_geometry(cut[r + 1] - cut[r] + nl, op->sp, op->g2s[r], E);
  }
  // Up to kPbRanks ranks: element-wise blocks wide enough that no rank holds more than kTPB
  // norm partials, so pass one's SpMV reduces every rank's gathered partials itself (one
  // load per lane and rank) and no rank-total launch remains — when that needs at most
  // 2 kElemRows rows per block. Measured on the 5M-arc instance (round 6, rank shares
  // through one RCCL rank, profiles/r06_rank_share_5m_wide.txt): N = 8, 306 -> 246
  // partials at 2,560 rows per block, slowest share 14.35 -> 13.78 ms; N = 4, 5,120 rows
  // per block, 20.69 -> 21.29 ms (k_p1_axpy's wider blocks cost more than the launch), so
  // not applied there. Every rank applies the same rule to the same split, so all agree
  // on every rank's count.
  int64_t rows_max = 0;
  for (int r = 0; r < R; ++r) rows_max = std::max<int64_t>(rows_max, cut[r + 1] - cut[r] + nl);
  const int64_t er_gp = (((rows_max + kTPB - 1) / kTPB) + 511) / 512 * 512;
  if (R <= kPbRanks && op->sp.elem_rows <= 0 && er_gp <= 2 * kElemRows &&
      *std::max_element(op->g2s.begin(), op->g2s.end()) > kTPB) {
    op->sp.elem_rows = (int)er_gp;
    for (int r = 0; r < R; ++r) {
      int64_t E = 0;
      elem_geometry(cut[r + 1] - cut[r] + nl, op->sp, op->g2s[r], E);
    }
  }
}

// Host half of a row-block rank from the WHOLE matrix (TPL_PLAN_ROWS, TPL_PLAN_HALO,
// tpl_dist_op_create_halo): block `me` of `starts` (nullptr: the tpl_dist_partition
// split), its rows with global column indices. halo: also the halo plan — B_q = the rows
// of rank q's block that a row of another rank references (one pass over the nonzeros),
// hH = max_q |B_q|, this rank's send list (B_me in local indices) and the column table:
// own column c -> c - starts[me], remote column c in B_q -> ld + q hH + (c's rank in B_q).
// The layout is built from the same CSR and global-column slices as plain row blocks, so
// the two hold the same reduction order; only the gathered positions differ.
void fill_rows(tpl_op_s* op, int R, int me, int64_t n, const int64_t* starts,
               const int64_t* row_ptr, const int32_t* col_idx, const double* vals, bool halo) {
  if (n < R) fail(TPL_ERR_INVALID_ARGUMENT, "fewer rows than ranks");
  if (n >= INT32_MAX / 2) fail(TPL_ERR_UNSUPPORTED, "n must be < 2^30");
  if (row_ptr[0] != 0) fail(TPL_ERR_INVALID_ARGUMENT, "row_ptr must start at 0");
  if (row_ptr[n] > 0 && (!vals || !col_idx)) fail(TPL_ERR_INVALID_ARGUMENT, "col_idx/vals is NULL");
  check_csr(n, n, row_ptr, col_idx);
  op->starts.resize(R + 1);
  if (starts) {
    if (starts[0] != 0 || starts[R] != n) fail(TPL_ERR_INVALID_ARGUMENT, "bad partition");
    for (int r = 0; r < R; ++r)
      if (starts[r + 1] <= starts[r]) fail(TPL_ERR_INVALID_ARGUMENT, "empty or unordered block");
    op->starts.assign(starts, starts + R + 1);
  } else {
    std::vector<double> prefix(n + 1);
    for (int64_t i = 0; i <= n; ++i) prefix[i] = 12.0 * (double)row_ptr[i] + 40.0 * (double)i;
    balanced_cuts(prefix, R, op->starts.data());
  }
  const int64_t r0 = op->starts[me], r1 = op->starts[me + 1];
  op->n = r1 - r0;
  op->n_glob = n;
  op->nnz = row_ptr[r1] - row_ptr[r0];
  if (op->nnz >= INT32_MAX) fail(TPL_ERR_UNSUPPORTED, "nnz must be < 2^31");
  op->h_rowptr.resize(op->n + 1);
  for (int64_t i = 0; i <= op->n; ++i) op->h_rowptr[i] = (int32_t)(row_ptr[r0 + i] - row_ptr[r0]);
  op->h_col.assign(col_idx + row_ptr[r0], col_idx + row_ptr[r1]);
  op->h_val.assign(vals + row_ptr[r0], vals + row_ptr[r1]);
  if (!halo) return;
  const std::vector<int64_t>& st = op->starts;
  std::vector<uint8_t> need(n, 0);
  for (int r = 0; r < R; ++r)
    for (int64_t q = row_ptr[st[r]]; q < row_ptr[st[r + 1]]; ++q) {
      const int32_t c = col_idx[q];
      if (c < st[r] || c >= st[r + 1]) need[c] = 1;
    }
  std::vector<int32_t> pos(n, -1);
  int64_t H = 0;
  for (int q = 0; q < R; ++q) {
    int32_t m = 0;
    for (int64_t c = st[q]; c < st[q + 1]; ++c)
      if (need[c]) pos[c] = m++;
    H = std::max<int64_t>(H, m);
  }
  op->halo = true;
  op->hH = H;
  const int64_t ld = ((std::max<int64_t>(op->n, 1) + 63) / 64) * 64;  // set_stride's
  if (ld + (int64_t)R * H >= (int64_t)INT32_MAX)
    fail(TPL_ERR_UNSUPPORTED, "halo partition: own block + nranks x halo width >= 2^31");
  op->halo_send.clear();
  for (int64_t c = r0; c < r1; ++c)
    if (need[c]) op->halo_send.push_back((int32_t)(c - r0));
  op->halo_map.assign(n, -1);
  for (int64_t c = r0; c < r1; ++c) op->halo_map[c] = (int32_t)(c - r0);
  for (int q = 0; q < R; ++q)
    if (q != me)
      for (int64_t c = st[q]; c < st[q + 1]; ++c)
        if (pos[c] >= 0) op->halo_map[c] = (int32_t)(ld + (int64_t)q * H + pos[c]);
}

// The partition every binding's "auto" takes (tpl_dist_choose_partition): replicated long
// rows when the matrix allows them, else halo row blocks when the halo is at most half the
// widest block, else plain row blocks. Host only; the same answer on every rank.
int choose_partition(int64_t n, const int64_t* row_ptr, const int32_t* col_idx, int R) {
  if (!row_ptr || R < 1) fail(TPL_ERR_INVALID_ARGUMENT, "bad argument");
  {
    tpl_op_s tmp;
    tpl_dist_s pd;
    pd.nranks = R;
    tmp.dist = &pd;
    // the split's feasibility does not depend on the rank; the values are not read for it
    std::vector<double> ones(std::max<int64_t>(row_ptr[n], 1), 1.0);
    try {
      fill_replicated(&tmp, R, 0, n, row_ptr, col_idx, ones.data());
      tmp.dist = nullptr;
      return TPL_PLAN_REPLICATED;
    } catch (const Error& e) {
      tmp.dist = nullptr;
      if (e.code != TPL_ERR_UNSUPPORTED) throw;
    }
  }
  tpl_op_s tmp;
  tpl_dist_s pd;
  pd.nranks = R;
  tmp.dist = &pd;
  std::vector<double> ones(std::max<int64_t>(row_ptr[n], 1), 1.0);
  fill_rows(&tmp, R, 0, n, nullptr, row_ptr, col_idx, ones.data(), true);
  tmp.dist = nullptr;
  int64_t widest = 0;
  for (int r = 0; r < R; ++r) widest = std::max<int64_t>(widest, tmp.starts[r + 1] - tmp.starts[r]);
  return 2 * tmp.hH <= widest ? TPL_PLAN_HALO : TPL_PLAN_ROWS;
}

} // namespace

// =========================================================== C ABI
extern "C" {

const char* tpl_version(void) { return "tpl_amd 0.1.0 gfx950"; }

int tpl_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

tpl_status tpl_ctx_create(int device, tpl_ctx_t* out) {
  return guarded([&] {
    if (!out) fail(TPL_ERR_INVALID_ARGUMENT, "out is NULL");
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0)
      fail(TPL_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= cnt) fail(TPL_ERR_INVALID_ARGUMENT, "device index out of range");
    HIPCHK(hipSetDevice(device));
    auto c = std::make_unique<tpl_ctx_s>();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    *out = c.release();
  });
}

tpl_status tpl_ctx_destroy(tpl_ctx_t ctx) {
  return guarded([&] {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
  });
}

tpl_status tpl_ctx_synchronize(tpl_ctx_t ctx) {
  return guarded([&] {
    if (!ctx) fail(TPL_ERR_INVALID_ARGUMENT, "ctx is NULL");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  });
}

tpl_status tpl_op_create_csr(tpl_ctx_t ctx, int64_t n, int64_t nnz, const int64_t* row_ptr,
                             const int32_t* col_idx, const double* vals, tpl_op_t* out) {
  return guarded([&] {
    if (!ctx || !out) fail(TPL_ERR_INVALID_ARGUMENT, "ctx/out is NULL");
    if (n < 0 || nnz < 0) fail(TPL_ERR_INVALID_ARGUMENT, "negative size");
    if (n >= INT32_MAX || nnz >= INT32_MAX)
      fail(TPL_ERR_UNSUPPORTED, "n and nnz must be < 2^31 (int32 device offsets)");
    if (!row_ptr) fail(TPL_ERR_INVALID_ARGUMENT, "row_ptr is NULL");
    if (nnz > 0 && !vals) fail(TPL_ERR_INVALID_ARGUMENT, "col_idx/vals is NULL");
    if (row_ptr[n] != nnz) fail(TPL_ERR_INVALID_ARGUMENT, "row_ptr must start at 0 and end at nnz");
    check_csr(n, n, row_ptr, col_idx);
    HIPCHK(hipSetDevice(ctx->device));
    auto op = std::make_unique<tpl_op_s>();
    op->ctx = ctx;
    op->device = ctx->device;
    op->stream = ctx->stream;
    op->n = n;
    op->n_glob = n;
    op->nnz = nnz;
    op->h_rowptr.resize(n + 1);
    for (int64_t i = 0; i <= n; ++i) op->h_rowptr[i] = (int32_t)row_ptr[i];
    op->h_col.assign(col_idx, col_idx + nnz);
    op->h_val.assign(vals, vals + nnz);
    init_op(op.get());
    *out = op.release();
  });
}

tpl_status tpl_op_destroy(tpl_op_t op) {
  return guarded([&] {
    if (!op) return;
    if (op->plan_only) {  // host vectors only
      delete op;
      return;
    }
    hipSetDevice(op->device);
    hipStreamSynchronize(op->stream);
    drop_graphs(op);
    for (const auto& kv : op->allocs) hipFree(const_cast<void*>(kv.first));  // every dev_alloc
    if (op->h_state) hipHostFree(op->h_state);
    if (op->ev0) hipEventDestroy(op->ev0);
    if (op->ev1) hipEventDestroy(op->ev1);
    for (hipEvent_t e : op->tev)
      if (e) hipEventDestroy(e);
    delete op;
  });
}

int64_t tpl_op_nrows(tpl_op_t op) { return op ? op->n : -1; }
int tpl_op_flags(tpl_op_t op) {
  if (!op) return -1;
  return (op->dist ? 1 : 0) | (op->eager ? 2 : 0) | (op->lay.val_i8 ? 4 : 0) |
         (op->lay.s_col16 ? 8 : 0) | (op->lay.b_col16 ? 16 : 0) | (op->last_one_graph ? 32 : 0) |
         (!op->perm.empty() || op->local_order ? 64 : 0) | (op->pb_ld > 0 ? 128 : 0);
}

tpl_status tpl_op_set_reorder(tpl_op_t op, int mode) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    if (mode < 0 || mode > 2) fail(TPL_ERR_INVALID_ARGUMENT, "reorder mode must be 0, 1 or 2");
    set_device(op);
    sync_checked(op);
    op->reorder = mode;
    rebuild_schedule(op);
  });
}

tpl_status tpl_op_permutation(tpl_op_t op, int32_t* perm) {
  return guarded([&] {
    if (!op || (!perm && op->n > 0)) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    if (op->perm.empty())
      for (int64_t i = 0; i < op->n; ++i) perm[i] = (int32_t)i;
    else
      std::copy(op->perm.begin(), op->perm.end(), perm);
  });
}

tpl_status tpl_op_set_value_format(tpl_op_t op, int compress) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    set_device(op);
    op->sp.compress_values = compress != 0;
    op->sp.compress_cols = compress != 0;
    sync_checked(op);
    rebuild_schedule(op);
  });
}
int64_t tpl_op_nnz(tpl_op_t op) { return op ? op->nnz : -1; }

tpl_status tpl_op_apply(tpl_op_t op, const double* x, double* y, int mem) {
  return guarded([&] {
    if (!op || ((!x || !y) && op->n > 0)) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    set_device(op);
    if (op->n == 0) return;
    upload_vec(op, op->tmp, x, mem);
    if (op->dist && !op->hybrid) {
      halo_pack(op, op->tmpG);
      gather_vec(op, op->tmpG);
    }
    const CsrDev A = csr_dev(op);
    HIPCHK(launch::spmv(A, op->tmpG, op->W, op->stream));
    if (op->hybrid && A.n_long > 0) {
      dist_allgather(op, op->d_yall, (size_t)A.y_ld);
      HIPCHK(launch::long_epi_y(A, op->d_yall, op->dist->nranks, op->W, op->stream));
    }
    download_vec(op, y, op->W, 1, mem);
    sync_checked(op);
  });
}

tpl_status tpl_lanczos_pass_one(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                                double* alphas, double* betas, size_t* steps, double* b_norm,
                                int mem) {
  return guarded([&] {
    if (!op || !alphas || !betas || !steps || !b_norm)
      fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    set_device(op);
    check_b(op, b, b_len);
    check_k(k);
    run_pass_one(op, b, k, mem, false, false);
    const HostDecomp d = fetch_decomp(op, k);
    if (d.flags[1]) fail_input("Input vector `b` must not be a zero vector.");
    std::memcpy(alphas, d.alphas, d.steps * sizeof(double));
    if (d.steps > 1) std::memcpy(betas, d.betas, (d.steps - 1) * sizeof(double));
    *steps = d.steps;
    *b_norm = d.b_norm;
  });
}

tpl_status tpl_lanczos_standard(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                                double* alphas, double* betas, size_t* steps, double* b_norm,
                                double* v_out, int mem, int reorth, tpl_step_cb cb,
                                void* cb_user) {
  return guarded([&] {
    if (!op || !alphas || !betas || !steps || !b_norm)
      fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    set_device(op);
    check_b(op, b, b_len);
    check_k(k);
    HostDecomp d;
    if (!cb) {
      if (reorth < 0 || reorth > 2) fail(TPL_ERR_INVALID_ARGUMENT, "reorth must be 0, 1 or 2");
      run_pass_one(op, b, k, mem, true, reorth);
      d = fetch_decomp(op, k);
    } else {
      // src/algorithms/lanczos.rs:86-128 with the host callback after every step, polled
      // in batches: the device runs a batch of steps ahead (1, 2, 4, ... up to
      // kCbBatchMax steps: at most as many speculative steps as were already confirmed),
      // then the callback sees steps j = first .. last of the batch in order, each with
      // the T_j view of that step (alphas[0..j), betas[0..j-1)) and V's first j columns.
      // A stop at step j truncates the decomposition to j steps: later steps never change
      // earlier alphas, betas or columns, so the result is exactly the one-step-at-a-time
      // result, with one host synchronisation per batch instead of per step.
      ensure_state(op, k, reorth != 0);
      ensure_basis(op, k);
      // the callback's view in the caller's row order: each batch's new columns are
      // gathered into d_Vext (an n x k buffer, reordered operators only)
      double* Vview = op->d_V;
      if (op->d_perm) {
        if (op->vext_cols < k) {
          dev_free(op, op->d_Vext);
          op->vext_cols = 0;
          dev_alloc(op, &op->d_Vext, (size_t)op->n * k * sizeof(double));
          op->vext_cols = k;
        }
        Vview = op->d_Vext;
      }
      upload_vec(op, op->b, b, mem);
      enqueue_p1_prologue(op);
      size_t stop_at = k;
      int batch = 1;
      for (int j0 = 1; j0 <= (int)k;) {
        const int j1 = std::min<int>((int)k, j0 + batch - 1);
        for (int j = j0; j <= j1; ++j) {
          enqueue_p1_step(op, j, (int)k, op->d_V + (size_t)(j - 1) * op->n);
          if (reorth && j < (int)k) enqueue_reorth(op, j, reorth);
        }
        if (Vview != op->d_V)
          HIPCHK(launch::permute(op->n, j1 - j0 + 1, Vview + (size_t)(j0 - 1) * op->n, op->n,
                                 op->d_V + (size_t)(j0 - 1) * op->n, op->n, op->d_iperm,
                                 op->stream));
        d = fetch_decomp(op, k);
        bool go = true;
        for (int j = j0; j <= j1 && go; ++j) {
          if (d.flags[0] && d.steps < (size_t)j) {  // zero b, or breakdown before step j
            stop_at = d.steps;
            go = false;
            break;
          }
          go = cb((size_t)j, Vview, op->n, d.alphas, (size_t)j, d.betas, (size_t)j - 1,
                  cb_user) != 0;
          if (!go) stop_at = (size_t)j;
        }
        if (!go) break;
        j0 = j1 + 1;
        batch = std::min(2 * batch, kCbBatchMax);
      }
      d = fetch_decomp(op, k);
      d.steps = std::min(d.steps, stop_at);
    }
    if (d.flags[1]) fail_input("Input vector `b` must not be a zero vector.");
    std::memcpy(alphas, d.alphas, d.steps * sizeof(double));
    if (d.steps > 1) std::memcpy(betas, d.betas, (d.steps - 1) * sizeof(double));
    *steps = d.steps;
    *b_norm = d.b_norm;
    // second passes of the steps the caller keeps: a step callback may stop before the
    // device's last step (batched polling runs ahead), so count the kept steps' records
    op->reorth_second = reorth == 1 && d.steps > 1 ? (int64_t)d.steps - 1 : 0;
    if (reorth == 2 && d.steps > 1) {
      std::vector<int> rec(d.steps - 1);
      HIPCHK(hipMemcpy(rec.data(), reorth_records(op), rec.size() * sizeof(int),
                       hipMemcpyDeviceToHost));
      for (int r : rec) op->reorth_second += r;
    }
    if (v_out && d.steps > 0) {
      download_vec(op, v_out, op->d_V, (int64_t)d.steps, mem);
      sync_checked(op);
    }
  });
}

tpl_status tpl_lanczos_pass_two(tpl_op_t op, const double* b, int64_t b_len, const double* alphas,
                                size_t n_alphas, const double* betas, size_t n_betas,
                                size_t steps, double b_norm, const double* y, size_t y_len,
                                double* x_out, double* v_out, int mem) {
  return guarded([&] {
    if (!op || !x_out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    set_device(op);
    check_b(op, b, b_len);
    // src/algorithms/lanczos_two_pass.rs:220-227
    if (steps != y_len) fail_param_mismatch("y_k", steps, y_len);
    // :229-235
    if (b_norm <= kBreakdownTol)
      fail_input("The initial vector `b` must not be a zero vector.");
    if (steps == 0) { // :237-244
      zero_out(op, x_out, mem);
      return;
    }
    if (n_alphas < steps || n_betas + 1 < steps || !alphas || (steps > 1 && !betas) || !y)
      fail(TPL_ERR_INVALID_ARGUMENT, "decomposition arrays shorter than steps_taken");
    ensure_state(op, steps);
    // decomposition -> device: norms[0], alphas, betas, y
    std::vector<double> host(1 + 3 * op->kcap, 0.0);
    (void)host;
    HIPCHK(hipMemcpyAsync(op->S.norms, &b_norm, sizeof(double), hipMemcpyHostToDevice, op->stream));
    HIPCHK(hipMemcpyAsync(op->S.alphas, alphas, steps * sizeof(double), hipMemcpyHostToDevice,
                          op->stream));
    if (steps > 1)
      HIPCHK(hipMemcpyAsync(op->S.betas, betas, (steps - 1) * sizeof(double),
                            hipMemcpyHostToDevice, op->stream));
    HIPCHK(hipMemcpyAsync(op->S.y, y, steps * sizeof(double), hipMemcpyHostToDevice, op->stream));
    upload_vec(op, op->b, b, mem);
    if (v_out) {
      ensure_basis(op, steps);
      enqueue_pass2(op, steps, op->d_V);
    } else {
      run_pass2(op, steps);
    }
    download_vec(op, x_out, op->x, 1, mem);
    if (v_out) download_vec(op, v_out, op->d_V, (int64_t)steps, mem);
    sync_checked(op);
  });
}

tpl_status tpl_lanczos_two_pass(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                                tpl_ftk_fn f, void* f_user, double* x_out, int mem) {
  return guarded([&] {
    if (!op || !x_out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    set_device(op);
    check_b(op, b, b_len);
    check_k(k);
    // the built-in inv / exp on the device: the whole solve one graph (pass one, f(T_k)
    // from the device alpha / beta, pass two), no host round trip between the passes
    const bool is_inv = f == &tpl_ftk_inv, is_exp = f == &tpl_ftk_exp;
    const size_t kmax = !op->device_ftk ? 0
                        : is_inv ? (op->device_ftk == 1 ? kDevFtkMaxK : kDevFtkAutoK)
                        : is_exp ? kDevExpMaxK : 0;
    bool have_p1 = false;  // pass one already ran (the device handed f back to the host)
    if ((is_inv || is_exp) && !op->dist && k <= kmax) {
      // inv: the host solver's operations in its order, bit for bit (src/solvers.rs:148-174);
      // exp: a parallel evaluation of the same function (k_ftk_exp), EVD-class accuracy
      ensure_state(op, k);
      upload_vec(op, op->b, b, mem);
      run_two_pass_dev(op, k, is_exp ? kDevExp : kDevInv);
      download_vec(op, x_out, op->x, 1, mem);
      HIPCHK(hipMemcpyAsync(op->h_state, op->d_state, kFlagBytes, hipMemcpyDeviceToHost,
                            op->stream));
      sync_checked(op);
      int32_t flags[kFlagBytes / 4];
      std::memcpy(flags, op->h_state, kFlagBytes);
      if (flags[1]) fail_input("Input vector `b` must not be a zero vector.");
      if (flags[2] == 0) {
        op->last_one_graph = true;
        zero_out(op, x_out, mem);
        return;
      }
      if (!flags[4]) {
        op->last_one_graph = true;
        return;
      }
      // the device handed f(T_k) back (T_k not finite, or a spectrum too wide for the
      // expansion): the host solver on the same decomposition, then pass two again
      have_p1 = true;
    }
    // 1. pass one (src/solvers.rs:148)
    op->last_one_graph = false;
    if (!have_p1) run_pass_one(op, b, k, mem, false, false);
    const HostDecomp d = fetch_decomp(op, k);
    if (d.flags[1]) fail_input("Input vector `b` must not be a zero vector.");
    if (d.steps == 0) { // :150-152
      zero_out(op, x_out, mem);
      return;
    }
    // 2. f(T_k) e_1 on the host (:155-165)
    std::vector<double> y;
    call_ftk(f, f_user, d, y);
    // 3. y = y' * ||b|| (:169)
    for (auto& v : y) v = v * d.b_norm;
    HIPCHK(hipMemcpyAsync(op->S.y, y.data(), d.steps * sizeof(double), hipMemcpyHostToDevice,
                          op->stream));
    // 4. pass two (:174)
    run_pass2(op, d.steps);
    download_vec(op, x_out, op->x, 1, mem);
    sync_checked(op);
  });
}

tpl_status tpl_lanczos(tpl_op_t op, const double* b, int64_t b_len, size_t k, tpl_ftk_fn f,
                       void* f_user, double* x_out, int mem) {
  return guarded([&] {
    if (!op || !x_out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    set_device(op);
    check_b(op, b, b_len);
    check_k(k);
    // the built-in inv / exp on the device after the standard pass, then the
    // reconstruction: no host round trip (the same rules as tpl_lanczos_two_pass; y'
    // unscaled, the GEMV multiplies by ||b||)
    const bool is_inv = f == &tpl_ftk_inv, is_exp = f == &tpl_ftk_exp;
    const size_t kmax = !op->device_ftk ? 0
                        : is_inv ? (op->device_ftk == 1 ? kDevFtkMaxK : kDevFtkAutoK)
                        : is_exp ? kDevExpMaxK : 0;
    const bool dev_f = (is_inv || is_exp) && !op->dist && k <= kmax;
    // 1. standard pass, V_k in HBM (src/solvers.rs:61); a device inv's LU eliminated
    //    during it
    run_pass_one(op, b, k, mem, true, false, dev_f && is_inv);
    op->last_one_graph = false;
    if (dev_f) {
      enqueue_ftk_only(op, k, is_exp ? kDevExp : kDevInv, 0);
      HIPCHK(launch::gemv_recon(op->n, -1, op->S, op->d_V, op->x, op->stream));
      const HostDecomp dd = fetch_decomp(op, k);
      if (dd.flags[1]) fail_input("Input vector `b` must not be a zero vector.");
      if (dd.steps == 0) {
        zero_out(op, x_out, mem);
        return;
      }
      if (!dd.flags[4]) {
        op->last_one_graph = true;
        download_vec(op, x_out, op->x, 1, mem);
        sync_checked(op);
        return;
      }
      // handed back to the host (exp only): the host solver below, on the same V_k
    }
    const HostDecomp d = fetch_decomp(op, k);
    if (d.flags[1]) fail_input("Input vector `b` must not be a zero vector.");
    if (d.steps == 0) { // :64-66
      zero_out(op, x_out, mem);
      return;
    }
    // 2. y' = f(T_k) e_1 (:71-85)
    std::vector<double> y;
    call_ftk(f, f_user, d, y);
    HIPCHK(hipMemcpyAsync(op->S.y, y.data(), d.steps * sizeof(double), hipMemcpyHostToDevice,
                          op->stream));
    // 3. x = ||b|| V_k y' (:96-104)
    HIPCHK(launch::gemv_recon(op->n, (int)d.steps, op->S, op->d_V, op->x, op->stream));
    download_vec(op, x_out, op->x, 1, mem);
    sync_checked(op);
  });
}

tpl_status tpl_op_schedule(tpl_op_t op, int32_t* n_short, int32_t* n_long, int32_t* G2,
                           int64_t* E, int32_t* short_rows_out, int32_t* long_rows_out) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    const Layout& L = op->lay;
    if (n_short) *n_short = (int32_t)L.srows.size();
    if (n_long) *n_long = (int32_t)L.lrows.size();
    if (G2) *G2 = L.G2;
    if (E) *E = L.E;
    if (short_rows_out) std::copy(L.srows.begin(), L.srows.end(), short_rows_out);
    if (long_rows_out) std::copy(L.lrows.begin(), L.lrows.end(), long_rows_out);
  });
}

tpl_status tpl_op_set_schedule(tpl_op_t op, int32_t short_row_max, int32_t max_g2) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    set_device(op);
    if (short_row_max != 0) op->sp.short_row_max = short_row_max < 0 ? -1 : short_row_max;
    if (max_g2 > 0) op->sp.max_g2 = max_g2;
    sync_checked(op);
    rebuild_schedule(op);
  });
}

tpl_status tpl_op_slices(tpl_op_t op, int32_t* slices) {
  return guarded([&] {
    if (!op || !slices) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    *slices = op->lay.nslices;
  });
}

tpl_status tpl_op_set_slices(tpl_op_t op, int32_t slices) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    if (slices < 0 || slices > kSlices || (slices & (slices - 1)) != 0)
      fail(TPL_ERR_INVALID_ARGUMENT,
           "slices must be 0 (auto) or a power of two up to " + std::to_string(kSlices));
    set_device(op);
    op->sp.slices = slices;
    sync_checked(op);
    rebuild_schedule(op);
  });
}

tpl_status tpl_copy_to_host(void* dst, const void* src_device, size_t bytes) {
  return guarded([&] {
    if (bytes == 0) return;
    if (!dst || !src_device) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    HIPCHK(hipMemcpy(dst, src_device, bytes, hipMemcpyDeviceToHost));
  });
}

double tpl_kernel_algo_bytes(tpl_op_t op, int kernel) {
  // B_spmv = 12 nnz + 4 (n+1) + 16 n (fp64 value + int32 column per
  // nonzero, int32 row_ptr, x read once, y written once). The fused kernels add the
  // epilogue vectors they must touch (DESIGN.md "Algorithmic bytes").
  if (!op) return 0.0;
  const double n = (double)op->n, nnz = (double)op->nnz;
  const double spmv = 12.0 * nnz + 4.0 * (n + 1.0) + 16.0 * n;
  switch (kernel) {
    case TPL_KERNEL_SPMV: return spmv;
    case TPL_KERNEL_PASS1_SPMV: return spmv + 8.0 * n;   // + r_{j-1} read (w is the y write)
    case TPL_KERNEL_PASS1_AXPY: return 24.0 * n;         // w, r_j read; r_{j+1} written
    case TPL_KERNEL_PASS1_STEP: return spmv + 8.0 * n + 24.0 * n;
    // + v_{j-1} read; x read and written once per three steps (grouped x updates)
    case TPL_KERNEL_PASS2_SPMV: return spmv + 8.0 * n + 16.0 * n / 3.0;
    case TPL_KERNEL_EXCHANGE_P1:
    case TPL_KERNEL_EXCHANGE_P2: {
      if (!op->dist) return 0.0;
      const double R = (double)op->dist->nranks;
      if (op->hybrid) {  // per rank: n_long partials + its chunk alpha partials (y_ld1),
        // then the norm total; pass two: n_long partials + 1
        const double nl = (double)op->lay.lrows.size();
        return kernel == TPL_KERNEL_EXCHANGE_P1 ? 8.0 * R * (op->y_ld1 + 1.0)
                                                : 8.0 * R * (nl + 1.0);
      }
      const double vec = (double)(op->halo ? op->hH : op->ld);
      // pass one: the alpha and beta totals and one vector part per rank (halo: its halo
      // slot); pass two: the vector part only (the row-block pass two gathers v, no totals)
      return kernel == TPL_KERNEL_EXCHANGE_P1 ? 8.0 * R * (vec + 2.0) : 8.0 * R * vec;
    }
    default: return 0.0;
  }
}

tpl_status tpl_op_reorth_second_passes(tpl_op_t op, int64_t* count) {
  return guarded([&] {
    if (!op || !count) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    *count = op->reorth_second;
  });
}

tpl_status tpl_op_device_bytes(tpl_op_t op, uint64_t* bytes) {
  return guarded([&] {
    if (!op || !bytes) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    uint64_t t = 0;
    for (const auto& kv : op->allocs) t += kv.second;
    *bytes = t;
  });
}

tpl_status tpl_op_set_device_ftk(tpl_op_t op, int mode) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    if (mode < 0 || mode > 2) fail(TPL_ERR_INVALID_ARGUMENT, "device f(T_k) mode must be 0, 1 or 2");
    op->device_ftk = mode;
  });
}

tpl_status tpl_op_ftk_device(tpl_op_t op, int which, const double* alphas, size_t n,
                             const double* betas, double* y_out, int* on_device) {
  return guarded([&] {
    if (!op || !alphas || !y_out || !on_device || (n > 1 && !betas))
      fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    if (which != 0 && which != 1) fail(TPL_ERR_INVALID_ARGUMENT, "which must be 0 (inv) or 1 (exp)");
    if (n == 0) fail(TPL_ERR_INVALID_ARGUMENT, "n must be >= 1");
    if (n > (which == 0 ? kDevFtkMaxK : kDevExpMaxK))
      fail(TPL_ERR_UNSUPPORTED, "k above the device f(T_k) bound");
    set_device(op);
    ensure_state(op, n);
    // the solver state as pass one leaves it: steps_taken = n, ||b|| = 1, no error
    int32_t flags[kFlagBytes / 4] = {0, 0, (int32_t)n, 0, 0, 0, 0, 0};
    const double one = 1.0;
    HIPCHK(hipMemcpyAsync(op->S.flags, flags, kFlagBytes, hipMemcpyHostToDevice, op->stream));
    HIPCHK(hipMemcpyAsync(op->S.norms, &one, sizeof(double), hipMemcpyHostToDevice, op->stream));
    HIPCHK(hipMemcpyAsync(op->S.alphas, alphas, n * sizeof(double), hipMemcpyHostToDevice,
                          op->stream));
    if (n > 1)
      HIPCHK(hipMemcpyAsync(op->S.betas, betas, (n - 1) * sizeof(double), hipMemcpyHostToDevice,
                            op->stream));
    enqueue_ftk_only(op, n, which == 1 ? kDevExp : kDevInv, 1);
    HIPCHK(hipMemcpyAsync(y_out, op->S.y, n * sizeof(double), hipMemcpyDeviceToHost, op->stream));
    HIPCHK(hipMemcpyAsync(flags, op->S.flags, kFlagBytes, hipMemcpyDeviceToHost, op->stream));
    sync_checked(op);
    *on_device = flags[4] ? 0 : 1;
  });
}

tpl_status tpl_op_enable_timing(tpl_op_t op, int on) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    op->timing = on != 0;
    op->p2_launches = 0;
    op->p1_samples = 0;
  });
}

tpl_status tpl_op_step_samples(tpl_op_t op, double* p1_spmv_us, double* p1_axpy_us,
                               int32_t* samples) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    set_device(op);
    if (!op->timing || op->p1_samples <= 0 || !op->d_stamps)
      fail(TPL_ERR_INVALID_ARGUMENT,
           "no sampled solve (enable timing, then run a two-pass solve with a device f, k >= 11)");
    unsigned long long t[2 * kStampSteps + 1];
    HIPCHK(hipMemcpyAsync(t, op->d_stamps, sizeof(t), hipMemcpyDeviceToHost, op->stream));
    sync_checked(op);
    double s1 = 0.0, s2 = 0.0;  // 100 MHz ticks
    for (int i = 0; i < kStampSteps; ++i) {
      s1 += (double)(t[2 * i + 1] - t[2 * i]);
      s2 += (double)(t[2 * i + 2] - t[2 * i + 1]);
    }
    if (p1_spmv_us) *p1_spmv_us = 0.01 * s1 / kStampSteps;
    if (p1_axpy_us) *p1_axpy_us = 0.01 * s2 / kStampSteps;
    if (samples) *samples = kStampSteps;
  });
}

tpl_status tpl_op_pass_timing(tpl_op_t op, double* pass1_us, double* pass2_spmv_us,
                              int64_t* pass2_launches) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    if (!op->timing || op->p2_launches <= 0)
      fail(TPL_ERR_INVALID_ARGUMENT, "no timed solve (enable timing, then run a two-pass solve)");
    set_device(op);
    HIPCHK(hipEventSynchronize(op->tev[3]));
    float a = 0.f, b = 0.f;
    HIPCHK(hipEventElapsedTime(&a, op->tev[0], op->tev[1]));
    HIPCHK(hipEventElapsedTime(&b, op->tev[2], op->tev[3]));
    if (pass1_us) *pass1_us = 1000.0 * (double)a;
    if (pass2_spmv_us) *pass2_spmv_us = 1000.0 * (double)b;
    if (pass2_launches) *pass2_launches = op->p2_launches;
  });
}

tpl_status tpl_profile_kernel(tpl_op_t op, int kernel, int iters, double* avg_us,
                              double* algo_bytes) {
  return guarded([&] {
    if (!op || !avg_us || iters <= 0) fail(TPL_ERR_INVALID_ARGUMENT, "bad argument");
    set_device(op);
    if (op->kcap < 4) ensure_state(op, 4);
    const CsrDev A = csr_dev(op);
    const CsrDev A1 = csr_dev(op, true);  // pass-one launches (hybrid: pass-one segment stride)
    const int big = (int)op->kcap; // j < k: the AXPY kernel does its vector work
    // Launch i of the timed sequence. The pass-two kernel rotates its three basis
    // buffers exactly as enqueue_pass2 does (the gathered vector is the previous
    // launch's output, as in a real sweep); the pass-one kernels re-run step 2.
    auto launch_one = [&](int i) {
      switch (kernel) {
        case TPL_KERNEL_SPMV:
          HIPCHK(launch::spmv(A, op->V2[0], op->W, op->stream));
          break;
        case TPL_KERNEL_PASS1_SPMV:
          HIPCHK(launch::p1_spmv(A1, op->S, op->RG[2], op->R[2], op->b, op->W, nullptr, 2,
                                 op->stream));
          break;
        case TPL_KERNEL_PASS1_AXPY:
          HIPCHK(launch::p1_axpy(A1, op->S, op->W, op->R[2], op->R[0], 2, big, 0, op->stream));
          break;
        case TPL_KERNEL_PASS1_STEP:  // both pass-one launches, re-running step 2
          HIPCHK(launch::p1_spmv(A1, op->S, op->RG[2], op->R[2], op->b, op->W, nullptr, 2,
                                 op->stream));
          HIPCHK(launch::p1_axpy(A1, op->S, op->W, op->R[2], op->R[0], 2, big, 0, op->stream));
          break;
        case TPL_KERNEL_PASS2_SPMV:
          HIPCHK(launch::p2_spmv(A, op->S, op->V2G[(i + 2) % 3], op->V2[(i + 2) % 3],
                                 op->V2[(i + 1) % 3], op->V2[i % 3], op->x, nullptr, 2,
                                 i % 3 == 2 ? 3 : 0, op->stream));
          break;
        case TPL_KERNEL_EXCHANGE_P1:
          enqueue_p1_exchange_a(op, A1);
          enqueue_p1_exchange_b(op, A1, 2);
          break;
        case TPL_KERNEL_EXCHANGE_P2:
          enqueue_p2_exchange(op, 2 + i);
          break;
        default: fail(TPL_ERR_INVALID_ARGUMENT, "unknown kernel id");
      }
    };
    const bool exchange = kernel == TPL_KERNEL_EXCHANGE_P1 || kernel == TPL_KERNEL_EXCHANGE_P2;
    if (exchange && !op->dist) fail(TPL_ERR_INVALID_ARGUMENT, "exchange ids need a partitioned operator");
    // Valid state for repeated launches: flags clear, partials/norms of a real step.
    HIPCHK(launch::p1_init(A1, op->S, op->b, op->stream));
    HIPCHK(launch::p1_spmv(A1, op->S, op->bG, op->b, nullptr, op->W, nullptr, 1, op->stream));
    HIPCHK(launch::p1_axpy(A1, op->S, op->W, op->b, op->R[2], 1, big, 0, op->stream));
    HIPCHK(hipMemcpyAsync(op->V2[1], op->b, op->n * sizeof(double), hipMemcpyDeviceToDevice,
                          op->stream));
    HIPCHK(hipMemcpyAsync(op->V2[2], op->R[2], op->n * sizeof(double), hipMemcpyDeviceToDevice,
                          op->stream));
    HIPCHK(launch::p2_coefs(op->S, (int)op->kcap, 0, op->stream));  // step 2's record
    sync_checked(op);
    auto time_eager = [&] {
      launch_one(0);
      sync_checked(op);
      HIPCHK(hipEventRecord(op->ev0, op->stream));
      for (int i = 0; i < iters; ++i) launch_one(i);
      HIPCHK(hipEventRecord(op->ev1, op->stream));
      HIPCHK(hipEventSynchronize(op->ev1));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, op->ev0, op->ev1));
      *avg_us = 1000.0 * (double)ms / iters;
      if (algo_bytes) *algo_bytes = tpl_kernel_algo_bytes(op, kernel);
    };
    // exchanges run as the solver runs them: eagerly when the transport cannot be
    // captured (the host transport synchronises the stream; an RCCL that refused capture
    // already switched the operator to eager launches, run_graph)
    if (exchange && (!op->dist->comm || op->eager || !use_graphs())) {
      time_eager();
      return;
    }
    // The launches are captured into one graph, as the solver runs them: back-to-back
    // hipLaunchKernel calls would time the host's submission rate for short kernels.
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    HIPCHK(hipStreamBeginCapture(op->stream, hipStreamCaptureModeThreadLocal));
    try {
      for (int i = 0; i < iters; ++i) launch_one(i);
    } catch (...) {
      hipStreamEndCapture(op->stream, &g);
      if (g) hipGraphDestroy(g);
      if (!exchange) throw;
      op->eager = true;  // as run_graph: the transport refused capture
      hipGetLastError();
      time_eager();
      return;
    }
    HIPCHK(hipStreamEndCapture(op->stream, &g));
    HIPCHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    HIPCHK(hipGraphLaunch(ge, op->stream)); // warm-up
    HIPCHK(hipEventRecord(op->ev0, op->stream));
    HIPCHK(hipGraphLaunch(ge, op->stream));
    HIPCHK(hipEventRecord(op->ev1, op->stream));
    HIPCHK(hipEventSynchronize(op->ev1));
    hipGraphExecDestroy(ge);
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, op->ev0, op->ev1));
    *avg_us = 1000.0 * (double)ms / iters;
    if (algo_bytes) *algo_bytes = tpl_kernel_algo_bytes(op, kernel);
  });
}


// ------------------------------------------------------------ locality order
tpl_status tpl_op_tune_order(tpl_op_t op, const int32_t* groups, int32_t count, int32_t iters,
                             int32_t* chosen, double* best_us) {
  return guarded([&] {
    if (!op || count < 0 || (count > 0 && !groups) || iters <= 0)
      fail(TPL_ERR_INVALID_ARGUMENT, "bad argument");
    if (op->dist) fail(TPL_ERR_UNSUPPORTED, "the locality order is single-GPU only");
    set_device(op);
    sync_checked(op);
    static const int32_t kDefault[] = {12, 13, 14, 15, 16, 17, 18, 19, 20, 22, 24};
    const int32_t* list = count > 0 ? groups : kDefault;
    const int32_t cnt = count > 0 ? count : (int32_t)(sizeof(kDefault) / sizeof(kDefault[0]));
    for (int32_t i = 0; i < cnt; ++i)
      if (list[i] <= 0) fail(TPL_ERR_INVALID_ARGUMENT, "group counts must be positive");
    // a failed timing launch leaves the operator as it was (order mode, group count)
    const int saved_reorder = op->reorder, saved_groups = op->sp.order_groups;
    try {
      op->reorder = 1;
      // any non-zero b: the timed SpMV launches need a step's valid partials and norms
      // (b is the solver's input staging buffer, re-written by every solve)
      const std::vector<double> ones(op->n, 1.0);
      double best = 0.0;
      int32_t best_g = op->sp.order_groups;
      for (int32_t i = 0; i < cnt; ++i) {
        op->sp.order_groups = list[i];
        rebuild_schedule(op);
        if (op->perm.empty()) break;  // no long rows: nothing to order
        if (op->n > 0)
          HIPCHK(hipMemcpy(op->b, ones.data(), op->n * sizeof(double), hipMemcpyHostToDevice));
        double t1 = 0.0, t2 = 0.0;
        for (const auto& kt : {std::make_pair(TPL_KERNEL_PASS1_SPMV, &t1),
                               std::make_pair(TPL_KERNEL_PASS2_SPMV, &t2)}) {
          const tpl_status st = tpl_profile_kernel(op, kt.first, iters, kt.second, nullptr);
          if (st != TPL_OK) fail(st, tpl_last_error());
        }
        if (i == 0 || t1 + t2 < best) {
          best = t1 + t2;
          best_g = list[i];
        }
      }
      op->sp.order_groups = best_g;
      rebuild_schedule(op);
      if (chosen) *chosen = best_g;
      if (best_us) *best_us = best;
    } catch (...) {
      op->reorder = saved_reorder;
      op->sp.order_groups = saved_groups;
      hipGetLastError();
      rebuild_schedule(op);
      throw;
    }
  });
}

tpl_status tpl_op_set_order_groups(tpl_op_t op, int32_t groups) {
  return guarded([&] {
    if (!op) fail(TPL_ERR_INVALID_ARGUMENT, "op is NULL");
    if (groups < 0) fail(TPL_ERR_INVALID_ARGUMENT, "group count must be >= 0 (0: default 16)");
    if (op->dist) fail(TPL_ERR_UNSUPPORTED, "the locality order is single-GPU only");
    set_device(op);
    sync_checked(op);
    op->sp.order_groups = groups > 0 ? groups : SchedParams{}.order_groups;
    rebuild_schedule(op);
  });
}

int32_t tpl_op_order_groups(tpl_op_t op) {
  if (!op) return -1;
  return !op->perm.empty() ? op->sp.order_groups : 0;
}

// ------------------------------------------------------------ row partition
tpl_status tpl_dist_partition(int64_t n, const int64_t* row_ptr, int nranks, int64_t* starts) {
  return guarded([&] {
    if (!row_ptr || !starts || nranks < 1) fail(TPL_ERR_INVALID_ARGUMENT, "bad argument");
    if (n < nranks) fail(TPL_ERR_INVALID_ARGUMENT, "fewer rows than ranks");
    // contiguous row blocks balanced by algorithmic bytes: 12 per nonzero (value +
    // column) + 40 per row (pass two's vector traffic)
    std::vector<double> prefix(n + 1);
    for (int64_t i = 0; i <= n; ++i) prefix[i] = 12.0 * (double)row_ptr[i] + 40.0 * (double)i;
    balanced_cuts(prefix, nranks, starts);
  });
}

tpl_status tpl_dist_unique_id(uint8_t* id) {
  return guarded([&] {
    if (!id) fail(TPL_ERR_INVALID_ARGUMENT, "id is NULL");
    static_assert(sizeof(ncclUniqueId) == TPL_DIST_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
  });
}

static tpl_dist_s* new_dist(int device, int rank, int nranks) {
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) fail(TPL_ERR_DEVICE, "no HIP device available");
  if (device < 0 || device >= cnt) fail(TPL_ERR_INVALID_ARGUMENT, "device index out of range");
  if (nranks < 1 || rank < 0 || rank >= nranks) fail(TPL_ERR_INVALID_ARGUMENT, "bad rank / nranks");
  HIPCHK(hipSetDevice(device));
  auto d = std::make_unique<tpl_dist_s>();
  d->ctx.device = device;
  d->rank = rank;
  d->nranks = nranks;
  HIPCHK(hipStreamCreateWithFlags(&d->ctx.stream, hipStreamNonBlocking));
  return d.release();
}

tpl_status tpl_dist_create(int device, int rank, int nranks, const uint8_t* id, tpl_dist_t* out) {
  return guarded([&] {
    if (!id || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    std::unique_ptr<tpl_dist_s> d(new_dist(device, rank, nranks));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    NCCLCHK(ncclCommInitRank(&d->comm, nranks, u, rank));
    *out = d.release();
  });
}

tpl_status tpl_dist_create_host(int device, int rank, int nranks, tpl_allgather_fn fn, void* user,
                                tpl_dist_t* out) {
  return guarded([&] {
    if (!fn || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    std::unique_ptr<tpl_dist_s> d(new_dist(device, rank, nranks));
    d->host_fn = fn;
    d->host_user = user;
    *out = d.release();
  });
}

tpl_status tpl_dist_destroy(tpl_dist_t d) {
  return guarded([&] {
    if (!d) return;
    hipSetDevice(d->ctx.device);
    if (d->ctx.stream) hipStreamSynchronize(d->ctx.stream);
    if (d->comm) ncclCommDestroy(d->comm);
    if (d->ctx.stream) hipStreamDestroy(d->ctx.stream);
    delete d;
  });
}

tpl_status tpl_dist_op_create_csr(tpl_dist_t d, int64_t n_global, const int64_t* starts,
                                  const int64_t* row_ptr, const int32_t* col_idx,
                                  const double* vals, tpl_op_t* out) {
  return guarded([&] {
    if (!d || !starts || !row_ptr || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    const int R = d->nranks;
    if (starts[0] != 0 || starts[R] != n_global) fail(TPL_ERR_INVALID_ARGUMENT, "bad partition");
    for (int r = 0; r < R; ++r)
      if (starts[r + 1] <= starts[r]) fail(TPL_ERR_INVALID_ARGUMENT, "empty or unordered block");
    if (n_global >= INT32_MAX / 2) fail(TPL_ERR_UNSUPPORTED, "n must be < 2^30");
    const int64_t n = starts[d->rank + 1] - starts[d->rank];
    const int64_t nnz = row_ptr[n];
    if (row_ptr[0] != 0 || nnz < 0 || nnz >= INT32_MAX)
      fail(TPL_ERR_INVALID_ARGUMENT, "row_ptr must start at 0; nnz < 2^31");
    if (nnz > 0 && !vals) fail(TPL_ERR_INVALID_ARGUMENT, "col_idx/vals is NULL");
    check_csr(n, n_global, row_ptr, col_idx);
    HIPCHK(hipSetDevice(d->ctx.device));
    auto op = std::make_unique<tpl_op_s>();
    op->ctx = &d->ctx;
    op->device = d->ctx.device;
    op->stream = d->ctx.stream;
    op->dist = d;
    op->eager = d->comm == nullptr;
    op->n = n;
    op->n_glob = n_global;
    op->nnz = nnz;
    op->starts.assign(starts, starts + R + 1);
    op->h_rowptr.resize(n + 1);
    for (int64_t i = 0; i <= n; ++i) op->h_rowptr[i] = (int32_t)row_ptr[i];
    op->h_col.assign(col_idx, col_idx + nnz);
    op->h_val.assign(vals, vals + nnz);
    init_op(op.get());
    *out = op.release();
  });
}


tpl_status tpl_dist_op_create_halo(tpl_dist_t d, int64_t n, const int64_t* starts,
                                   const int64_t* row_ptr, const int32_t* col_idx,
                                   const double* vals, tpl_op_t* out) {
  return guarded([&] {
    if (!d || !row_ptr || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    HIPCHK(hipSetDevice(d->ctx.device));
    auto op = std::make_unique<tpl_op_s>();
    op->ctx = &d->ctx;
    op->device = d->ctx.device;
    op->stream = d->ctx.stream;
    op->dist = d;
    op->eager = d->comm == nullptr;
    fill_rows(op.get(), d->nranks, d->rank, n, starts, row_ptr, col_idx, vals, true);
    init_op(op.get());
    *out = op.release();
  });
}

tpl_status tpl_dist_op_create_replicated(tpl_dist_t d, int64_t n, const int64_t* row_ptr,
                                         const int32_t* col_idx, const double* vals,
                                         tpl_op_t* out) {
  return guarded([&] {
    if (!d || !row_ptr || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    HIPCHK(hipSetDevice(d->ctx.device));
    auto op = std::make_unique<tpl_op_s>();
    op->ctx = &d->ctx;
    op->device = d->ctx.device;
    op->stream = d->ctx.stream;
    op->dist = d;
    op->eager = d->comm == nullptr;
    fill_replicated(op.get(), d->nranks, d->rank, n, row_ptr, col_idx, vals);
    init_op(op.get());
    *out = op.release();
  });
}

tpl_status tpl_dist_choose_partition(int64_t n, const int64_t* row_ptr, const int32_t* col_idx,
                                     int nranks, int* mode) {
  return guarded([&] {
    if (!mode) fail(TPL_ERR_INVALID_ARGUMENT, "mode is NULL");
    *mode = choose_partition(n, row_ptr, col_idx, nranks);
  });
}

tpl_status tpl_dist_op_create_auto(tpl_dist_t d, int64_t n, const int64_t* row_ptr,
                                   const int32_t* col_idx, const double* vals, tpl_op_t* out,
                                   int* mode) {
  return guarded([&] {
    if (!d || !row_ptr || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    const int m = choose_partition(n, row_ptr, col_idx, d->nranks);
    HIPCHK(hipSetDevice(d->ctx.device));
    auto op = std::make_unique<tpl_op_s>();
    op->ctx = &d->ctx;
    op->device = d->ctx.device;
    op->stream = d->ctx.stream;
    op->dist = d;
    op->eager = d->comm == nullptr;
    if (m == TPL_PLAN_REPLICATED)
      fill_replicated(op.get(), d->nranks, d->rank, n, row_ptr, col_idx, vals);
    else
      fill_rows(op.get(), d->nranks, d->rank, n, nullptr, row_ptr, col_idx, vals,
                m == TPL_PLAN_HALO);
    init_op(op.get());
    if (mode) *mode = m;
    *out = op.release();
  });
}

tpl_status tpl_operand_key(int64_t n, const void* ptr_arr, size_t ptr_len, size_t ptr_elem,
                           const void* idx_arr, size_t idx_len, size_t idx_elem,
                           const double* vals, size_t nnz, size_t samples, uint64_t* key) {
  return guarded([&] {
    if (!key) fail(TPL_ERR_INVALID_ARGUMENT, "key is NULL");
    if ((ptr_len && !ptr_arr) || (idx_len && !idx_arr) || (nnz && !vals))
      fail(TPL_ERR_INVALID_ARGUMENT, "NULL array with a nonzero length");
    if ((ptr_elem != 4 && ptr_elem != 8) || (idx_elem != 4 && idx_elem != 8))
      fail(TPL_ERR_INVALID_ARGUMENT, "index element size must be 4 or 8 bytes");
    uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a over 64-bit words
    auto mix = [&](uint64_t w) { h = (h ^ w) * 0x100000001b3ull; };
    // identity: the arrays' addresses and lengths, the dimension
    for (uint64_t w : {(uint64_t)n, (uint64_t)(uintptr_t)ptr_arr, (uint64_t)ptr_len,
                       (uint64_t)(uintptr_t)idx_arr, (uint64_t)idx_len,
                       (uint64_t)(uintptr_t)vals, (uint64_t)nnz})
      mix(w);
    key[0] = h;
    // contents: the first and last 8 words of each array and `samples` evenly spaced
    // ones (positions i * len / samples), so the check costs O(samples), not O(nnz)
    h = 0xcbf29ce484222325ull;
    auto sample = [&](const void* a, size_t len, size_t elem) {
      auto word = [&](size_t i) {
        return elem == 8 ? ((const uint64_t*)a)[i] : (uint64_t)((const uint32_t*)a)[i];
      };
      for (size_t i = 0; i < std::min<size_t>(len, 8); ++i) mix(word(i));
      for (size_t i = len > 8 ? len - 8 : len; i < len; ++i) mix(word(i));
      if (len > 16)
        for (size_t s = 0; s < samples; ++s) mix(word((size_t)((unsigned __int128)s * len / samples)));
    };
    sample(ptr_arr, ptr_len, ptr_elem);
    sample(idx_arr, idx_len, idx_elem);
    sample(vals, nnz, 8);
    key[1] = h;
  });
}

tpl_status tpl_op_local_rows(tpl_op_t op, int64_t* rows) {
  return guarded([&] {
    if (!op || !rows) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    if (op->hybrid) {
      std::copy(op->local_rows.begin(), op->local_rows.end(), rows);
    } else {
      const int64_t r0 = op->dist ? op->starts[op->dist->rank] : 0;
      for (int64_t i = 0; i < op->n; ++i) rows[i] = r0 + i;
    }
  });
}

// ------------------------------------------------------------ host-only plans
tpl_status tpl_plan_create(int64_t n, const int64_t* row_ptr, const int32_t* col_idx,
                           const double* vals, int mode, int nranks, int rank,
                           int32_t order_groups, tpl_op_t* out) {
  return guarded([&] {
    if (!row_ptr || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    if (mode < TPL_PLAN_SINGLE || mode > TPL_PLAN_HALO)
      fail(TPL_ERR_INVALID_ARGUMENT,
           "plan mode must be TPL_PLAN_SINGLE, _REPLICATED, _ROWS or _HALO");
    if (mode == TPL_PLAN_SINGLE ? (nranks != 1 || rank != 0)
                                : (nranks < 1 || rank < 0 || rank >= nranks))
      fail(TPL_ERR_INVALID_ARGUMENT, "bad rank / nranks");
    if (order_groups < 0) fail(TPL_ERR_INVALID_ARGUMENT, "group count must be >= 0 (0: default 16)");
    if (n < 0) fail(TPL_ERR_INVALID_ARGUMENT, "negative size");
    const int64_t nnz = row_ptr[n];
    if (nnz > 0 && (!vals || !col_idx)) fail(TPL_ERR_INVALID_ARGUMENT, "col_idx/vals is NULL");
    auto op = std::make_unique<tpl_op_s>();
    op->plan_only = true;
    if (mode == TPL_PLAN_SINGLE) {  // tpl_op_create_csr's host half
      if (n >= INT32_MAX || nnz >= INT32_MAX)
        fail(TPL_ERR_UNSUPPORTED, "n and nnz must be < 2^31 (int32 device offsets)");
      check_csr(n, n, row_ptr, col_idx);
      op->n = op->n_glob = n;
      op->nnz = nnz;
      op->h_rowptr.assign(row_ptr, row_ptr + n + 1);
      op->h_col.assign(col_idx, col_idx + nnz);
      op->h_val.assign(vals, vals + nnz);
      if (order_groups > 0) op->sp.order_groups = order_groups;
    } else {
      op->plan_dist = std::make_unique<tpl_dist_s>();
      op->plan_dist->rank = rank;
      op->plan_dist->nranks = nranks;
      op->dist = op->plan_dist.get();
      if (mode == TPL_PLAN_REPLICATED) {
        fill_replicated(op.get(), nranks, rank, n, row_ptr, col_idx, vals);
      } else {  // the block tpl_dist_partition gives this rank (tpl_dist_op_create_csr /
                // tpl_dist_op_create_halo)
        fill_rows(op.get(), nranks, rank, n, nullptr, row_ptr, col_idx, vals,
                  mode == TPL_PLAN_HALO);
      }
    }
    set_stride(op.get());
    rebuild_schedule(op.get());  // the layout only (plan_only: nothing is uploaded)
    *out = op.release();
  });
}

} // extern "C"
