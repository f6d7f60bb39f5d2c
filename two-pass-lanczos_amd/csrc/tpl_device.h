// tpl_device.h — structures shared by the HIP kernels (tpl_kernels.hip) and the
// host runtime (tpl_runtime.cpp). Everything here is plain data: the kernels take
// these structs by value as kernel arguments.
//
// SpMV schedule (built once per operator, tpl_runtime.cpp build_schedule):
//   * short rows (<= kShortRowMax nnz) are grouped into STREAM items of consecutive
//     rows (<= kStreamNnzCap nnz, <= kStreamRowsCap rows): one workgroup each, a
//     coalesced sweep of the item's nnz into LDS, then one thread per row.
//   * long rows are cut into kSlices column slices [s*n/8, (s+1)*n/8); a SLICE unit =
//     (group of 4 long rows, slice s), one wave per row. Workgroup b of the SpMV grid
//     handles slice b % 8: under the observed round-robin dispatch that keeps each
//     XCD's L2 on 1/8 of the gathered vector (speed only, never correctness). Slice
//     partials P[r][s] are summed by a small combine kernel, which also runs the
//     long rows' epilogue.
//
// Canonical reduction order (reproduced bit for bit by oracle/lanczos_oracle.c):
//   * tree256(a[256])  : per 64-lane wave an xor butterfly (offsets 32,16,8,4,2,1,
//                        a_l <- a_l + a_{l^off}), then (S0 + S1) + (S2 + S3).
//   * partials(P[N])   : thread t: s_t = 0; s_t += P[t + 256q] (q ascending); tree256.
//   * short row        : s = 0; s += round(a_k x_k), k ascending.
//   * long row         : per slice s: lane l: p_l = 0; p_l += round(a_k x_k) for
//                        k = off[s] + l + 64q; P[s] = butterfly64(p); y = 0; y += P[s], s = 0..7.
//   * alpha partial    : STREAM item i -> Pa[i]: thread t accumulates acc = fma(v, w, acc)
//                        over its rows row0 + t + 256q, then tree256.
//                        combine workgroup c -> Pa[n_stream + c]: thread t owns long row
//                        256c + t (acc = fma(v, w, 0)), tree256.
//   * norm partial     : workgroup b (of G2) owns [bE, min(n,(b+1)E)); thread t visits
//                        i0 = bE + 2t + 512q, then i0, i0+1: acc = fma(x,x,acc); tree256.
#pragma once
#include <stdint.h>

namespace tpl {

constexpr int kTPB = 256;            // threads per workgroup (4 waves of 64)
constexpr int kStreamNnzCap = 2048;  // max nnz of one STREAM item (LDS product buffer)
constexpr int kStreamRowsCap = 1024; // max rows of one STREAM item (4 rows per thread)
constexpr int kShortRowMax = 32;     // rows with more nnz are "long" (sliced)
constexpr int kSlices = 8;           // column slices of a long row (= XCDs)
constexpr int kLongRowsPerGroup = 4; // one wave per row
constexpr double kBreakdownTol = 2.220446049250313080847263336181640625e-13; // 1000*f64::EPSILON, src/algorithms/mod.rs:140-143

struct Item {
  int32_t row0, row1; // rows [row0, row1)
  int32_t nz0;        // row_ptr[row0]
  int32_t pad;
};

// Device view of the CSR operator plus its schedule.
struct CsrDev {
  const int32_t* row_ptr;  // n+1 (int32: nnz < 2^31)
  const int32_t* col;      // nnz
  const double* val;       // nnz
  const Item* items;       // n_stream STREAM items
  const int32_t* lrows;    // n_long long-row indices (ascending)
  const int32_t* loff;     // n_long x (kSlices+1) slice offsets into col/val
  double* P;               // n_long x kSlices slice partials
  int32_t n_stream;
  int32_t n_long;
  int32_t n_slice_blocks;  // kSlices * ceil(n_long / 4); SpMV grid = n_slice_blocks + n_stream
  int32_t n_comb_blocks;   // ceil(n_long / 256)
  int32_t G2;              // workgroups of the element-wise kernels == #norm partials
  int32_t NA;              // #alpha partials = n_stream + n_comb_blocks
  int64_t n;
  int64_t E;               // elements per workgroup of the element-wise kernels
};

// Device-resident solver state (one per operator).
struct DevState {
  int32_t* flags;   // [0] stop, [1] error (1 = zero b), [2] steps_taken
  double* norms;    // [0] = ||b||, [j] = beta_j                         (kcap+1)
  double* alphas;   // alphas[j-1] = alpha_j                              (kcap)
  double* betas;    // betas[j-1]  = beta_j                               (kcap)
  double* y;        // pass-two coefficients y_k (already * ||b||), or y' (kcap)
  double* Pa;       // alpha partials (NA)
  double* Pb;       // ||.||^2 partials (G2)
};

} // namespace tpl
