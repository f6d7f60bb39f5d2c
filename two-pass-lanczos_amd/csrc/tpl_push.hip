// tpl_push.hip — pushed long rows (CsrDev::push == 1).
//
// The long rows of a KKT operator (node rows, ~867 entries each at 500k arcs) gather
// the vector at random columns: ~1 M scattered 8-byte reads per SpMV, one L2 request
// each, which is what bounds the bin kernels (tpl_kernels.hip). When every long-row
// entry (i, a) lies in a short column a and mirrors the short row's entry (a, i) with
// the same value (structurally and numerically symmetric off-diagonal blocks, the KKT
// case), the long rows are computed from the short rows' side instead: the chunk that
// owns short row a already holds x_a (its own vector entry, loaded coalesced) and the
// entries (a, i), so it PUSHES the products A_ia x_a into LDS slots sorted by long row,
// sums each long row's run into one partial per (chunk, long row), and writes the
// chunk's n_long partials coalesced. Combiner workgroups then finish every long row
// from its n_chunks partials (16 lanes per row, fixed order — tpl_device.h). No
// scattered read remains on the SpMV path.
//
// Scheduling (tpl_runtime.cpp):
//   pass one, step j:  k_push_p1 (chunks: short rows, alpha partials, partials of
//                      A v_j) -> k_push_p1_comb (long rows: w, alpha products) ->
//                      k_p1_axpy (unchanged).
//   pass two, step j:  ONE launch k_push_p2 = [combiners | chunks]. The combiners
//                      finish the long rows of v_{j+1} from the partials of A v_j that
//                      the previous launch's chunks pushed; the chunks compute the short
//                      rows of v_{j+1} (gathering v_j at long columns, final since the
//                      previous launch) and push the partials of A v_{j+1} for the next
//                      launch (two partial buffers, by step parity). Pass-two
//                      coefficients are all known, so nothing inside a launch waits on
//                      anything else in it.
//   plain A x:         k_push_spmv (chunks) -> k_push_comb_y (long rows).
// Arithmetic per element is the reference's (round(a x) products, the same epilogue
// operations); only the long rows' summation order differs from the bins'.
#include "tpl_kcommon.h"

namespace tpl {

// partials() (tpl_device.h) in a workgroup of kPushTPB threads: threads 0..255 follow
// the canonical 256-thread order (tree256), the others contribute nothing.
__device__ __forceinline__ double finish_partials_256(const double* __restrict__ P, int N,
                                                      const PartialRegs<4>& r, double* red) {
  const int t = threadIdx.x;
  double s = 0.0;
  if (t < kTPB) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * kTPB < N) s = s + r.v[u];
    for (int i = t + 4 * kTPB; i < N; i += kTPB) s = s + P[i];  // N > 1024 (rare)
  }
  s = wave_sum(s);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  const double res = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return res;
}

// tree512: per-wave butterfly, then ((S0 + S1) + (S2 + S3)) + ((S4 + S5) + (S6 + S7)).
__device__ __forceinline__ double block_sum_512(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
  __syncthreads();
  return r;
}

// Vector entry of the row itself: what a chunk pushes in a plain SpMV (y optional).
struct PreX {
  double x;
};
__device__ __forceinline__ void keep_pre(PreX& p) { keep(p.x); }
struct EpiPushX {
  const double* xv;
  double* y;  // nullptr: push only (pass-two prologue)
  __device__ __forceinline__ PreX pre(int i) const { return PreX{xv[i]}; }
  __device__ __forceinline__ double apply(int i, double s, const PreX& p, double&) const {
    if (y) y[i] = s;
    return p.x;
  }
  __device__ __forceinline__ void long_alpha(int, double) const {}
};

// Pushing chunk: short-row positions [C*chunk, C*(chunk+1)), C = kPushTPB RPT, uniform
// width W. Writes the chunk's n_long partials to Pout[chunk * n_long + l].
// LDS: tp_cap product slots, then the long-run queue.
template <int W, int RPT, int V8, int C16, class Epi, class ScaleFn>
__device__ __forceinline__ bool push_chunk(const CsrDev& A, int chunk,
                                           const double* __restrict__ xsrc, ScaleFn scale_of,
                                           const Epi& epi, double& acc, double* lds,
                                           double* __restrict__ Pout) {
  constexpr int C = RPT * kPushTPB;
  const int t = threadIdx.x;
  const int nl = A.n_long;
  const int cbase = C16 ? A.s_cbase[chunk] : 0;
  const int base = chunk * C * W;
  int row[RPT];
  bool live[RPT];
  decltype(epi.pre(0)) pre[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int p = chunk * C + q * kPushTPB + t;
    live[q] = p < A.n_short;
    const int pc = clampi(p, A.n_short - 1);
    row[q] = A.s_identity ? pc : A.srows[pc];
  }
  // issue order = arrival order: entries (the gathers wait on them), run starts, the
  // rows' own vector entries, then the gathers
  int c[RPT][W], ps[RPT][W];
  double a[RPT][W], xv[RPT][W];
#pragma unroll
  for (int q = 0; q < RPT; ++q)
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int e = base + k * C + q * kPushTPB + t;
      c[q][k] = col_at<C16>(A.s_col, e, cbase);
      a[q][k] = val_at<V8>(A.s_val, e);
      ps[q][k] = A.s_pos[e];
    }
  // run bounds of this thread's long rows i = t + 256m: [seg[i], seg[i + 1])
  const uint16_t* seg = A.tp_seg + (size_t)chunk * (nl + 1);
  int sg[kPushSegLoads], sgn[kPushSegLoads];
#pragma unroll
  for (int m = 0; m < kPushSegLoads; ++m) {
    sg[m] = seg[clampi(t + m * kPushTPB, nl)];
    sgn[m] = seg[clampi(t + m * kPushTPB + 1, nl)];
  }
#pragma unroll
  for (int q = 0; q < RPT; ++q) pre[q] = epi.pre(row[q]);
#pragma unroll
  for (int q = 0; q < RPT; ++q)
#pragma unroll
    for (int k = 0; k < W; ++k) xv[q][k] = xsrc[c[q][k] < 0 ? 0 : c[q][k]];
  const Scale sc = scale_of();
  TPL_MARK(1);
  if (!sc.ok) return false;  // stopped / breakdown (uniform)
#pragma unroll
  for (int q = 0; q < RPT; ++q) keep_pre(pre[q]);
  // long-run queue: [0] count, then (long row, s0 | s1 << 16) per queued run
  int* lbig = reinterpret_cast<int*>(lds + A.tp_cap);
  if (t == 0) lbig[0] = 0;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    double sum = 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      double prod = a[q][k] * (xv[q][k] * sc.s);
      keep(prod);
      sum = c[q][k] >= 0 ? sum + prod : sum;
    }
    const double u = live[q] ? epi.apply(row[q], sum, pre[q], acc) : 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k)  // padding and short-column entries carry 0xFFFF
      if (ps[q][k] != 0xFFFF) lds[ps[q][k]] = a[q][k] * u;
  }
  __syncthreads();
  TPL_MARK(2);
  // Run sums (canonical order, tpl_device.h). Arcs arrive grouped by tail node, so a
  // chunk holds a few runs of hundreds of entries beside ~n_long runs of 0..4: a run of
  // at most kPushRun entries is summed by its thread in order; a longer one is queued
  // and summed by a whole wave (lane l: entries l + 64q, then the wave butterfly).
  // Rows in groups of three (a group whose first row is past n_long is skipped), the
  // first kRunRegs slots of each run read together: with ~1.8 head entries per run
  // (Poisson-like), a longer run (serial tail loop) is rare in a wave.
  constexpr int kRunRegs = 8, kGrp = 3;
#pragma unroll
  for (int m0 = 0; m0 < kPushSegLoads; m0 += kGrp) {
    if (m0 * kPushTPB >= nl) break;  // uniform
    double rv[kGrp][kRunRegs];
#pragma unroll
    for (int g = 0; g < kGrp; ++g)
#pragma unroll
      for (int u = 0; u < kRunRegs; ++u) {  // past the run: re-read its first slot (or
        const int m = m0 + g < kPushSegLoads ? m0 + g : kPushSegLoads - 1;  // the queue
        rv[g][u] = lds[sg[m] + (u < sgn[m] - sg[m] ? u : 0)];  // word when empty)
      }
#pragma unroll
    for (int g = 0; g < kGrp; ++g) {
      const int m = m0 + g;
      if (m >= kPushSegLoads) break;
      const int i = t + m * kPushTPB;
      const int s0 = sg[m], s1 = sgn[m];
      if (i >= nl) continue;
      if (s1 - s0 > kPushRun) {
        const int at = atomicAdd(lbig, 1);
        lbig[1 + 2 * at] = i;
        lbig[2 + 2 * at] = s0 | (s1 << 16);
        continue;
      }
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < kRunRegs; ++u) s = s0 + u < s1 ? s + rv[g][u] : s;
      for (int e = s0 + kRunRegs; e < s1; ++e) s = s + lds[e];  // rare: 9 .. kPushRun
      Pout[(size_t)chunk * nl + i] = s;
    }
  }
  __syncthreads();
  TPL_MARK(4);
  const int nbig = lbig[0], lane = t & 63;
  for (int b = t >> 6; b < nbig; b += kPushTPB / 64) {
    const int i = lbig[1 + 2 * b], se = lbig[2 + 2 * b];
    const int s0 = se & 0xFFFF, s1 = (int)((unsigned)se >> 16);
    double rs = 0.0;
    for (int k0 = s0 + lane; k0 < s1; k0 += 512) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = lds[k0 + 64 * u < s1 ? k0 + 64 * u : k0];
#pragma unroll
      for (int u = 0; u < 8; ++u) rs = k0 + 64 * u < s1 ? rs + v[u] : rs;
    }
    rs = wave_sum(rs);
    if (lane == 0) Pout[(size_t)chunk * nl + i] = rs;
  }
  TPL_MARK(3);
  return true;
}

template <int F, class Epi, class ScaleFn>
__device__ __forceinline__ bool push_chunk_f(const CsrDev& A, int chunk, const double* xsrc,
                                             ScaleFn scale_of, const Epi& epi, double& acc,
                                             double* lds, double* Pout) {
  return push_chunk<(F & 7), ((F >> 5) & 1) ? 4 : 1, ((F >> 3) & 1), ((F >> 4) & 1)>(
      A, chunk, xsrc, scale_of, epi, acc, lds, Pout);
}

// Combiner workgroup blk: long rows blk * kCombRows + (t >> 4); lane g = t & 15 sums the
// partials of chunks g + 16q, then the 16-lane butterfly; lane 0 finishes the row.
constexpr int kCombLoads = 16;  // partial loads in flight per lane (256 chunks a batch)
template <class Epi, class ScaleFn>
__device__ __forceinline__ void push_combine(const CsrDev& A, int blk,
                                             const double* __restrict__ Pin, ScaleFn scale_of,
                                             const Epi& epi) {
  const int t = threadIdx.x, g = t & 15;
  const int nl = A.n_long, nc = A.n_chunks;
  const int li = blk * kCombRows + (t >> 4);
  const bool live = li < nl;
  const int lc = live ? li : nl - 1;
  const int row = A.lrows[lc];
  double s = 0.0;
  for (int w0 = 0; w0 < nc; w0 += 16 * kCombLoads) {
    double v[kCombLoads];
#pragma unroll
    for (int u = 0; u < kCombLoads; ++u)
      v[u] = Pin[(size_t)clampi(w0 + g + 16 * u, nc - 1) * nl + lc];
#pragma unroll
    for (int u = 0; u < kCombLoads; ++u) s = (w0 + g + 16 * u < nc) ? s + v[u] : s;
  }
  auto pre = epi.pre(row);
  s = group16_sum(s);
  const Scale sc = scale_of();
  if (!sc.ok) return;
  keep_pre(pre);
  if (g == 0 && live) {
    double acc = 0.0;
    epi.apply(row, s, pre, acc);
    epi.long_alpha(li, acc);
  }
}

__device__ __forceinline__ double* push_buf(const CsrDev& A, int parity) {
  return A.tpP + (size_t)(parity & 1) * A.n_chunks * A.n_long;
}

// ------------------------------------------------------------------ kernels
// Pass one / standard, step j: the short rows (as k_p1_spmv's chunks) + the partials
// of A v_j for the long rows (buffer j % 2) + the short chunks' alpha partials.
template <int F>
__global__ __launch_bounds__(kPushTPB) void k_push_p1(CsrDev A, DevState S,
                                                  const double* __restrict__ xsrc,
                                                  const double* __restrict__ r_cur,
                                                  const double* __restrict__ r_prev,
                                                  double* __restrict__ W,
                                                  double* __restrict__ Vcol, int j) {
  __shared__ double red[kPushTPB / 64];
  extern __shared__ double lds[];
  PartialRegs<4> pr;  // G2 <= 1024 (threads 0..255 reduce them)
  load_partials(S.Pb_r, A.G2_r, pr);
  EpiPass1 epi;
  epi.r_cur = r_cur;
  epi.r_prev = (j >= 2) ? r_prev : r_cur;
  epi.has_prev = j >= 2;
  epi.invN_prev = 0.0;
  epi.invN_cur = 0.0;
  epi.beta_sub = 0.0;
  epi.W = W;
  epi.Vcol = Vcol;
  epi.Pa_long = nullptr;
  // beta_{j-1} (||b|| at j = 1) from the norm partials, as k_p1_spmv
  auto scale_fn = [&]() -> Scale {
    __builtin_amdgcn_sched_barrier(0);
    if (S.flags[0]) return Scale{0.0, false};
    epi.invN_prev = (j >= 2) ? 1.0 / S.norms[j - 2] : 0.0;
    const double beta = sqrt(finish_partials_256(S.Pb_r, A.G2_r, pr, red));
    if (beta <= kBreakdownTol) {
      // j == 1: zero b -> InputError (src/algorithms/mod.rs:267-273);
      // j  > 1: breakdown -> steps_taken = j - 1 (src/algorithms/lanczos_two_pass.rs:245-249)
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        S.flags[0] = 1;
        if (j == 1) S.flags[1] = 1;
      }
      return Scale{0.0, false};
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      S.norms[j - 1] = beta;
      if (j >= 2) S.betas[j - 2] = beta;
    }
    epi.invN_cur = 1.0 / beta;
    epi.beta_sub = (j >= 2) ? beta : 0.0;
    return Scale{epi.invN_cur, true};
  };
  double acc = 0.0;
  if (!push_chunk_f<F>(A, blockIdx.x, xsrc, scale_fn, epi, acc, lds, push_buf(A, j))) return;
  const double p = block_sum_512(acc, red);
  if (threadIdx.x == 0) S.Pa[blockIdx.x] = p;
}

// Pass one / standard, step j: the long rows from the partials of A v_j:
// w = y - beta_{j-1} v_{j-1}; alpha product v_j . w into Pa[n_chunks + l].
__global__ __launch_bounds__(kPushTPB) void k_push_p1_comb(CsrDev A, DevState S,
                                                       const double* __restrict__ r_cur,
                                                       const double* __restrict__ r_prev,
                                                       double* __restrict__ W,
                                                       double* __restrict__ Vcol, int j) {
  EpiPass1 epi;
  epi.r_cur = r_cur;
  epi.r_prev = (j >= 2) ? r_prev : r_cur;
  epi.has_prev = j >= 2;
  epi.W = W;
  epi.Vcol = Vcol;
  epi.Pa_long = S.Pa + A.n_chunks;
  epi.invN_prev = 0.0;
  epi.invN_cur = 0.0;
  epi.beta_sub = 0.0;
  auto scale_fn = [&]() -> Scale {
    __builtin_amdgcn_sched_barrier(0);
    if (S.flags[0]) return Scale{0.0, false};
    const double beta = S.norms[j - 1];
    epi.invN_prev = (j >= 2) ? 1.0 / S.norms[j - 2] : 0.0;
    epi.invN_cur = 1.0 / beta;
    epi.beta_sub = (j >= 2) ? beta : 0.0;
    return Scale{epi.invN_cur, true};
  };
  push_combine(A, blockIdx.x, push_buf(A, j), scale_fn, epi);
}

// Pass two, step j = 1 .. steps-1: [n_comb combiners | n_chunks chunks] (see top).
template <int F>
__global__ __launch_bounds__(kPushTPB) void k_push_p2(CsrDev A, DevState S,
                                                  const double* __restrict__ xsrc,
                                                  const double* __restrict__ v_cur,
                                                  const double* __restrict__ v_prev,
                                                  double* __restrict__ v_next,
                                                  double* __restrict__ x,
                                                  double* __restrict__ Vcol, int j, int nflush) {
  extern __shared__ double lds[];
  EpiPass2 epi;
  p2_epi_ptrs(epi, v_cur, v_prev, v_next, x, Vcol, j, nflush);
  auto coefs = [&]() -> Scale {
    __builtin_amdgcn_sched_barrier(0);
    p2_epi_coefs(epi, S, j, nflush);
    return Scale{1.0, true};
  };
  const int b = blockIdx.x;
  TPL_MARK(0);
  if (b < A.n_comb) {
    push_combine(A, b, push_buf(A, j), coefs, epi);
    TPL_MARK(5);
    return;
  }
  double acc = 0.0;
  push_chunk_f<F>(A, b - A.n_comb, xsrc, coefs, epi, acc, lds, push_buf(A, j + 1));
  TPL_MARK(5);
}

// Partials of A x for the long rows (buffer `parity`); y != nullptr: also y = A x on
// the short rows (plain SpMV). x is both the gather source and the pushed values.
template <int F>
__global__ __launch_bounds__(kPushTPB) void k_push_spmv(CsrDev A, const double* __restrict__ x,
                                                    double* __restrict__ y, int parity) {
  extern __shared__ double lds[];
  TPL_MARK(0);
  double acc = 0.0;
  push_chunk_f<F>(A, blockIdx.x, x, UnitScale{}, EpiPushX{x, y}, acc, lds, push_buf(A, parity));
  TPL_MARK(5);
}

__global__ __launch_bounds__(kPushTPB) void k_push_comb_y(CsrDev A, double* __restrict__ y,
                                                      int parity) {
  push_combine(A, blockIdx.x, push_buf(A, parity), UnitScale{}, EpiSpmv{y});
}

// ------------------------------------------------------------------ launchers
namespace launch {

// products, then the long-run queue (count + 2 words per run)
static inline size_t push_lds_bytes(const CsrDev& A) {
  return (size_t)A.tp_cap * sizeof(double) + (size_t)(2 * A.n_long + 2) * sizeof(int);
}
#define TPL_PUSH_CASE(KERNEL, F) \
  case F: hipLaunchKernelGGL(KERNEL<F>, grid_, block_, shm_, s_, args_...); break
// F = width (1..4) | int8 values << 3 | uint16 columns << 4 | 4 rows per thread << 5
#define TPL_PUSH_LAUNCH(KERNEL, A, G, s, ...)                                                   \
  [&](auto... args_) {                                                                         \
    const dim3 grid_(G), block_(kPushTPB);                                                          \
    const size_t shm_ = push_lds_bytes(A);                                                      \
    hipStream_t s_ = (s);                                                                       \
    switch ((A).s_width | ((A).val_i8 ? 8 : 0) | ((A).s_col16 ? 16 : 0) |                       \
            ((A).push_rpt == 4 ? 32 : 0)) {                                                     \
      TPL_PUSH_CASE(KERNEL, 1); TPL_PUSH_CASE(KERNEL, 2); TPL_PUSH_CASE(KERNEL, 3); TPL_PUSH_CASE(KERNEL, 4);     \
      TPL_PUSH_CASE(KERNEL, 9); TPL_PUSH_CASE(KERNEL, 10); TPL_PUSH_CASE(KERNEL, 11); TPL_PUSH_CASE(KERNEL, 12); \
      TPL_PUSH_CASE(KERNEL, 17); TPL_PUSH_CASE(KERNEL, 18); TPL_PUSH_CASE(KERNEL, 19); TPL_PUSH_CASE(KERNEL, 20); \
      TPL_PUSH_CASE(KERNEL, 25); TPL_PUSH_CASE(KERNEL, 26); TPL_PUSH_CASE(KERNEL, 27); TPL_PUSH_CASE(KERNEL, 28); \
      TPL_PUSH_CASE(KERNEL, 33); TPL_PUSH_CASE(KERNEL, 34); TPL_PUSH_CASE(KERNEL, 35); TPL_PUSH_CASE(KERNEL, 36); \
      TPL_PUSH_CASE(KERNEL, 41); TPL_PUSH_CASE(KERNEL, 42); TPL_PUSH_CASE(KERNEL, 43); TPL_PUSH_CASE(KERNEL, 44); \
      TPL_PUSH_CASE(KERNEL, 49); TPL_PUSH_CASE(KERNEL, 50); TPL_PUSH_CASE(KERNEL, 51); TPL_PUSH_CASE(KERNEL, 52); \
      TPL_PUSH_CASE(KERNEL, 57); TPL_PUSH_CASE(KERNEL, 58); TPL_PUSH_CASE(KERNEL, 59); TPL_PUSH_CASE(KERNEL, 60); \
      default: return hipErrorInvalidConfiguration;                                             \
    }                                                                                           \
    return hipGetLastError();                                                                   \
  }(__VA_ARGS__)

hipError_t push_p1(const CsrDev& A, const DevState& S, const double* xsrc, const double* r_cur,
                   const double* r_prev, double* W, double* Vcol, int j, hipStream_t s) {
  const hipError_t e =
      TPL_PUSH_LAUNCH(k_push_p1, A, A.n_chunks, s, A, S, xsrc, r_cur, r_prev, W, Vcol, j);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_push_p1_comb, dim3(A.n_comb), dim3(kPushTPB), 0, s, A, S, r_cur, r_prev, W,
                     Vcol, j);
  return hipGetLastError();
}
hipError_t push_p2(const CsrDev& A, const DevState& S, const double* xsrc, const double* v_cur,
                   const double* v_prev, double* v_next, double* x, double* Vcol, int j,
                   int nflush, hipStream_t s) {
  return TPL_PUSH_LAUNCH(k_push_p2, A, A.n_comb + A.n_chunks, s, A, S, xsrc, v_cur, v_prev,
                         v_next, x, Vcol, j, nflush);
}
// partials of A x into buffer `parity`; y != nullptr: the whole product y = A x
hipError_t push_spmv(const CsrDev& A, const double* x, double* y, int parity, hipStream_t s) {
  const hipError_t e = TPL_PUSH_LAUNCH(k_push_spmv, A, A.n_chunks, s, A, x, y, parity);
  if (e != hipSuccess || !y) return e;
  hipLaunchKernelGGL(k_push_comb_y, dim3(A.n_comb), dim3(kPushTPB), 0, s, A, y, parity);
  return hipGetLastError();
}

} // namespace launch
} // namespace tpl

#if TPL_STAMP
// this translation unit's copy of the stamps (the push kernels write it)
extern "C" int tpl_debug_stamps_push(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tpl::g_stamps), sizeof(unsigned long long) * tpl::kMarks * n);
}
#endif
