// tpl_kernels.hip — CDNA4 (gfx950) kernels of the two-pass Lanczos engine.
//
// One Lanczos step of the reference (src/algorithms/mod.rs:167-212 + :292-340)
//     w = A v_j ; w -= beta_{j-1} v_{j-1} ; alpha_j = v_j . w ; w -= alpha_j v_j ;
//     beta_j = ||w|| ; v_{j+1} = w * (1/beta_j)
// has two grid-wide dependencies (alpha before the second AXPY, beta before the
// next SpMV), so pass one runs as two launches per step:
//   k_p1_spmv  : [reduce beta partials -> beta_{j-1}, breakdown test]
//                fused SpMV gathering x = r_j * (1/beta_{j-1})  (the normalisation
//                v_j = w/beta folded into the gather, bit-identical to storing v_j)
//                epilogue w = y - beta_{j-1} v_{j-1}; alpha partials (v_j . w)
//   k_p1_axpy  : [reduce alpha partials -> alpha_j]  r_{j+1} = w - alpha_j v_j ;
//                ||r_{j+1}||^2 partials
// Pass two (src/algorithms/lanczos_two_pass.rs:176-312) knows every coefficient,
// so each step is ONE launch (k_p2_spmv): SpMV + both AXPYs + scale + x += y v.
//
// Arithmetic follows the reference op by op (-ffp-contract=off for this file):
//   sub(w, mul(beta, v)) -> w - beta*v (two roundings), v = w * (1/beta)
//   (reciprocal then multiply), x = x + y*v. Reductions use a FIXED tree
//   (tpl_device.h) so results are run-to-run bitwise reproducible and pass two
//   regenerates pass one's basis bit for bit (reference: basis_drift_fro = 0.0,
//   results/orthogonality_*.csv).
#include <hip/hip_runtime.h>
#include "tpl_device.h"

namespace tpl {

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
  // xor butterfly: every lane ends with the same, order-fixed value.
  v = v + __shfl_xor(v, 32);
  v = v + __shfl_xor(v, 16);
  v = v + __shfl_xor(v, 8);
  v = v + __shfl_xor(v, 4);
  v = v + __shfl_xor(v, 2);
  v = v + __shfl_xor(v, 1);
  return v;
}

// tree256; every thread returns the block total. red: 4 doubles of LDS.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ double reduce_partials(const double* __restrict__ P, int G,
                                                  double* red) {
  double s = 0.0;
  for (int i = threadIdx.x; i < G; i += kTPB) s = s + P[i];
  return block_sum(s, red);
}

// --------------------------------------------------------------- SpMV core
// Walks the item list of workgroup blockIdx.x (items b, b+G, ...) and calls
// epi(row, rowsum, acc) once per row, on the thread the canonical order assigns.
template <class Epi>
__device__ __forceinline__ void spmv_items(const CsrDev& A, const double* __restrict__ xsrc,
                                           const double xscale, double* prod, double* red,
                                           double& acc, const Epi& epi) {
  const int t = threadIdx.x;
  for (int it = blockIdx.x; it < A.n_items; it += A.G) {
    const Item item = A.items[it];
    if (item.kind == kItemStream) {
      const int nz0 = item.nz0;
      const int cnt = A.row_ptr[item.row1] - nz0;
      // Phase 1: coalesced sweep of the item's nnz; gather x; products -> LDS.
#pragma unroll
      for (int u = 0; u < kStreamNnzCap / kTPB; ++u) {
        const int q = t + u * kTPB;
        if (q < cnt) {
          const int c = A.col[nz0 + q];
          const double a = A.val[nz0 + q];
          prod[q] = a * (xsrc[c] * xscale);
        }
      }
      __syncthreads();
      // Phase 2: one thread per row, ascending-column sequential sum.
      for (int i = item.row0 + t; i < item.row1; i += kTPB) {
        const int b = A.row_ptr[i] - nz0, e = A.row_ptr[i + 1] - nz0;
        double s = 0.0;
        for (int q = b; q < e; ++q) s = s + prod[q];
        epi(i, s, acc);
      }
      __syncthreads(); // LDS reuse by the next item
    } else if (item.kind == kItemWave) {
      const int w = t >> 6, lane = t & 63;
      const int i = item.row0 + w;
      double s = 0.0;
      if (i < item.row1) {
        const int e = A.row_ptr[i + 1];
        int q = A.row_ptr[i] + lane;
        // 4 independent gathers in flight per lane; adds stay in canonical order.
        for (; q + 192 < e; q += 256) {
          const int c0 = A.col[q], c1 = A.col[q + 64], c2 = A.col[q + 128], c3 = A.col[q + 192];
          const double a0 = A.val[q], a1 = A.val[q + 64], a2 = A.val[q + 128], a3 = A.val[q + 192];
          const double p0 = a0 * (xsrc[c0] * xscale), p1 = a1 * (xsrc[c1] * xscale);
          const double p2 = a2 * (xsrc[c2] * xscale), p3 = a3 * (xsrc[c3] * xscale);
          s = s + p0;
          s = s + p1;
          s = s + p2;
          s = s + p3;
        }
        for (; q < e; q += 64) s = s + A.val[q] * (xsrc[A.col[q]] * xscale);
      }
      s = wave_sum(s);
      if (i < item.row1 && lane == 0) epi(i, s, acc);
    } else { // kItemBlock: one workgroup per row
      const int i = item.row0;
      const int e = A.row_ptr[i + 1];
      double s = 0.0;
      int q = A.row_ptr[i] + t;
      for (; q + 3 * kTPB < e; q += 4 * kTPB) {
        const int c0 = A.col[q], c1 = A.col[q + kTPB], c2 = A.col[q + 2 * kTPB], c3 = A.col[q + 3 * kTPB];
        const double a0 = A.val[q], a1 = A.val[q + kTPB], a2 = A.val[q + 2 * kTPB], a3 = A.val[q + 3 * kTPB];
        const double p0 = a0 * (xsrc[c0] * xscale), p1 = a1 * (xsrc[c1] * xscale);
        const double p2 = a2 * (xsrc[c2] * xscale), p3 = a3 * (xsrc[c3] * xscale);
        s = s + p0;
        s = s + p1;
        s = s + p2;
        s = s + p3;
      }
      for (; q < e; q += kTPB) s = s + A.val[q] * (xsrc[A.col[q]] * xscale);
      s = block_sum(s, red);
      if (t == 0) epi(i, s, acc);
    }
  }
}

// ------------------------------------------------------------- epilogues
struct EpiSpmv {
  double* y;
  __device__ __forceinline__ void operator()(int i, double s, double&) const { y[i] = s; }
};

// pass one / standard: w = y - beta_{j-1} v_{j-1}; alpha partial v_j . w
struct EpiPass1 {
  const double* r_cur;  // r_j (v_j = r_j * invN_cur)
  const double* r_prev; // r_{j-1} or nullptr (j == 1: v_0 = 0)
  double invN_cur, invN_prev, beta_sub;
  double* W;
  double* Vcol;         // standard variant: column j-1 of V_k, else nullptr
  __device__ __forceinline__ void operator()(int i, double s, double& acc) const {
    const double v = r_cur[i] * invN_cur;
    const double vp = r_prev ? r_prev[i] * invN_prev : 0.0;
    const double w = s - beta_sub * vp;
    W[i] = w;
    if (Vcol) Vcol[i] = v;
    acc = fma(v, w, acc);
  }
};

// pass two: w = (y - beta_{j-1} v_{j-1}) - alpha_j v_j; v_{j+1} = w / beta_j; x += y_{j+1} v_{j+1}
struct EpiPass2 {
  const double* v_cur;
  const double* v_prev; // nullptr at j == 1
  double beta_sub, alpha, invb, ycoef;
  double* v_next;
  double* x;
  double* Vcol; // lanczos_pass_two_with_basis: column j of V'_k, else nullptr
  __device__ __forceinline__ void operator()(int i, double s, double&) const {
    const double vc = v_cur[i];
    const double vp = v_prev ? v_prev[i] : 0.0;
    double w = s - beta_sub * vp;
    w = w - alpha * vc;
    const double vn = w * invb;
    v_next[i] = vn;
    x[i] = x[i] + ycoef * vn;
    if (Vcol) Vcol[i] = vn;
  }
};

// ------------------------------------------------------------------ kernels
__global__ __launch_bounds__(kTPB) void k_spmv(CsrDev A, const double* __restrict__ x,
                                               double* __restrict__ y) {
  __shared__ double prod[kStreamNnzCap];
  __shared__ double red[4];
  double acc = 0.0;
  spmv_items(A, x, 1.0, prod, red, acc, EpiSpmv{y});
}

// Pass-one prologue: ||b||^2 partials, reset flags.
__global__ __launch_bounds__(kTPB) void k_p1_init(CsrDev A, DevState S,
                                                  const double* __restrict__ b) {
  __shared__ double red[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S.flags[0] = 0;
    S.flags[1] = 0;
    S.flags[2] = 0;
  }
  const int64_t beg = (int64_t)blockIdx.x * A.E;
  const int64_t end = beg + A.E < A.n ? beg + A.E : A.n;
  double acc = 0.0;
  for (int64_t i0 = beg + 2 * threadIdx.x; i0 < end; i0 += 2 * kTPB) {
    if (i0 + 1 < end) {
      const double2 v = *reinterpret_cast<const double2*>(b + i0);
      acc = fma(v.x, v.x, acc);
      acc = fma(v.y, v.y, acc);
    } else {
      const double v = b[i0];
      acc = fma(v, v, acc);
    }
  }
  const double p = block_sum(acc, red);
  if (threadIdx.x == 0) S.Pb[blockIdx.x] = p;
}

// Pass one / standard, step j >= 1. r_cur = r_j (== b at j = 1).
__global__ __launch_bounds__(kTPB) void k_p1_spmv(CsrDev A, DevState S,
                                                  const double* __restrict__ r_cur,
                                                  const double* __restrict__ r_prev,
                                                  double* __restrict__ W,
                                                  double* __restrict__ Vcol, int j) {
  __shared__ double prod[kStreamNnzCap];
  __shared__ double red[4];
  if (S.flags[0]) return; // stopped (breakdown / zero b) in an earlier launch
  const double beta = sqrt(reduce_partials(S.Pb, A.G, red)); // beta_{j-1} (||b|| at j = 1)
  if (beta <= kBreakdownTol) {
    // j == 1: zero b -> InputError (src/algorithms/mod.rs:267-273);
    // j  > 1: breakdown -> steps_taken = j - 1, beta not pushed (src/algorithms/lanczos_two_pass.rs:245-249).
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      S.flags[0] = 1;
      if (j == 1) S.flags[1] = 1;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S.norms[j - 1] = beta;
    if (j >= 2) S.betas[j - 2] = beta;
  }
  EpiPass1 epi;
  epi.r_cur = r_cur;
  epi.r_prev = (j >= 2) ? r_prev : nullptr;
  epi.invN_cur = 1.0 / beta;
  epi.invN_prev = (j >= 2) ? 1.0 / S.norms[j - 2] : 0.0;
  epi.beta_sub = (j >= 2) ? beta : 0.0;
  epi.W = W;
  epi.Vcol = Vcol;
  double acc = 0.0;
  spmv_items(A, r_cur, epi.invN_cur, prod, red, acc, epi);
  const double p = block_sum(acc, red);
  if (threadIdx.x == 0) S.Pa[blockIdx.x] = p;
}

// Pass one / standard, step j: alpha_j; r_{j+1} = w - alpha_j v_j; ||r_{j+1}||^2 partials.
__global__ __launch_bounds__(kTPB) void k_p1_axpy(CsrDev A, DevState S,
                                                  const double* __restrict__ W,
                                                  const double* __restrict__ r_cur,
                                                  double* __restrict__ r_next, int j, int k) {
  __shared__ double red[4];
  if (S.flags[0]) return;
  const double alpha = reduce_partials(S.Pa, A.G, red);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S.alphas[j - 1] = alpha;
    S.flags[2] = j;
  }
  if (j == k) return; // beta_k is never used (src/algorithms/lanczos_two_pass.rs:252-254)
  const double invN = 1.0 / S.norms[j - 1];
  const int64_t beg = (int64_t)blockIdx.x * A.E;
  const int64_t end = beg + A.E < A.n ? beg + A.E : A.n;
  double acc = 0.0;
  for (int64_t i0 = beg + 2 * threadIdx.x; i0 < end; i0 += 2 * kTPB) {
    if (i0 + 1 < end) {
      const double2 w = *reinterpret_cast<const double2*>(W + i0);
      const double2 rc = *reinterpret_cast<const double2*>(r_cur + i0);
      double2 r;
      r.x = w.x - alpha * (rc.x * invN);
      r.y = w.y - alpha * (rc.y * invN);
      *reinterpret_cast<double2*>(r_next + i0) = r;
      acc = fma(r.x, r.x, acc);
      acc = fma(r.y, r.y, acc);
    } else {
      const double r = W[i0] - alpha * (r_cur[i0] * invN);
      r_next[i0] = r;
      acc = fma(r, r, acc);
    }
  }
  const double p = block_sum(acc, red);
  if (threadIdx.x == 0) S.Pb[blockIdx.x] = p;
}

// Pass two prologue: v_1 = b * (1/||b||); x = v_1 * y_1 (src/algorithms/lanczos_two_pass.rs:248-252).
__global__ __launch_bounds__(kTPB) void k_p2_init(int64_t n, DevState S,
                                                  const double* __restrict__ b,
                                                  double* __restrict__ v1,
                                                  double* __restrict__ x,
                                                  double* __restrict__ Vcol) {
  const double invN = 1.0 / S.norms[0];
  const double y0 = S.y[0];
  for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kTPB) {
    const double v = b[i] * invN;
    v1[i] = v;
    x[i] = v * y0;
    if (Vcol) Vcol[i] = v;
  }
}

// Pass two, step j = 1 .. steps-1: regenerate v_{j+1}, accumulate x.
__global__ __launch_bounds__(kTPB) void k_p2_spmv(CsrDev A, DevState S,
                                                  const double* __restrict__ v_cur,
                                                  const double* __restrict__ v_prev,
                                                  double* __restrict__ v_next,
                                                  double* __restrict__ x,
                                                  double* __restrict__ Vcol, int j) {
  __shared__ double prod[kStreamNnzCap];
  __shared__ double red[4];
  EpiPass2 epi;
  epi.v_cur = v_cur;
  epi.v_prev = (j >= 2) ? v_prev : nullptr;
  epi.beta_sub = (j >= 2) ? S.betas[j - 2] : 0.0;
  epi.alpha = S.alphas[j - 1];
  epi.invb = 1.0 / S.betas[j - 1];
  epi.ycoef = S.y[j];
  epi.v_next = v_next;
  epi.x = x;
  epi.Vcol = Vcol;
  double acc = 0.0;
  spmv_items(A, v_cur, 1.0, prod, red, acc, epi);
}

// One-pass reconstruction x = ||b|| (V_k y') (src/solvers.rs:96-104); V column-major, ld = n.
__global__ __launch_bounds__(kTPB) void k_gemv_recon(int64_t n, int steps, DevState S,
                                                     const double* __restrict__ V,
                                                     double* __restrict__ x) {
  const double bnorm = S.norms[0];
  for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kTPB) {
    double s = 0.0;
    for (int c = 0; c < steps; ++c) s = fma(V[(int64_t)c * n + i], S.y[c], s);
    x[i] = bnorm * s;
  }
}

// ---------------------------------------------------- full re-orthogonalisation
// Extension with no reference counterpart (the reference's one-pass variant runs
// only the three-term recurrence, src/algorithms/mod.rs:167-212): classical
// Gram-Schmidt applied twice (CGS2) of r_{j+1} against V_k[:, 0..cols) before
// beta_j is formed. V is column-major (ld = n): lane i of a wave reads V[c*n + i],
// so every column sweep is a coalesced stream.
constexpr int kReorthCols = 8; // columns per workgroup in the h = V^T r kernel

// h partials: grid (G, ceil(cols/8)); workgroup (b, g) owns rows [bE, min(n,(b+1)E))
// and columns [8g, 8g+8). P[c*G + b] = tree256 of the thread accumulators.
__global__ __launch_bounds__(kTPB) void k_reorth_dot(int64_t n, int cols,
                                                     const double* __restrict__ V,
                                                     const double* __restrict__ r,
                                                     double* __restrict__ P, int G, int64_t E) {
  __shared__ double red[4];
  const int c0 = blockIdx.y * kReorthCols;
  const int nc = cols - c0 < kReorthCols ? cols - c0 : kReorthCols;
  const int64_t beg = (int64_t)blockIdx.x * E;
  const int64_t end = beg + E < n ? beg + E : n;
  double acc[kReorthCols];
#pragma unroll
  for (int u = 0; u < kReorthCols; ++u) acc[u] = 0.0;
  for (int64_t i = beg + threadIdx.x; i < end; i += kTPB) {
    const double ri = r[i];
#pragma unroll
    for (int u = 0; u < kReorthCols; ++u)
      if (u < nc) acc[u] = fma(V[(int64_t)(c0 + u) * n + i], ri, acc[u]);
  }
#pragma unroll
  for (int u = 0; u < kReorthCols; ++u) {
    const double s = block_sum(acc[u], red);
    if (u < nc && threadIdx.x == 0) P[(int64_t)(c0 + u) * G + blockIdx.x] = s;
  }
}

// h[c] = sum of the G partials of column c (one workgroup per column).
__global__ __launch_bounds__(kTPB) void k_reorth_reduce(const double* __restrict__ P, int G,
                                                        double* __restrict__ h) {
  __shared__ double red[4];
  const double s = reduce_partials(P + (int64_t)blockIdx.x * G, G, red);
  if (threadIdx.x == 0) h[blockIdx.x] = s;
}

// r -= V h ; optional ||r||^2 partials in the canonical norm order (E partition).
__global__ __launch_bounds__(kTPB) void k_reorth_update(int64_t n, int cols,
                                                        const double* __restrict__ V,
                                                        double* __restrict__ r,
                                                        const double* __restrict__ h,
                                                        double* __restrict__ Pnorm, int64_t E) {
  __shared__ double red[4];
  const int64_t beg = (int64_t)blockIdx.x * E;
  const int64_t end = beg + E < n ? beg + E : n;
  double acc = 0.0;
  for (int64_t i0 = beg + 2 * threadIdx.x; i0 < end; i0 += 2 * kTPB) {
    for (int e = 0; e < 2; ++e) {
      const int64_t i = i0 + e;
      if (i < end) {
        double s = 0.0;
        for (int c = 0; c < cols; ++c) s = fma(V[(int64_t)c * n + i], h[c], s);
        const double ri = r[i] - s;
        r[i] = ri;
        acc = fma(ri, ri, acc);
      }
    }
  }
  if (Pnorm) {
    const double p = block_sum(acc, red);
    if (threadIdx.x == 0) Pnorm[blockIdx.x] = p;
  }
}

} // namespace tpl

// ------------------------------------------------------------ host launchers
namespace tpl {
namespace launch {

static inline int elem_grid(int64_t n) {
  int64_t g = (n + kTPB - 1) / kTPB;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

hipError_t spmv(const CsrDev& A, const double* x, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_spmv, dim3(A.G), dim3(kTPB), 0, s, A, x, y);
  return hipGetLastError();
}
hipError_t p1_init(const CsrDev& A, const DevState& S, const double* b, hipStream_t s) {
  hipLaunchKernelGGL(k_p1_init, dim3(A.G), dim3(kTPB), 0, s, A, S, b);
  return hipGetLastError();
}
hipError_t p1_spmv(const CsrDev& A, const DevState& S, const double* r_cur, const double* r_prev,
                   double* W, double* Vcol, int j, hipStream_t s) {
  hipLaunchKernelGGL(k_p1_spmv, dim3(A.G), dim3(kTPB), 0, s, A, S, r_cur, r_prev, W, Vcol, j);
  return hipGetLastError();
}
hipError_t p1_axpy(const CsrDev& A, const DevState& S, const double* W, const double* r_cur,
                   double* r_next, int j, int k, hipStream_t s) {
  hipLaunchKernelGGL(k_p1_axpy, dim3(A.G), dim3(kTPB), 0, s, A, S, W, r_cur, r_next, j, k);
  return hipGetLastError();
}
hipError_t p2_init(int64_t n, const DevState& S, const double* b, double* v1, double* x,
                   double* Vcol, hipStream_t s) {
  hipLaunchKernelGGL(k_p2_init, dim3(elem_grid(n)), dim3(kTPB), 0, s, n, S, b, v1, x, Vcol);
  return hipGetLastError();
}
hipError_t p2_spmv(const CsrDev& A, const DevState& S, const double* v_cur, const double* v_prev,
                   double* v_next, double* x, double* Vcol, int j, hipStream_t s) {
  hipLaunchKernelGGL(k_p2_spmv, dim3(A.G), dim3(kTPB), 0, s, A, S, v_cur, v_prev, v_next, x,
                     Vcol, j);
  return hipGetLastError();
}
hipError_t gemv_recon(int64_t n, int steps, const DevState& S, const double* V, double* x,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_gemv_recon, dim3(elem_grid(n)), dim3(kTPB), 0, s, n, steps, S, V, x);
  return hipGetLastError();
}
hipError_t reorth_dot(int64_t n, int cols, const double* V, const double* r, double* P, int G,
                      int64_t E, hipStream_t s) {
  dim3 grid(G, (cols + kReorthCols - 1) / kReorthCols);
  hipLaunchKernelGGL(k_reorth_dot, grid, dim3(kTPB), 0, s, n, cols, V, r, P, G, E);
  return hipGetLastError();
}
hipError_t reorth_reduce(int cols, const double* P, int G, double* h, hipStream_t s) {
  hipLaunchKernelGGL(k_reorth_reduce, dim3(cols), dim3(kTPB), 0, s, P, G, h);
  return hipGetLastError();
}
hipError_t reorth_update(int64_t n, int cols, const double* V, double* r, const double* h,
                         double* Pnorm, int G, int64_t E, hipStream_t s) {
  hipLaunchKernelGGL(k_reorth_update, dim3(G), dim3(kTPB), 0, s, n, cols, V, r, h, Pnorm, E);
  return hipGetLastError();
}

} // namespace launch
} // namespace tpl
