// tpl_device.h — structures shared by the HIP kernels (tpl_kernels.hip) and the
// host runtime (tpl_runtime.cpp). Everything here is plain data: the kernels take
// these structs by value as kernel arguments.
//
// Canonical reduction order (the contract the CPU oracle reproduces bit for bit,
// oracle/lanczos_oracle.c; DESIGN.md "Reduction order"):
//   * tree256(a[256])  : per 64-lane wave an xor butterfly (offsets 32,16,8,4,2,1,
//                        a_l <- a_l + a_{l^off}), then (S0 + S1) + (S2 + S3).
//   * partials(P[G])   : thread t: s_t = 0; s_t += P[t + 256q] (q ascending); tree256.
//   * row sum          : STREAM item  -> s = 0; s += round(v_k x_k), k ascending
//                        WAVE item    -> lane l: s_l += round(v_k x_k), k = nz0+l+64q; butterfly64
//                        BLOCK item   -> thread t: k = nz0+t+256q; tree256
//   * alpha partial    : thread accumulators acc_t = fma(v_i, w_i, acc_t) over
//                        (items b, b+G, b+2G, ...) x (the rows that thread owns), then tree256
//                        (STREAM: row0+t+256q -> thread t; WAVE: row0+w -> thread 64w;
//                        BLOCK: -> thread 0)
//   * norm partial     : workgroup b owns [bE, min(n,(b+1)E)); thread t visits
//                        i0 = bE + 2t + 512q, then i0, i0+1: acc_t = fma(x,x,acc_t); tree256
#pragma once
#include <stdint.h>

namespace tpl {

constexpr int kTPB = 256;            // threads per workgroup (4 waves of 64)
constexpr int kStreamNnzCap = 2048;  // max nnz of one STREAM item (LDS product buffer)
constexpr int kStreamRowsCap = 1024; // max rows of one STREAM item (4 rows per thread)
constexpr int kWaveRowsPerItem = 4;  // one wave per row
constexpr double kBreakdownTol = 2.220446049250313080847263336181640625e-13; // 1000*f64::EPSILON, src/algorithms/mod.rs:140-143

enum ItemKind : int32_t { kItemStream = 0, kItemWave = 1, kItemBlock = 2 };

struct Item {
  int32_t row0, row1; // rows [row0, row1)
  int32_t nz0;        // row_ptr[row0]
  int32_t kind;       // ItemKind
};

// Device view of the CSR operator plus its schedule.
struct CsrDev {
  const int32_t* row_ptr; // n+1 (int32: nnz < 2^31)
  const int32_t* col;     // nnz
  const double* val;      // nnz
  const Item* items;      // n_items
  int32_t n_items;
  int32_t G;              // persistent workgroups of the SpMV kernels == #partials
  int64_t n;
  int64_t E;              // elements per workgroup of the element-wise kernels
};

// Device-resident solver state (one per operator).
struct DevState {
  int32_t* flags;   // [0] stop, [1] error (1 = zero b), [2] steps_taken
  double* norms;    // [0] = ||b||, [j] = beta_j                         (kcap+1)
  double* alphas;   // alphas[j-1] = alpha_j                              (kcap)
  double* betas;    // betas[j-1]  = beta_j                               (kcap)
  double* y;        // pass-two coefficients y_k (already * ||b||), or y' (kcap)
  double* Pa;       // alpha partials (G)
  double* Pb;       // ||.||^2 partials (G)
};

} // namespace tpl
