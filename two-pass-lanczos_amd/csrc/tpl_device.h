// tpl_device.h — structures shared by the HIP kernels (tpl_kernels.hip) and the
// host runtime (tpl_runtime.cpp). Everything here is plain data: the kernels take
// these structs by value as kernel arguments.
//
// SpMV layout (built once per operator, tpl_runtime.cpp build_layout):
//   * SHORT rows (<= kShortRowMax nnz), taken in ascending order, are stored as
//     sliced ELL: chunk c holds short-row positions [C*c, C*c + C) (C = kChunkRows);
//     entry k of position p sits at chunk_base[c] + k*C + (p - C*c) (column-major
//     inside the chunk, padded to the chunk's widest row with col = -1). One workgroup
//     per chunk, thread t owns positions C*c + t + 256q: every CSR load is coalesced
//     and no row pointer is chased. When every chunk has the same width and the
//     short rows are exactly rows 0..n_short-1 (the KKT arc block), chunk bases and
//     row indices are computed, not loaded.
//   * LONG rows are cut into kSlices column slices [n*s/8, n*(s+1)/8); a SLICE unit =
//     (group g of 16 long rows, slice s): wave w walks rows 16g + w + 4i (i = 0..3),
//     handled by workgroup n_chunks + 8g + s of the SpMV grid (chunks first) — under
//     the observed round-robin dispatch each XCD's L2 then only caches 1/8 of the
//     gathered vector (speed only, never correctness). Each unit publishes its 4 partials write-through (sc1) and bumps
//     the group's counter; the 8th arriver sums the partials and runs the long rows'
//     epilogue (split-K "last arriver" hand-off, cdna_hip_programming.md G16).
//
// Canonical reduction order (reproduced bit for bit by oracle/lanczos_oracle.c):
//   * tree256(a[256])  : per 64-lane wave an xor butterfly (offsets 32,16,8,4,2,1,
//                        a_l <- a_l + a_{l^off}), then (S0 + S1) + (S2 + S3).
//   * partials(P[N])   : thread t: s_t = 0; s_t += P[t + 256q] (q ascending); tree256.
//   * short row        : s = 0; s += round(a_k x_k), k ascending.
//   * long row         : per slice s: lane l: p_l = 0; p_l += round(a_k x_k) for
//                        k = off[s] + l + 64q; P[s] = butterfly64(p); y = 0; y += P[s], s = 0..7.
//   * alpha partial    : SHORT chunk c -> Pa[c]: thread t: acc = fma(v, w, acc) over its
//                        positions kChunkRows*c + t + 256q (q ascending), tree256;
//                        long group g -> Pa[n_chunks + g]: thread 64w: acc = fma(v, w, acc)
//                        over long rows 16g + w + 4i (i = 0..3), all others 0, tree256.
//   * norm partial     : workgroup b (of G2) owns [bE, min(n,(b+1)E)); thread t visits
//                        i0 = bE + 2t + 512q, then i0, i0+1: acc = fma(x,x,acc); tree256.
#pragma once
#include <stdint.h>

namespace tpl {

constexpr int kTPB = 256;            // threads per workgroup (4 waves of 64)
#ifndef TPL_CHUNK_ROWS
#define TPL_CHUNK_ROWS 256
#endif
constexpr int kChunkRows = TPL_CHUNK_ROWS; // short-row positions per SELL chunk
constexpr int kRowsPerThread = kChunkRows / kTPB;
constexpr int kShortRowMax = 32;     // rows with more nnz are "long" (sliced)
constexpr int kSlices = 8;           // column slices of a long row (= XCDs)
#ifndef TPL_LONG_ROWS_PER_WAVE
#define TPL_LONG_ROWS_PER_WAVE 4
#endif
constexpr int kLongRowsPerWave = TPL_LONG_ROWS_PER_WAVE;  // long rows a wave walks in turn
constexpr int kLongRowsPerGroup = 4 * kLongRowsPerWave;    // long rows per slice unit
constexpr double kBreakdownTol = 2.220446049250313080847263336181640625e-13; // 1000*f64::EPSILON, src/algorithms/mod.rs:140-143

// Device view of the operator plus its layout.
struct CsrDev {
  // long rows: CSR (global arrays, only long rows' entries are read)
  const int32_t* row_ptr;   // n+1 (int32: nnz < 2^31)
  const int32_t* col;       // nnz
  const double* val;        // nnz
  const int32_t* lrows;     // n_long long-row indices (ascending)
  const int32_t* loff;      // n_long x (kSlices+1) slice offsets into col/val
  double* P;                // n_long x kSlices slice partials (sc1 hand-off)
  int32_t* cnt;             // n_groups arrival counters (zero between launches)
  // short rows: sliced ELL
  const int32_t* srows;     // n_short short-row indices (ascending); unused if s_identity
  const int32_t* s_col;     // padded entries (col = -1 for padding)
  const double* s_val;
  const int32_t* c_base;    // n_chunks chunk base offsets; unused if s_width > 0
  const int32_t* c_width;   // n_chunks chunk widths; unused if s_width > 0
  int32_t s_width;          // > 0: every chunk has this width (bases computed)
  int32_t s_identity;       // 1: short rows are exactly 0 .. n_short-1
  int32_t n_short;
  int32_t n_chunks;
  int32_t n_long;
  int32_t n_groups;         // ceil(n_long / kLongRowsPerGroup)
  int32_t n_slice_blocks;   // kSlices * n_groups; SpMV grid = n_chunks + n_slice_blocks
  int32_t G2;               // workgroups of the element-wise kernels == #norm partials
  int32_t NA;               // #alpha partials = n_chunks + n_groups
  int32_t pad;
  int64_t n;
  int64_t E;                // elements per workgroup of the element-wise kernels
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
