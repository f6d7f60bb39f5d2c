// tpl_kcommon.h — device building blocks of the kernels (tpl_kernels.hip): DPP
// reductions, epilogues, the sliced-ELL chunk and the long-row bin. Included only by
// .hip files.
#pragma once
#include <hip/hip_runtime.h>
#include "tpl_device.h"
#include "tpl_lab.h"  // diagnostic stamp hooks (empty in the product build)

namespace tpl {

// ---------------------------------------------------------------- reductions
// 64-bit lane exchange through a DPP pattern (two 32-bit moves).
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, kCtrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), kCtrl, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double swz_xor16_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)b, 0x401F);  // bitmode: xor 16 within 32
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x401F);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Sum over the 64 lanes of a wave (all lanes active), as the xor butterfly with
// offsets 1, 2, 4, 8, 16, 32: lane l <- a_l + a_{l^h}. Once a stage is done every
// group of 2h lanes holds one value, so any exchange pairing a group with its
// partner group gives the same bits (IEEE addition is commutative); that lets the
// stages run on DPP (quad_perm, half-row and row mirrors), one swizzle and a
// readlane instead of LDS permutes. Every lane returns the same, order-fixed value.
__device__ __forceinline__ double wave_sum(double v) {
  v = v + dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v = v + dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v = v + dpp_f64<0x141>(v);  // row_half_mirror: partner quad in the 8-lane group
  v = v + dpp_f64<0x140>(v);  // row_mirror: partner 8-lane group in the row
  v = v + swz_xor16_f64(v);   // xor 16
  return readlane_f64(v, 0) + readlane_f64(v, 32);
}

// Sum over each aligned group of 8 lanes (butterfly offsets 1, 2, 4), all on DPP.
__device__ __forceinline__ double group8_sum(double v) {
  v = v + dpp_f64<0xB1>(v);   // xor 1
  v = v + dpp_f64<0x4E>(v);   // xor 2
  v = v + dpp_f64<0x141>(v);  // partner quad in the 8-lane group
  return v;
}

// Sum over each aligned group of 16 lanes (butterfly offsets 1, 2, 4, 8), all on DPP.
__device__ __forceinline__ double group16_sum(double v) {
  v = v + dpp_f64<0xB1>(v);   // xor 1
  v = v + dpp_f64<0x4E>(v);   // xor 2
  v = v + dpp_f64<0x141>(v);  // partner quad in the 8-lane group
  v = v + dpp_f64<0x140>(v);  // partner 8-lane group in the 16-lane row
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

// block_sum for a kernel's last reduction, whose total only thread 0 stores: the same
// bits, without the trailing barrier (red is not reused), so waves 1-3 retire at once.
__device__ __forceinline__ double block_sum_tail(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// Issue the partial loads (independent) early ...
template <int R>
struct PartialRegs {
  double v[R];
};
// (Every load below is unconditional with a clamped index and its result masked
// afterwards: a load under a runtime condition makes hipcc branch around it and
// drain vmcnt per element, serialising the round trips — guide §5 trap (c).)
__device__ __forceinline__ int clampi(int i, int hi) { return i < hi ? i : hi; }
template <int R>
__device__ __forceinline__ void load_partials(const double* __restrict__ P, int N,
                                              PartialRegs<R>& r) {
#pragma unroll
  for (int u = 0; u < R; ++u) r.v[u] = P[clampi(threadIdx.x + u * kTPB, N - 1)];
}
// ... and reduce them later in the canonical order (s = 0; s += P[t + 256q]).
template <int R>
__device__ __forceinline__ double finish_partials(const double* __restrict__ P, int N,
                                                  const PartialRegs<R>& r, double* red) {
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < R; ++u)
    if ((int)threadIdx.x + u * kTPB < N) s = s + r.v[u];
  // N > 256 R (the 5M-arc instance: ~13k alpha partials): the rest in batches of 8
  // loads in flight, added in the same ascending order (a plain loop waits for each
  // load before the next is issued: one round trip per 256 partials)
  for (int i0 = threadIdx.x + R * kTPB; i0 - (int)threadIdx.x < N; i0 += 8 * kTPB) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = P[clampi(i0 + u * kTPB, N - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u * kTPB < N) s = s + t[u];
  }
  return block_sum(s, red);
}

// Vector results of a step (w, v_{j+1}, x) are consumed only by the NEXT launch. Stored
// write-through (agent-scope relaxed stores: global_store ... sc1) they leave the XCD's L2
// while the kernel runs, instead of as dirty lines written back at the kernel boundary
// (MI355X_MICROARCH.md "boundary": + dirty bytes / 6 TB/s). Measured against plain and
// non-temporal stores for each of w, v_{j+1} and x (r02-r03, variant builds, same box,
// alternated): write-through kept for all three. r_{j+1} (k_p1_axpy)
// is the exception: 16-B non-temporal stores.
__device__ __forceinline__ void st_out(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Live timing (tpl_op_step_samples): workgroup 0 records the launch's start on the
// chip's 100 MHz real-time clock (a vector store; stamp is nullptr except in the sampled
// launches of a timed solve).
__device__ __forceinline__ void launch_stamp(unsigned long long* stamp) {
  if (stamp && blockIdx.x == 0 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();
}

// Pins a value as computed unconditionally: without it the compiler sinks the loads
// feeding a product used under a select (padding entries) into a branch, where they
// issue late behind an s_waitcnt vmcnt(0) and serialise the workgroup's round trips.
__device__ __forceinline__ void keep(double& v) { asm volatile("" : "+v"(v)); }

// ----------------------------------------------------------- epilogues
// pre(i) loads the row's own vector entries (issued early); apply(i, s, pre, acc)
// finishes the row given its SpMV sum s (acc: the thread's alpha accumulator).
struct PreNone {};
struct EpiSpmv {
  double* y;
  __device__ __forceinline__ PreNone pre(int) const { return {}; }
  __device__ __forceinline__ double apply(int i, double s, const PreNone&, double&) const {
    st_out(y + i, s);
    return s;
  }
  __device__ __forceinline__ void long_alpha(int, double) const {}
};

// pass one / standard: w = y - beta_{j-1} v_{j-1}; alpha partial += v_j . w
struct Pre1 {
  double rc, rp;
};
struct EpiPass1 {
  const double* r_cur;  // r_j (v_j = r_j * invN_cur)
  const double* r_prev; // r_{j-1}; == r_cur (never used) at j == 1 where v_0 = 0
  bool has_prev;
  double invN_cur, invN_prev, beta_sub;
  double* W;
  double* Vcol;         // standard variant: column j-1 of V_k, else nullptr
  double* Pa_long;      // alpha partials of the long rows (Pa + n_chunks)
  __device__ __forceinline__ Pre1 pre(int i) const { return Pre1{r_cur[i], r_prev[i]}; }
  // long row r: its alpha partial is the single rounded product v * w
  __device__ __forceinline__ void long_alpha(int r, double acc) const { st_out(Pa_long + r, acc); }
  // returns v_j[i]
  __device__ __forceinline__ double apply(int i, double s, const Pre1& p, double& acc) const {
    const double v = p.rc * invN_cur;
    const double vp = has_prev ? p.rp * invN_prev : 0.0;
    const double w = s - beta_sub * vp;
    st_out(W + i, w);
    if (Vcol) Vcol[i] = v;
    acc = fma(v, w, acc);
    return v;
  }
};

// pass two: w = (y - beta_{j-1} v_{j-1}) - alpha_j v_j; v_{j+1} = w / beta_j; x += y_j v_{j+1}.
// The x updates are applied in groups: a step with nflush = m adds the last m terms
// (y_{j-2} v_{j-1}, y_{j-1} v_j, y_j v_{j+1}: all three are in registers) one after the
// other, exactly as m separate steps would round them; nflush = 0 leaves x untouched.
// The host flushes every third step and at the last one, so x is read and written once
// per three steps instead of every step.
// The step's coefficients come in a record (DevState::p2c, written by k_p2_coefs
// before the steps): record j = {beta_{j-1} (0 at j = 1), alpha_j, 1/beta_j, y_j, y_{j-1},
// y_{j-2}, active, 0}. Lane l loads field l & 7 together with its row's own vector entries,
// i.e. after the gathers, and the epilogue reads the fields with readlane. The unit gather
// scale is known at entry, so the products, the LDS piece sums and the long rows' hand-off
// never wait for the coefficients (with scalar coefficient loads, every workgroup waited
// for a miss to the fabric before its first product: MI355X L2s drop lines other XCDs wrote
// at each kernel start). Bitwise the same operations as EpiPass2 (1/beta_j is the same IEEE
// division, made once per step by k_p2_coefs). active = 0: a one-graph solve's launch at or
// past steps_taken — the SpMV still runs (the arrival counters stay balanced), the
// epilogue stores nothing.
struct Pre2R {
  double vc, vp, x, cv;
};
struct EpiPass2R {
  const double* v_cur;
  const double* v_prev; // == v_cur (never used) at j == 1 where v_0 = 0
  const double* rec;    // this step's coefficient record (8 doubles)
  bool has_prev;
  int nflush;           // 0..3 x terms applied by this step
  double* v_next;
  double* x;
  double* Vcol;
  __device__ __forceinline__ Pre2R pre(int i) const {
    return Pre2R{v_cur[i], v_prev[i], nflush ? x[i] : 0.0, rec[threadIdx.x & 7]};
  }
  __device__ __forceinline__ double apply(int i, double s, const Pre2R& p, double&) const {
    if (readlane_f64(p.cv, 6) == 0.0) return 0.0;  // inactive launch (uniform)
    const double beta_sub = readlane_f64(p.cv, 0), alpha = readlane_f64(p.cv, 1);
    const double invb = readlane_f64(p.cv, 2), ycoef = readlane_f64(p.cv, 3);
    const double vp = has_prev ? p.vp : 0.0;
    double w = s - beta_sub * vp;
    w = w - alpha * p.vc;
    const double vn = w * invb;
    st_out(v_next + i, vn);
    if (nflush) {
      double xv = p.x;
      if (nflush >= 3) xv = xv + readlane_f64(p.cv, 5) * p.vp;
      if (nflush >= 2) xv = xv + readlane_f64(p.cv, 4) * p.vc;
      st_out(x + i, xv + ycoef * vn);
    }
    if (Vcol) Vcol[i] = vn;
    return vn;
  }
  __device__ __forceinline__ void long_alpha(int, double) const {}
};

// Kernel-argument fields both paths of an SpMV-shaped kernel read, pinned in SGPRs at
// entry: all kernel-argument loads then share ONE scalar round trip, instead of a second
// one behind the first branch (hipcc sinks a load into the branch that uses it).
__device__ __forceinline__ void pin_layout_args(const CsrDev& A) {
  asm volatile("" ::"s"(A.s_col), "s"(A.s_val), "s"(A.s_cbase), "s"(A.b_col), "s"(A.b_val),
               "s"(A.b_seg), "s"(A.b_hdr), "s"(A.b_cbase));
  asm volatile("" ::"s"(A.n_short), "s"(A.n_slice_blocks), "s"(A.n_slices), "s"(A.bin_cap),
               "s"(A.s_identity), "s"(A.n_chunks));
}

// keep() for a row's epilogue inputs (used only for live rows / finalising threads)
__device__ __forceinline__ void keep_pre(PreNone&) {}
__device__ __forceinline__ void keep_pre(Pre1& p) { keep(p.rc); keep(p.rp); }
__device__ __forceinline__ void keep_pre(Pre2R& p) { keep(p.vc); keep(p.vp); keep(p.x); keep(p.cv); }

// Result of a workgroup's prologue: the gather scale, or "stop" (uniform across the grid).
struct Scale {
  double s;
  bool ok;
};
struct UnitScale {
  __device__ __forceinline__ Scale operator()() const { return Scale{1.0, true}; }
};

// Matrix values: fp64, or int8 when every value is a small integer (V8 = 1; the
// conversion to double is exact, so products and sums are bit-identical).
template <int V8>
__device__ __forceinline__ double val_at(const void* p, int i) {
  if (V8) return (double)reinterpret_cast<const int8_t*>(p)[i];
  return reinterpret_cast<const double*>(p)[i];
}

// Column indices: int32 (padding -1), or — C16 — uint16 offsets from a per-chunk /
// per-bin base (padding 0xFFFF) when every chunk / bin spans fewer than 65535 columns.
template <int C16>
__device__ __forceinline__ int col_at(const void* p, int i, int base) {
  if (C16) {
    const int off = reinterpret_cast<const uint16_t*>(p)[i];
    return off == 0xFFFF ? -1 : base + off;
  }
  return reinterpret_cast<const int32_t*>(p)[i];
}

// A thread's run of N consecutive stored entries (tpl_device.h kPackedEntries), read
// with the widest loads its bytes allow (16 / 8 / 4 / 2 B per load).
template <int N, class T>
__device__ __forceinline__ void load_run(const T* __restrict__ p, T (&out)[N]) {
  constexpr int B = N * (int)sizeof(T);
  if constexpr (B >= 16) {
    static_assert(B % 16 == 0, "whole 16-B loads");
#pragma unroll
    for (int i = 0; i < B / 16; ++i) {
      const uint4 q = reinterpret_cast<const uint4*>(p)[i];
      __builtin_memcpy(reinterpret_cast<char*>(out) + 16 * i, &q, 16);
    }
  } else if constexpr (B == 8) {
    const uint2 q = *reinterpret_cast<const uint2*>(p);
    __builtin_memcpy(out, &q, 8);
  } else if constexpr (B == 4) {
    const unsigned int q = *reinterpret_cast<const unsigned int*>(p);
    __builtin_memcpy(out, &q, 4);
  } else {
    static_assert(B == 2, "2-B run");
    const unsigned short q = *reinterpret_cast<const unsigned short*>(p);
    __builtin_memcpy(out, &q, 2);
  }
}
template <int C16> struct ColType { typedef int32_t T; };
template <> struct ColType<1> { typedef uint16_t T; };
template <int V8> struct ValType { typedef double T; };
template <> struct ValType<1> { typedef int8_t T; };
// Entries [e0, e0 + N) of a packed run: columns (-1: padding) and values.
template <int N, int V8, int C16>
__device__ __forceinline__ void load_entry_run(const void* colp, const void* valp, int e0, int cbase,
                                               int (&c)[N], double (&a)[N]) {
  typename ColType<C16>::T cr[N];
  typename ValType<V8>::T vr[N];
  load_run<N>(reinterpret_cast<const typename ColType<C16>::T*>(colp) + e0, cr);
  load_run<N>(reinterpret_cast<const typename ValType<V8>::T*>(valp) + e0, vr);
#pragma unroll
  for (int u = 0; u < N; ++u) {
    if (C16) c[u] = cr[u] == 0xFFFF ? -1 : cbase + (int)cr[u];
    else c[u] = (int)cr[u];
    a[u] = (double)vr[u];
  }
}

// ------------------------------------------------------ short rows (sliced ELL)
// Chunk with a compile-time width W (entries loaded unconditionally: the sliced-ELL
// storage is allocated for whole chunks, padding has col = -1).
// PK: the entries are stored in the packed device order (tpl_device.h packed_chunk_width).
template <int W, int V8, int C16, int WIN, bool PK, class Epi, class ScaleFn>
__device__ __forceinline__ bool short_chunk_w(const CsrDev& A, int chunk, int base,
                                              const double* __restrict__ xsrc, ScaleFn scale_of,
                                              const Epi& epi, double& acc, double* lds) {
  const int t = threadIdx.x;
  const int cbase = C16 ? A.s_cbase[chunk] : 0;
  // WIN: the chunk's column window [cbase, cbase + s_win) is loaded coalesced into LDS
  // (issued first, in parallel with the entries) and gathered from there: the KKT arc
  // rows' columns all lie in the 1,155 node columns, so ~1 M divergent L1 gathers per
  // SpMV become LDS reads and the chunk's chain shrinks to one memory round trip.
  double wv[WIN ? kWinLoads : 1];
  if (WIN) {
#pragma unroll
    for (int u = 0; u < kWinLoads; ++u) {
      const int k = t + u * kTPB;
      wv[u] = xsrc[cbase + k < A.s_win_max ? cbase + k : A.s_win_max];
    }
  }
  int row[kRowsPerThread];
  bool live[kRowsPerThread];
  decltype(epi.pre(0)) pre[kRowsPerThread];
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) {
    const int p = chunk * kChunkRows + q * kTPB + t;
    live[q] = p < A.n_short;
    const int pc = clampi(p, A.n_short - 1);
    // the row-list load waited for inside its own branch: left pending into the join it
    // would make the identity path wait for every load in flight (the DevState loads
    // ahead of the entries included) before issuing its entries
    int r = pc;
    if (!A.s_identity) {
      r = A.srows[pc];
      asm volatile("" : "+v"(r));
    }
    row[q] = r;
  }
  // Issue order = arrival order: the entries first (the gathers wait on them), then
  // the row's own vector entries (needed only by the epilogue), then the gathers.
  int c[kRowsPerThread][W];
  double a[kRowsPerThread][W], xv[kRowsPerThread][W];
  if constexpr (PK) {  // packed: this thread's kRowsPerThread x W entries are consecutive
    int cr[kRowsPerThread * W];
    double ar[kRowsPerThread * W];
    load_entry_run<kRowsPerThread * W, V8, C16>(A.s_col, A.s_val, base + t * kRowsPerThread * W,
                                                 cbase, cr, ar);
#pragma unroll
    for (int q = 0; q < kRowsPerThread; ++q)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        c[q][k] = cr[q * W + k];
        a[q][k] = ar[q * W + k];
      }
  } else {
#pragma unroll
    for (int q = 0; q < kRowsPerThread; ++q)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int e = base + k * kChunkRows + q * kTPB + t;
        c[q][k] = col_at<C16>(A.s_col, e, cbase);
        a[q][k] = val_at<V8>(A.s_val, e);
      }
  }
  if (WIN) {
#pragma unroll
    for (int u = 0; u < kWinLoads; ++u)
      if (t + u * kTPB < A.s_win) lds[t + u * kTPB] = wv[u];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kRowsPerThread; ++q)
#pragma unroll
      for (int k = 0; k < W; ++k) xv[q][k] = lds[c[q][k] < 0 ? 0 : c[q][k] - cbase];
  } else {
#pragma unroll
    for (int q = 0; q < kRowsPerThread; ++q)
#pragma unroll
      for (int k = 0; k < W; ++k) xv[q][k] = xsrc[c[q][k] < 0 ? 0 : c[q][k]];
  }
  // the rows' own vector entries after the gathers: needed only by the epilogue, issued
  // first they delay the bins' critical loads
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) pre[q] = epi.pre(row[q]);
  const Scale sc = scale_of();
  TPL_MARK(1);
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) keep_pre(pre[q]);
  // The products before the stop test (uniform): kept (opaque) they pin the gathers ahead
  // of it — tested first, the compiler sinks the gathers into the branch and every
  // workgroup waits for the stop flag's load before it issues them.
  double sum[kRowsPerThread];
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) {
    sum[q] = 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      double prod = a[q][k] * (xv[q][k] * sc.s);
      keep(prod);
      sum[q] = sum[q] + (c[q][k] >= 0 ? prod : -0.0);  // padding adds -0.0: exact
    }
  }
  if (!sc.ok) return false; // stopped / breakdown (uniform)
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q)
    if (live[q]) epi.apply(row[q], sum[q], pre[q], acc);
  TPL_MARK(2);
  return true;
}

// Any width (rare: chunks wider than 4). One row position at a time, entries in
// batches of 8 with every load of a batch in flight; kept lean in registers, since a
// kernel's VGPR budget is the maximum over all of its paths.
template <int V8, int C16, class Epi, class ScaleFn>
__device__ __forceinline__ bool short_chunk_any(const CsrDev& A, int chunk, int base, int W,
                                                const double* __restrict__ xsrc, ScaleFn scale_of,
                                                const Epi& epi, double& acc) {
  const int t = threadIdx.x;
  const int cbase = C16 ? A.s_cbase[chunk] : 0;
  const Scale sc = scale_of();
  if (!sc.ok) return false;
#pragma unroll 1
  for (int q = 0; q < kRowsPerThread; ++q) {
    const int p = chunk * kChunkRows + q * kTPB + t;
    const bool live = p < A.n_short;
    const int pc = clampi(p, A.n_short - 1);
    const int row = A.s_identity ? pc : A.srows[pc];
    auto pre = epi.pre(row);
    double s = 0.0;
#pragma unroll 1
    for (int k0 = 0; k0 < W; k0 += 8) {
      int c[8];
      double a[8], xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = base + clampi(k0 + u, W - 1) * kChunkRows + q * kTPB + t;
        c[u] = col_at<C16>(A.s_col, e, cbase);
        a[u] = val_at<V8>(A.s_val, e);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = xsrc[c[u] < 0 ? 0 : c[u]];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        double prod = a[u] * (xv[u] * sc.s);
        keep(prod);
        s = s + ((c[u] >= 0 && k0 + u < W) ? prod : -0.0);  // padding adds -0.0: exact
      }
    }
    keep_pre(pre);
    if (live) epi.apply(row, s, pre, acc);
  }
  return true;
}

// CW > 0: the kernel was specialised for a uniform chunk width CW (tpl::launch picks
// it from A.s_width); CW == 0: generic, any per-chunk width.
template <int CW, int V8, int C16, int WIN, class Epi, class ScaleFn>
__device__ __forceinline__ bool short_chunk(const CsrDev& A, int chunk,
                                            const double* __restrict__ xsrc, ScaleFn scale_of,
                                            const Epi& epi, double& acc, double* lds) {
  if (CW > 0)
    return short_chunk_w<CW, V8, C16, (CW > 0 && C16) ? WIN : 0, packed_chunk_width(CW)>(
        A, chunk, chunk * kChunkRows * CW, xsrc, scale_of, epi, acc, lds);
  int W, base;
  if (A.s_width > 0) {
    W = A.s_width;
    base = chunk * kChunkRows * W;
  } else {
    W = A.c_width[chunk];
    base = A.c_base[chunk];
  }
  switch (W) {
    case 1: return short_chunk_w<1, V8, C16, 0, false>(A, chunk, base, xsrc, scale_of, epi, acc, lds);
    case 2: return short_chunk_w<2, V8, C16, 0, false>(A, chunk, base, xsrc, scale_of, epi, acc, lds);
    case 3: return short_chunk_w<3, V8, C16, 0, false>(A, chunk, base, xsrc, scale_of, epi, acc, lds);
    case 4: return short_chunk_w<4, V8, C16, 0, false>(A, chunk, base, xsrc, scale_of, epi, acc, lds);
    default: return short_chunk_any<V8, C16>(A, chunk, base, W, xsrc, scale_of, epi, acc);
  }
}

// ------------------------------------------------------ long rows (bins)
// Thread t's entries u = 0 .. kBinBatch-1 of the load batch at e0: positions e0 + 256u + t
// (stored at e0 + kBinBatch t + u when packed, tpl_device.h kPackedEntries).
template <int V8, int C16>
__device__ __forceinline__ void load_bin_batch(const CsrDev& A, int e0, int cbase, int (&c)[kBinBatch],
                                               double (&a)[kBinBatch]) {
  const int t = threadIdx.x;
  if constexpr (kPackedEntries) {
    load_entry_run<kBinBatch, V8, C16>(A.b_col, A.b_val, e0 + kBinBatch * t, cbase, c, a);
  } else {
#pragma unroll
    for (int u = 0; u < kBinBatch; ++u) {
      c[u] = col_at<C16>(A.b_col, e0 + u * kTPB + t, cbase);
      a[u] = val_at<V8>(A.b_val, e0 + u * kTPB + t);
    }
  }
}

// Bin m of slice s. Thread t loads entries t + 256u of the bin (coalesced, at
// computed addresses) and its bin-table slot; the products go to LDS; each piece is
// then summed by one wave (lane-strided + butterfly) and handed back to thread j,
// which owns piece j and publishes it; whoever completes a row's S slices finalises it
// (S = 1: the piece is the row, finished in place).
// lds: bin_cap doubles of products, kTPB ints of piece starts, kTPB piece sums.
template <int V8, int C16, class Epi, class ScaleFn>
__device__ __forceinline__ void long_bin(const CsrDev& A, int m, int s,
                                         const double* __restrict__ xsrc, ScaleFn scale_of,
                                         const Epi& epi, double* lds) {
  const int t = threadIdx.x;
  const int bin = __builtin_amdgcn_readfirstlane(m * A.n_slices + s);  // scalar loads below
  const int base = bin * A.bin_cap;
  const int cbase = C16 ? A.b_cbase[bin] : 0;
  const int hdr = A.b_hdr[bin];
  // Issue order: the entries first (the gathers wait on them), then the bin table
  // (its slot index waits on the header).
  int c[kBinBatch];
  double a[kBinBatch], xv[kBinBatch];
  load_bin_batch<V8, C16>(A, base, cbase, c, a);
  __builtin_amdgcn_sched_barrier(0);
  // only the slots up to the end marker are read (threads past it re-read the marker)
  const int npieces = hdr & 0xFFFF, nbig = hdr >> 16;
  const BinSeg sg = A.b_seg[bin * kTPB + (t < npieces ? t : npieces)];
#pragma unroll
  for (int u = 0; u < kBinBatch; ++u) xv[u] = xsrc[c[u] < 0 ? 0 : c[u]];
  // the finalising thread's own row entries travel with the gathers
  auto pre = epi.pre(sg.row < 0 ? 0 : sg.row);
  const Scale sc = scale_of();
  TPL_MARK(1);
  // padding slots (col = -1) are never summed (pieces cover real entries only), so the
  // product is stored unconditionally: a select here lets the compiler sink the loads
  // of that entry into a branch and serialise them behind everything else in flight.
  // The same holds for the stop test (uniform): after the LDS stores, which pin the
  // entries and gathers ahead of it.
#pragma unroll
  for (int u = 0; u < kBinBatch; ++u) lds[u * kTPB + t] = a[u] * (xv[u] * sc.s);
  if (!sc.ok) return; // stopped / breakdown: slots untouched
  for (int u0 = kBinBatch * kTPB; u0 < A.bin_cap; u0 += kBinBatch * kTPB) { // bins wider than one batch (rare)
    load_bin_batch<V8, C16>(A, base + u0, cbase, c, a);
#pragma unroll
    for (int u = 0; u < kBinBatch; ++u) xv[u] = xsrc[c[u] < 0 ? 0 : c[u]];
#pragma unroll
    for (int u = 0; u < kBinBatch; ++u)
      lds[u0 + u * kTPB + t] = a[u] * (xv[u] * sc.s);
  }
  int* starts = reinterpret_cast<int*>(lds + A.bin_cap);
  double* psum = lds + A.bin_cap + kTPB / 2;  // kTPB doubles after the starts
  starts[t] = sg.ri < 0 ? -1 - sg.start : sg.start;  // < 0: no piece (value encodes the fill)
  __syncthreads();
  TPL_MARK(2);
  // Entries past a piece's end add -0.0 instead of being skipped by a select after the
  // add: x + (-0.0) is x bit for bit for every x (signed zeros, infinities and NaNs
  // included), so the sums are unchanged and the select leaves the dependent add chain.
  // Piece sums (canonical long-row order). A piece longer than kBigPiece is summed by a
  // 16-lane group — lane g sums its entries g + 16q, then the 16-lane butterfly; those
  // pieces come first in the table (nbig of them). Any other piece is summed by an 8-lane
  // group — lane g sums its entries g + 8q, then the 8-lane butterfly. The work is dealt
  // to the 4 waves as wave tasks: big task i sums big pieces 4i .. 4i + 3 (four 16-lane
  // groups), small task i the other pieces nbig + 8i .. 8i + 7 (eight 8-lane groups); wave
  // w takes tasks w, w + 4, ... So a bin of, e.g., 9 long and 7 short pieces sums them
  // in ONE round (3 big tasks + 1 small task) where separate 16-lane and 8-lane rounds
  // took two — every extra round cost its bin ≈0.4 µs (round-5 stamps, scripts/lab/
  // bin_cost.py). Which wave sums a piece never enters its sum: the bits are unchanged.
  {
    const int lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int tb = (nbig + 3) >> 2, ts = (npieces - nbig + 7) >> 3;
    for (int task = wv; task < tb + ts; task += kTPB / 64) {  // wave-uniform
      if (task < tb) {
        const int g16 = lane & 15;
        const int j = 4 * task + (lane >> 4);
        const bool valid = j < nbig;
        const int jc = valid ? j : 0;
        const int st = starts[jc], nx = starts[jc + 1];
        const int b0 = valid ? st : 0;
        const int en = valid ? (nx >= 0 ? nx : -1 - nx) : 0;
        // this lane's entries k + 16q, q ascending: whole blocks of 8 first (8 reads in
        // flight, then 8 adds with no bounds test on the chain: the longest pieces run
        // tens of blocks), then the last 0..7 with the tests
        int k = b0 + g16;
        const int cnt = k < en ? (en - k + 15) >> 4 : 0;
        double acc = 0.0;
        for (int blk = cnt >> 3; blk > 0; --blk, k += 128) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = lds[k + 16 * u];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + v[u];
        }
        const int rem = cnt & 7;
        if (rem > 0) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = lds[u < rem ? k + 16 * u : k];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + (u < rem ? v[u] : -0.0);
        }
        acc = group16_sum(acc);
        if (g16 == 0 && valid) psum[j] = acc;
      } else {
        const int g8 = lane & 7;
        const int j = nbig + 8 * (task - tb) + (lane >> 3);
        const int jc = j < kTPB - 2 ? j : kTPB - 2;
        const int st = starts[jc], nx = starts[jc + 1];
        const bool valid = j < npieces;
        const int b0 = valid ? st : 0;
        const int en = valid ? (nx >= 0 ? nx : -1 - nx) : 0;
        double acc = 0.0;
        for (int k0 = b0 + g8; k0 < en; k0 += 64) {  // 8 reads in flight, then the adds
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = lds[k0 + 8 * u < en ? k0 + 8 * u : k0];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + (k0 + 8 * u < en ? v[u] : -0.0);
        }
        acc = group8_sum(acc);
        if (g8 == 0 && valid) psum[j] = acc;
      }
    }
  }
  TPL_MARK(7);
  TPL_MARK(8);
  __syncthreads();
  TPL_MARK(3);
  // the finalising thread's row entries, loaded with the gathers, waited on only now: the
  // piece sums' LDS stores and barriers keep their loads ahead, and the sums run while
  // they are in flight
  keep_pre(pre);
  if (sg.ri < 0) return; // no piece for this thread
  const double p = psum[t];
  const int ns = A.n_slices;
  // sg.pad = the row's packed pieces - 1 (only pieces with entries are packed; the
  // slots of the others are never written and hold +0.0). One piece: it is the whole row
  // (0 + p, then + 0.0 for the other slots, which changes no bit): no hand-off.
  if (ns == 1 || sg.pad == 0) {
    const double y = 0.0 + p;
    if (A.long_defer) {
      A.ypart[sg.ri] = y;
      return;
    }
    double acc = 0.0;
    epi.apply(sg.row, y, pre, acc);
    epi.long_alpha(sg.ri, acc);
    return;
  }
  // Hand-off (MI355X_MICROARCH.md, valid forms, first table row): publish the piece sum
  // write-through (sc1), drain this wave's stores, then ONE agent-scope atomic increment
  // of the row's arrival counter, wrapping at the row's piece count (atomic_inc: old >=
  // pad ? 0 : old + 1, so the counter runs on across launches); the publisher whose
  // increment returns pad (the row's last arrival) is the only one that reads the S slots
  // (sc1 loads, after its increment has returned) and finalises the row. The atomics of a
  // row are totally ordered at the memory side, so exactly one publisher per launch sees
  // the last count and every slot it reads was drained before the atomic that preceded
  // its own. No thread ever waits on another: nothing depends on dispatch order.
  unsigned long long* slots = reinterpret_cast<unsigned long long*>(A.P + (size_t)sg.ri * kSlotStride);
  __hip_atomic_store(slots + s, (unsigned long long)__double_as_longlong(p), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TPL_MARK(4);
  const unsigned int arrived = __builtin_amdgcn_atomic_inc32(
      A.Pcnt + (size_t)sg.ri * kCntStride, (unsigned)sg.pad, __ATOMIC_RELAXED, "agent");
  asm volatile("" ::: "memory");  // the slot loads stay behind the returned increment
  if (arrived != (unsigned)sg.pad) return;
  // 16-B sc1 loads of slot pairs (slot arrays are 64-B aligned): four instead of eight 8-B
  // loads (same box, alternated: k_p2_spmv -0.1 us, pass one -0.15 us per step). The four
  // loads and their wait are ONE asm statement: the compiler must not touch the destination
  // registers between the issue and the s_waitcnt (copying them early reads whatever they
  // held). Slots past the slice count re-read slot 0 (summed only up to ns).
  static_assert(kSlices == 8, "four slot pairs");
  unsigned long long v[kSlices];
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  u64x2 r0, r1, r2, r3;
  const unsigned long long* p0 = slots;
  const unsigned long long* p1 = slots + (2 < ns ? 2 : 0);
  const unsigned long long* p2 = slots + (4 < ns ? 4 : 0);
  const unsigned long long* p3 = slots + (6 < ns ? 6 : 0);
  asm volatile(
      "global_load_dwordx4 %0, %4, off sc1\n\t"
      "global_load_dwordx4 %1, %5, off sc1\n\t"
      "global_load_dwordx4 %2, %6, off sc1\n\t"
      "global_load_dwordx4 %3, %7, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(p0), "v"(p1), "v"(p2), "v"(p3)
      : "memory");
  v[0] = r0.x; v[1] = r0.y; v[2] = r1.x; v[3] = r1.y;
  v[4] = r2.x; v[5] = r2.y; v[6] = r3.x; v[7] = r3.y;
  double y = 0.0;
#pragma unroll
  for (int k = 0; k < kSlices; ++k)
    if (k < ns) y = y + __longlong_as_double((long long)v[k]);
  if (A.long_defer) {  // partitioned: this rank's part of the row; finished after the exchange
    A.ypart[sg.ri] = y;
    return;
  }
  double acc = 0.0;
  epi.apply(sg.row, y, pre, acc);
  epi.long_alpha(sg.ri, acc);
}

// XCD-contiguous placement (speed only; any bijection is correct). Workgroups are
// dealt round-robin to the 8 XCDs, block B on XCD B % 8 (observed on every launch:
// block 0 on XCD 0, scripts/lab/xcd_rr.hip), and an XCD's L2 keeps the lines a kernel
// wrote there for the next kernel (scripts/lab/l2_keep.hip: 32 MB re-read 7.4 us on
// the writing XCD vs 10.4 us elsewhere). Row block rb (A.E rows) therefore runs on XCD
// x for rb in [rb_first(x), rb_first(x + 1)) — contiguous eighths of the rows — in every
// kernel: the element-wise kernels (elem_block), the short chunks of the SpMV-shaped
// kernels (chunk_of_block: chunk c lies in row block c / (E / kChunkRows)), and, with
// 8 column slices, the bins of slice s (block 8m + s, on XCD s) gather exactly the
// eighth of the vector that XCD s's chunks and element-wise blocks read and write.
// Measured at 500k arcs (8 slices): k_p2_spmv 9.07 -> 8.55 us, solve 12.07 -> 11.70 ms
// against 2048-row blocks dealt round-robin.
__device__ __forceinline__ int rb_first(int G2, int x) { return (x * G2 + 7) >> 3; }
// element-wise grid (8 ceil(G2 / 8) blocks): block i -> row block, or -1 (padding)
__device__ __forceinline__ int elem_block(const CsrDev& A, int i) {
  const int x = i & 7, q = i >> 3;
  const int rb = rb_first(A.G2, x) + q;
  return rb < rb_first(A.G2, x + 1) ? rb : -1;
}
// chunk part of an SpMV grid: block i of the part -> short chunk, or -1 (padding)
__device__ __forceinline__ int chunk_of_block(const CsrDev& A, int i) {
  const int cpe = (int)(A.E / kChunkRows);  // chunks per row block
  const int x = (i + A.n_slice_blocks) & 7, q = i >> 3;
  const int c = rb_first(A.G2, x) * cpe + q;
  return (c < rb_first(A.G2, x + 1) * cpe && c < A.n_chunks) ? c : -1;
}

// Minimum waves per SIMD requested for the SpMV-shaped kernels (occupancy vs VGPRs).
constexpr int kSpmvMinWaves = 1;
// Grid: [bins of the long rows][short chunks] (or chunks first). Returns the chunk
// index whose alpha partial this workgroup owns, or -1.
// F = CW | V8 << 3 | SC16 << 4 | BC16 << 5 | WIN << 6: uniform chunk width (0: any), int8
// values, uint16 column offsets in the chunks / in the bins, chunk column window in LDS.
template <int F, class Epi, class ScaleFn>
__device__ __forceinline__ int spmv_block_impl(const CsrDev& A, const double* __restrict__ xsrc,
                                               ScaleFn scale_of, const Epi& epi, double& acc,
                                               double* lds) {
  const int b = blockIdx.x;
  if (b < A.n_slice_blocks) {
    // bin (m, s) -> block: with S = 8T >= 8 slices, slice s runs on XCD s / T (block
    // b = 8 (T m + s % T) + s / T), the XCD whose rows its columns are (speed only)
    int m, s;
    if (A.n_slices >= 8) {
      const int T = A.n_slices >> 3, q = b >> 3;
      s = T * (b & 7) + q % T;
      m = q / T;
    } else {
      m = b / A.n_slices;
      s = b % A.n_slices;
    }
    long_bin<((F >> 3) & 1), ((F >> 5) & 1)>(A, m, s, xsrc, scale_of, epi, lds);
    return -1;
  }
  const int chunk = chunk_of_block(A, b - A.n_slice_blocks);
  if (chunk < 0) return -1;  // grid padding
  return short_chunk<(F & 7), ((F >> 3) & 1), ((F >> 4) & 1), ((F >> 6) & 1)>(A, chunk, xsrc, scale_of, epi, acc, lds)
             ? chunk : -1;
}

template <int F, class Epi, class ScaleFn>
__device__ __forceinline__ int spmv_block(const CsrDev& A, const double* __restrict__ xsrc,
                                          ScaleFn scale_of, const Epi& epi, double& acc,
                                          double* lds) {
  TPL_MARK(0);
  TPL_MARK_ID();
  const int r = spmv_block_impl<F>(A, xsrc, scale_of, epi, acc, lds);
  TPL_MARK(5);
  return r;
}

} // namespace tpl
