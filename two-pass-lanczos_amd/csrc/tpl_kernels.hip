// tpl_kernels.hip — CDNA4 (gfx950) kernels of the two-pass Lanczos engine.
//
// One Lanczos step of the reference (src/algorithms/mod.rs:167-212 + :292-340)
//     w = A v_j ; w -= beta_{j-1} v_{j-1} ; alpha_j = v_j . w ; w -= alpha_j v_j ;
//     beta_j = ||w|| ; v_{j+1} = w * (1/beta_j)
// has two grid-wide dependencies (alpha before the second AXPY, beta before the
// next SpMV). Pass one therefore runs two launches per step:
//   k_p1_spmv  [reduce beta partials -> beta_{j-1}, breakdown test]
//              fused SpMV gathering x = r_j * (1/beta_{j-1}) (the normalisation
//              v_j = w/beta folded into the gather, bit-identical to storing v_j);
//              epilogue w = y - beta_{j-1} v_{j-1}; alpha partials
//   k_p1_axpy  [reduce alpha partials -> alpha_j] r_{j+1} = w - alpha_j v_j ;
//              ||r_{j+1}||^2 partials
// Pass two (src/algorithms/lanczos_two_pass.rs:176-312) knows every coefficient, so
// each step is ONE launch (k_p2_spmv): SpMV + both AXPYs + scale + x += y v.
//
// Arithmetic follows the reference op by op (-ffp-contract=off for this file):
//   sub(w, mul(beta, v)) -> w - beta*v (two roundings), v = w * (1/beta)
//   (reciprocal then multiply), x = x + y*v. Reductions use the FIXED trees of
//   tpl_device.h, so results are run-to-run bitwise reproducible and pass two
//   regenerates pass one's basis bit for bit (reference: basis_drift_fro = 0.0,
//   results/orthogonality_*.csv).
//
// Latency structure (measured on MI355X: a graph-launched empty kernel costs 1.6 us,
// and a dependent memory round trip 1-2 us once the chip is loaded): every
// workgroup issues its independent loads (stop flag, grid partials, entries,
// epilogue vectors) before its first wait. A short-row chunk costs two round trips
// (entries -> gathers); a long-row bin the same two plus an LDS pass, and the
// slice-7 bins one more (polling the other slices' partials).
#include "tpl_kcommon.h"

namespace tpl {

// ------------------------------------------------------------------ kernels
template <int F>
__global__ __launch_bounds__(kTPB, kSpmvMinWaves) void k_spmv(CsrDev A, const double* __restrict__ x,
                                               double* __restrict__ y) {
  extern __shared__ double lds[];
  double acc = 0.0;
  spmv_block<F>(A, x, UnitScale{}, EpiSpmv{y}, acc, lds);
}

// Pass-one prologue: ||b||^2 partials, reset flags.
__global__ __launch_bounds__(kTPB) void k_p1_init(CsrDev A, DevState S,
                                                  const double* __restrict__ b) {
  __shared__ double red[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S.flags[0] = 0;
    S.flags[1] = 0;
    S.flags[2] = 0;
    S.flags[3] = 0;
    S.flags[4] = 0;
    S.flags[5] = 0;
  }
  const int rb = elem_block(A, blockIdx.x);
  if (rb < 0) return;
  const int64_t beg = (int64_t)rb * A.E;
  const int64_t end = beg + A.E < A.n ? beg + A.E : A.n;
  double acc = 0.0;
  for (int64_t i0 = beg + 2 * threadIdx.x; i0 < end; i0 += 2 * kTPB) {
    if (i0 + 1 < end) {
      const double2 v = *reinterpret_cast<const double2*>(b + i0);
      acc = i0 < A.norm_n ? fma(v.x, v.x, acc) : acc;
      acc = i0 + 1 < A.norm_n ? fma(v.y, v.y, acc) : acc;
    } else {
      const double v = b[i0];
      acc = i0 < A.norm_n ? fma(v, v, acc) : acc;
    }
  }
  const double p = block_sum_tail(acc, red);
  if (threadIdx.x == 0) S.Pb[rb] = p;
}

// Pass one / standard, step j >= 1. r_cur = r_j (== b at j = 1), this rank's rows;
// xsrc = the gather source holding r_j for every column (== r_cur on one GPU, the
// all-gathered vector when the rows are partitioned over ranks).
// beta_{j-1} comes from the G2_r norm partials k_p1_axpy left: NBP per thread (1 when
// G2_r <= 256, the usual case; 4 up to 1024), loaded at entry ahead of the entries and
// gathers, reduced in scale_fn once they are in flight. The registers of those loads stay
// live across the whole SpMV, so they set the kernel's occupancy: with one partial per
// thread (the wave totals exchanged through LDS behind one barrier) k_p1_spmv<58> needs
// 58 VGPRs, 8 waves per SIMD, and the 1,560-workgroup grid at 500k arcs is resident at
// once; with four per lane (each wave reducing all 256 itself, no barrier: r03) it needed
// 76 (6 waves): 24 workgroups waited for a slot and the chunks started at 1.8 us (median)
// instead of 0.4 (stamps, scripts/stamps.py). Same box, alternated three times: solve
// 9.12-9.17 vs 9.50-9.56 ms, pass one 11.35-11.45 vs 12.17-12.21 us per step, isolated
// k_p1_spmv 6.60-6.67 vs 7.46-7.68 us; the tree and so the bits are the same.
constexpr int p1_min_waves(int F, int NBP) {
  return (NBP > 1 && (F & 8) && ((F & 7) == 1 || (F & 7) == 2)) ? 6 : kSpmvMinWaves;
}
template <int F, int NBP>
__device__ __forceinline__ void p1_spmv_body(const CsrDev& A, const DevState& S,
                                             const double* __restrict__ xsrc,
                                             const double* __restrict__ r_cur,
                                             const double* __restrict__ r_prev,
                                             double* __restrict__ W, double* __restrict__ Vcol,
                                             int j, unsigned long long* stamp, double* red,
                                             double* redb, double* lds,
                                             double* redr = nullptr) {
  // every kernel argument in ONE scalar round trip, the launch stamp's pointer included:
  // a branch on an argument before this point (the stamp test) split the loads into three
  // dependent round trips ahead of the first vector load (ISA, round 6)
  pin_layout_args(A);
  asm volatile("" ::"s"(S.Pb_r), "s"(S.flags), "s"(S.norms), "s"(S.betas), "s"(S.Pa), "s"(A.G2_r),
               "s"(xsrc), "s"(r_cur), "s"(r_prev), "s"(W), "s"(Vcol), "s"(j), "s"(stamp));
  launch_stamp(stamp);
  PartialRegs<(NBP > 0 ? NBP : -NBP)> pr;
  if constexpr (NBP > 0) {
    load_partials(S.Pb_r, A.G2_r, pr);
  } else {
    // NBP = -kPbRanks (replicated partition, round 6): every rank's norm partials,
    // all-gathered pb_ld apart and zero-padded; lane t loads partial t of each rank
    const int ld = A.pb_ld, R = A.G2_r;
#pragma unroll
    for (int r = 0; r < -NBP; ++r)
      pr.v[r] = S.Pb_r[(size_t)clampi(r, R - 1) * ld + clampi((int)threadIdx.x, ld - 1)];
  }
  // the stop flag and beta_{j-2} with the partials, ahead of the entries and gathers:
  // read later, their wait would drain every gather in flight before the beta chain
  int stop0 = S.flags[0];
  double norm_prev = (j >= 2) ? S.norms[j - 2] : 1.0;
  // keep these loads first: sunk below the gathers by the scheduler, their wait would
  // again drain every gather before the beta chain
  __builtin_amdgcn_sched_barrier(0);
  EpiPass1 epi;
  epi.r_cur = r_cur;
  epi.r_prev = (j >= 2) ? r_prev : r_cur;
  epi.has_prev = j >= 2;
  epi.invN_prev = 0.0;
  epi.invN_cur = 0.0;
  epi.beta_sub = 0.0;
  epi.W = W;
  epi.Vcol = Vcol;
  epi.Pa_long = S.Pa + A.n_chunks;
  // beta_{j-1} (||b|| at j = 1) from the norm partials; fills the epilogue. Runs once the
  // workgroup's loads are in flight.
  auto scale_fn = [&]() -> Scale {
    __builtin_amdgcn_sched_barrier(0);
    // opaque here: the optimiser would otherwise hoist the stop test and the reciprocal
    // to the loads, making every workgroup wait for them before issuing its entries
    asm volatile("" : "+v"(stop0), "+v"(norm_prev));
    if (stop0) return Scale{0.0, false};
    epi.invN_prev = (j >= 2) ? 1.0 / norm_prev : 0.0;
    // the canonical tree (s = 0; s += P[t + 256u]; tree256), one barrier: its LDS words
    // (redb) are not reused, and the barrier waits for LDS traffic only, never for the
    // gathers in flight
    double beta;
    if constexpr (NBP == 1) {
      double sq = 0.0;
      if ((int)threadIdx.x < A.G2_r) sq = sq + pr.v[0];
      beta = sqrt(block_sum_tail(sq, redb));
    } else if constexpr (NBP > 1) {  // any count (more than 256 NBP in batches)
      beta = sqrt(finish_partials(S.Pb_r, A.G2_r, pr, redb));
    } else {
      // each rank's total by the tree the rank-total launch applied (k_reorth_reduce:
      // s = 0; s += P[t]; wave sums; (S0 + S1) + (S2 + S3) — the zero padding adds +0.0 to
      // +0.0), then the R totals exactly as the one-partial path above reduces the
      // all-gathered totals: the bits of the rank-total launch + all-gather, one launch
      // less per pass-one step. One barrier more than that path; it waits
      // for LDS traffic only, never for the gathers in flight.
      const int R = A.G2_r, ld = A.pb_ld;
#pragma unroll
      for (int r = 0; r < -NBP; ++r) {
        if (r < R) {  // uniform
          double sr = 0.0;
          if ((int)threadIdx.x < ld) sr = sr + pr.v[r];
          sr = wave_sum(sr);
          if ((threadIdx.x & 63) == 0) redr[4 * r + (threadIdx.x >> 6)] = sr;
        }
      }
      __syncthreads();
      double sq = 0.0;
      if ((int)threadIdx.x < R) {
        const double* q = redr + 4 * threadIdx.x;
        sq = sq + ((q[0] + q[1]) + (q[2] + q[3]));
      }
      beta = sqrt(block_sum_tail(sq, redb));
    }
    if (beta <= kBreakdownTol) {
      // j == 1: zero b -> InputError (src/algorithms/mod.rs:267-273);
      // j  > 1: breakdown -> steps_taken = j - 1, beta not pushed
      //         (src/algorithms/lanczos_two_pass.rs:245-249).
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
  const int slot = spmv_block<F>(A, xsrc, scale_fn, epi, acc, lds);
  if (slot < 0) return; // uniform per workgroup
  const double p = block_sum_tail(acc, red);
  // write-through: every k_p1_axpy workgroup, on every XCD, reads all the partials
  // next (measured: pass one -0.2 to -0.3 us per step against a plain store)
  if (threadIdx.x == 0) st_out(S.Pa + slot, p);
}
// G2_r <= 256 norm partials (one per thread) ...
template <int F>
__global__ __launch_bounds__(kTPB, p1_min_waves(F, 1)) void k_p1_spmv(CsrDev A, DevState S,
                                                  const double* __restrict__ xsrc,
                                                  const double* __restrict__ r_cur,
                                                  const double* __restrict__ r_prev,
                                                  double* __restrict__ W,
                                                  double* __restrict__ Vcol, int j,
                                                  unsigned long long* stamp) {
  TPL_MARK_FIRST();
  __shared__ double red[4], redb[4];
  extern __shared__ double lds[];
  p1_spmv_body<F, 1>(A, S, xsrc, r_cur, r_prev, W, Vcol, j, stamp, red, redb, lds);
}
// ... every rank's norm partials, gathered (replicated partition: CsrDev::pb_ld) ...
template <int F>
__global__ __launch_bounds__(kTPB, p1_min_waves(F, 1)) void k_p1_spmv_gp(CsrDev A, DevState S,
                                                  const double* __restrict__ xsrc,
                                                  const double* __restrict__ r_cur,
                                                  const double* __restrict__ r_prev,
                                                  double* __restrict__ W,
                                                  double* __restrict__ Vcol, int j,
                                                  unsigned long long* stamp) {
  __shared__ double red[4], redb[4], redr[4 * kPbRanks];
  extern __shared__ double lds[];
  p1_spmv_body<F, -kPbRanks>(A, S, xsrc, r_cur, r_prev, W, Vcol, j, stamp, red, redb, lds,
                             redr);
}
// ... and more (four per thread first, the rest in batches; the 5M-arc instance's 1,024
// row blocks)
template <int F>
__global__ __launch_bounds__(kTPB, p1_min_waves(F, 4)) void k_p1_spmv_wide(CsrDev A, DevState S,
                                                  const double* __restrict__ xsrc,
                                                  const double* __restrict__ r_cur,
                                                  const double* __restrict__ r_prev,
                                                  double* __restrict__ W,
                                                  double* __restrict__ Vcol, int j,
                                                  unsigned long long* stamp) {
  __shared__ double red[4], redb[4];
  extern __shared__ double lds[];
  p1_spmv_body<F, 4>(A, S, xsrc, r_cur, r_prev, W, Vcol, j, stamp, red, redb, lds);
}

// ---- T_k^{-1} e_1 on the device (the one-graph inv): the host solver's operations
// (tpl_ftk.cpp: the LAPACK dgtsv scheme, tridiagonal elimination with partial pivoting,
// then back substitution), bit for bit.
// Running row i of the elimination: its pivot, super-diagonal and right-hand side.
struct LuRow {
  double d, du, b;
};
// Eliminate row i (dl = beta_i, d1 = alpha_{i+1}, du1 = beta_{i+1} or 0 when row i + 1 is
// the last; more = row i + 2 exists): stores row i of U (D, DU, DU2) and of the
// transformed right-hand side (B), advances `cur` to row i + 1. The operations of the
// host loop in its order (-ffp-contract=off).
__device__ __forceinline__ void lu_row(int i, bool more, double dli, double d1, double du1,
                                       LuRow& cur, double* D, double* DU, double* DU2,
                                       double* B) {
  double dip1 = d1, duip1 = du1, bip1 = 0.0, du2i = 0.0;
  if (fabs(cur.d) >= fabs(dli)) {
    const double fact = dli / cur.d;
    dip1 = dip1 - fact * cur.du;
    bip1 = bip1 - fact * cur.b;
    D[i] = cur.d;
    DU[i] = cur.du;
    B[i] = cur.b;
  } else {
    const double fact = cur.d / dli;
    D[i] = dli;
    const double temp = dip1;
    dip1 = cur.du - fact * temp;
    if (more) {
      du2i = duip1;
      duip1 = -fact * du2i;
    }
    DU[i] = temp;
    B[i] = bip1;            // b[i] <- old b[i+1] (= 0: b[i+1] is first set at step i)
    bip1 = cur.b - fact * bip1;
  }
  DU2[i] = du2i;
  cur.d = dip1;
  cur.du = duip1;
  cur.b = bip1;
}
// a / b given y = RN(1 / b): Markstein's correction q = RN(q0 + RN(a - b q0) y), q0 =
// RN(a y), is the correctly rounded quotient — the IEEE division's bits — whenever no
// intermediate leaves the normal range; elsewhere (zeros, huge or tiny magnitudes,
// non-finite values) the IEEE division itself. Three dependent operations instead of the
// division's ten on the back substitution's chain. (Checked against IEEE division on
// 10^9 random pairs in range, exact and binade-boundary quotients included: no
// difference; tests/native/div_rn_check.c restates it on the host, tests/test_native.py)
__device__ __forceinline__ bool exp_in_range(double v) {
  const unsigned e = (unsigned)(__double2hiint(v) >> 20) & 0x7FFu;  // biased exponent
  return e - (1023u - 900u) <= 1800u;  // 2^-900 <= |v| < 2^901
}
__device__ __forceinline__ double div_rn(double a, double b, double y, bool b_ok) {
  if (b_ok && exp_in_range(a)) {
    const double q0 = a * y;
    const double q = fma(fma(-b, q0, a), y, q0);
    if (exp_in_range(q)) return q;
  } else if (b_ok && a == 0.0) {
    return a * y;  // +-0 with the quotient's sign
  }
  return a / b;
}

// Pass one / standard, step j: alpha_j; r_{j+1} = w - alpha_j v_j; ||r_{j+1}||^2 partials.
// NP: alpha partials loaded per thread up front (the launcher picks the smallest of 2, 4,
// 8, 12 with 256 NP >= NA_r; more are reduced in batches): clamped duplicate loads of a
// small partial array only cost issue slots and cache traffic.
// elim (one-graph inv): one more workgroup (the last) eliminates row j - 3 of T_k's LU
// (lu_row): its inputs beta_{j-3}, alpha_{j-2} and beta_{j-2} (0-based) are all known
// once this step's k_p1_spmv has reduced beta — the row is done off the critical path,
// so only the last rows and the back substitution remain after pass one (k_ftk_inv).
template <int NP>
__global__ __launch_bounds__(kTPB) void k_p1_axpy(CsrDev A, DevState S,
                                                  const double* __restrict__ W,
                                                  const double* __restrict__ r_cur,
                                                  double* __restrict__ r_next, int j, int k,
                                                  int elim, unsigned long long* stamp) {
  __shared__ double red[4];
  // every kernel argument in ONE scalar round trip before any branch on one of them (the
  // stamp and elim tests used to split the loads into three dependent round trips ahead of
  // the first vector load: ISA, round 6)
  asm volatile("" ::"s"(A.E), "s"(A.n), "s"(A.norm_n), "s"(A.NA_r), "s"(S.Pa_r), "s"(S.flags),
               "s"(S.norms), "s"(S.alphas), "s"(S.Pb));
  asm volatile("" ::"s"(W), "s"(r_cur), "s"(r_next), "s"(j), "s"(k), "s"(elim), "s"(stamp));
  launch_stamp(stamp);
  if (elim && blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x != 0 || j < 3) return;
    const int i = j - 3;
    double* D = S.lu;
    double* st = S.lu + 4 * (size_t)S.kcap;
    // every input with the flags (one round trip): the row's coefficients and the running
    // row (the initial one at i = 0: alpha_0, beta_0, 1)
    const int stop = S.flags[0], done = S.flags[5];
    const double dli = S.betas[i], d1 = S.alphas[i + 1], du1 = S.betas[i + 1];
    LuRow cur{st[0], st[1], st[2]};
    const double a0 = S.alphas[0];
    if (stop || done != i) return;  // breakdown at this step: the tail finishes the rows
    if (i == 0) cur = LuRow{a0, dli, 1.0};
    lu_row(i, true, dli, d1, du1, cur, D, D + S.kcap, D + 2 * (size_t)S.kcap,
           D + 3 * (size_t)S.kcap);
    st[0] = cur.d;
    st[1] = cur.du;
    st[2] = cur.b;
    S.flags[5] = i + 1;
    return;
  }
  const int rb = elem_block(A, blockIdx.x);
  if (rb < 0) return;
  TPL_MARK_AT(kAxpyMarkBase, 0);
  PartialRegs<NP> pr;
  const int na_ = A.NA_r;
  load_partials(S.Pa_r, na_, pr);
  const int64_t beg = (int64_t)rb * A.E;
  const int64_t end = beg + A.E < A.n ? beg + A.E : A.n;
  // All of this thread's pairs (up to kAxPairs) are loaded before alpha is known, at
  // clamped addresses (vectors are padded to 64 doubles, so a pair starting below
  // `end` is always readable); the loads are unconditional so none is sunk behind the
  // reduction.
  constexpr int kAxPairs = 4;
  const int64_t i00 = beg + 2 * threadIdx.x;
  double2 w0[kAxPairs], rc0[kAxPairs];
#pragma unroll
  for (int q = 0; q < kAxPairs; ++q) {
    const int64_t i0 = i00 + (int64_t)q * 2 * kTPB;
    const int64_t ic = i0 < end ? i0 : beg;
    w0[q] = *reinterpret_cast<const double2*>(W + ic);
    rc0[q] = *reinterpret_cast<const double2*>(r_cur + ic);
  }
  // The DevState scalars (stop flag, ||r_j||) are read only now, with the vector loads
  // in flight: waited on at entry they would add a dependent round trip.
  __builtin_amdgcn_sched_barrier(0);
  const int stop = S.flags[0];
  const double normj = S.norms[j - 1];
  TPL_MARK_AT(kAxpyMarkBase, 1);
#if TPL_STAMP
  // diagnostic build: when the alpha partials (issued first) have landed, the vector loads
  // (2 kAxPairs issued after them) still in flight
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  TPL_MARK_AT(kAxpyMarkBase, 4);
#endif
  // alpha while the vectors are in flight: its wait covers the partials (issued first)
  // only. The reduction's LDS stores and barrier keep the vector loads ahead of it, and
  // nothing tests the (uniform) stop flag before it: a branch there would let the compiler
  // sink the loads into it, behind the reduction.
  const double alpha = finish_partials(S.Pa_r, na_, pr, red);
  TPL_MARK_AT(kAxpyMarkBase, 2);
  if (stop) return;
  if (rb == 0 && threadIdx.x == 0) {
    S.alphas[j - 1] = alpha;
    S.flags[2] = j;
  }
  if (j == k) return; // beta_k is never used (src/algorithms/lanczos_two_pass.rs:252-254)
  const double invN = 1.0 / normj;
  double acc = 0.0;
  auto step = [&](int64_t i0, double2 w, double2 rc) {
    double2 r;
    r.x = w.x - alpha * (rc.x * invN);
    r.y = w.y - alpha * (rc.y * invN);
    // 16-B non-temporal stores: r_{j+1} leaves the L2 during the kernel instead of as
    // 4 MB of dirty lines at the boundary (same box, alternated twice: pass one 12.16-12.22
    // vs 12.33 us per step with plain 16-B stores; write-through +0.5 us)
    if (i0 + 1 < end) {
      typedef double d2v __attribute__((ext_vector_type(2)));
      d2v rv = {r.x, r.y};
      __builtin_nontemporal_store(rv, reinterpret_cast<d2v*>(r_next + i0));
    } else {
      __builtin_nontemporal_store(r.x, r_next + i0);
    }
    acc = i0 < A.norm_n ? fma(r.x, r.x, acc) : acc;
    acc = i0 + 1 < end && i0 + 1 < A.norm_n ? fma(r.y, r.y, acc) : acc;
  };
#pragma unroll
  for (int q = 0; q < kAxPairs; ++q) {
    const int64_t i0 = i00 + (int64_t)q * 2 * kTPB;
    if (i0 < end) step(i0, w0[q], rc0[q]);
  }
  for (int64_t i0 = i00 + (int64_t)kAxPairs * 2 * kTPB; i0 < end; i0 += 2 * kTPB) // E > 2048
    step(i0, *reinterpret_cast<const double2*>(W + i0),
         *reinterpret_cast<const double2*>(r_cur + i0));
  TPL_MARK_AT(kAxpyMarkBase, 3);
  const double p = block_sum_tail(acc, red);
  if (threadIdx.x == 0) S.Pb[rb] = p;  // plain: write-through measured +0.35 us here
  TPL_MARK_AT(kAxpyMarkBase, 5);
}

// Pass two prologue: v_1 = b * (1/||b||); x = v_1 * y_1 (src/algorithms/lanczos_two_pass.rs:248-252).
// dyn: steps_taken is known only on the device (one-graph solve): nothing to do after
// an error (zero b) or when pass one took no step.
__global__ __launch_bounds__(kTPB) void k_p2_init(int64_t n, DevState S,
                                                  const double* __restrict__ b,
                                                  double* __restrict__ v1,
                                                  double* __restrict__ x,
                                                  double* __restrict__ Vcol, int dyn) {
  if (dyn && (S.flags[1] || S.flags[2] < 1)) return;
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

// Pass two, step j = 1 .. steps-1: regenerate v_{j+1}, accumulate x. rec: step j's
// coefficient record (EpiPass2R: loaded after the gathers, never waited on before the
// epilogue; the gather scale is 1).
template <int F>
__global__ __launch_bounds__(kTPB, kSpmvMinWaves) void k_p2_spmv(CsrDev A,
                                                  const double* __restrict__ rec,
                                                  const double* __restrict__ xsrc,
                                                  const double* __restrict__ v_cur,
                                                  const double* __restrict__ v_prev,
                                                  double* __restrict__ v_next,
                                                  double* __restrict__ x,
                                                  double* __restrict__ Vcol, int j,
                                                  int nflush) {
  extern __shared__ double lds[];
  pin_layout_args(A);
  asm volatile("" ::"s"(rec), "s"(xsrc), "s"(v_cur), "s"(v_prev), "s"(v_next), "s"(x), "s"(Vcol),
               "s"(j), "s"(nflush));
  EpiPass2R epi;
  epi.v_cur = v_cur;
  epi.v_prev = (j >= 2) ? v_prev : v_cur;
  epi.rec = rec;
  epi.has_prev = j >= 2;
  epi.nflush = nflush;
  epi.v_next = v_next;
  epi.x = x;
  epi.Vcol = Vcol;
  double acc = 0.0;
  spmv_block<F>(A, xsrc, UnitScale{}, epi, acc, lds);
}

// Pass-two step records (EpiPass2R): record j (1 <= j < k) = {beta_{j-1} (0 at j = 1),
// alpha_j, 1 / beta_j, y_j, y_{j-1}, y_{j-2} (0 at j = 1), active, 0}. dyn (one-graph
// solve): active = j < steps_taken (the device-held count), else 1.
__global__ __launch_bounds__(kTPB) void k_p2_coefs(DevState S, int k, int dyn) {
  const int j = blockIdx.x * kTPB + threadIdx.x;
  if (j < 1 || j >= k) return;
  double* r = S.p2c + 8 * (size_t)j;
  double2 r01, r23, r45, r67;
  r01.x = j >= 2 ? S.betas[j - 2] : 0.0;
  r01.y = S.alphas[j - 1];
  r23.x = 1.0 / S.betas[j - 1];
  r23.y = S.y[j];
  r45.x = S.y[j - 1];
  r45.y = j >= 2 ? S.y[j - 2] : 0.0;
  r67.x = dyn ? ((S.flags[1] == 0 && j < S.flags[2]) ? 1.0 : 0.0) : 1.0;
  r67.y = 0.0;
  reinterpret_cast<double2*>(r)[0] = r01;
  reinterpret_cast<double2*>(r)[1] = r23;
  reinterpret_cast<double2*>(r)[2] = r45;
  reinterpret_cast<double2*>(r)[3] = r67;
}

// One-graph solve, after the k - 1 step launches: the x terms still pending at the last
// step (last = steps_taken - 1 not a multiple of 3 — the step launches flush only at
// multiples of 3, the host-side schedule p2_flush also at `last`), added exactly as the
// last step's grouped flush would: x + y_{last-1} v_last (2 pending) + y_last v_{last+1}.
__global__ __launch_bounds__(kTPB) void k_p2_tail(int64_t n, DevState S, double* __restrict__ x,
                                                  const double* __restrict__ V0,
                                                  const double* __restrict__ V1,
                                                  const double* __restrict__ V2) {
  if (S.flags[1]) return;
  const int last = S.flags[2] - 1;
  if (last < 1) return;
  const int pending = last % 3;
  if (pending == 0) return;
  const double* ring[3] = {V0, V1, V2};
  const double* vl = ring[last % 3];
  const double* vn = ring[(last + 1) % 3];
  const double y1 = S.y[last - 1], y0 = S.y[last];
  for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kTPB) {
    double xv = x[i];
    if (pending == 2) xv = xv + y1 * vl[i];
    x[i] = xv + y0 * vn[i];
  }
}

// f(T_k) = T_k^{-1} on the device: y = ||b|| * T_k^{-1} e_1, bit for bit the host solver
// tpl_ftk_inv (tpl_ftk.cpp: the LAPACK dgtsv scheme — tridiagonal elimination with partial
// pivoting, then back substitution; IEEE operations, -ffp-contract=off). Both halves are
// one dependent chain. The elimination's rows [0, flags[5]) were done during pass one by
// k_p1_axpy's extra workgroup (one row per step, one-graph inv); the rest — the last
// rows, or all of them (tpl_op_ftk_device, the one-pass solver) — run here on lane 0
// with alpha and beta staged in LDS. The back substitution divides by pivots known before
// it starts, so their reciprocals are taken first on all lanes and every division of the
// chain becomes Markstein's correction (div_rn: three dependent operations, the IEEE
// quotient's bits); a row whose operands leave div_rn's range sets a flag and the whole
// substitution is redone with IEEE divisions. The chain runs on lane 0 with nothing else
// on it: x' goes to LDS (all lanes scale and store y after), the range tests of its
// numerators and quotients are deferred to all lanes (round 4: 85.6 us at k = 500 with
// them and the global stores on the chain). Dynamic LDS: 11 k doubles.
// scale: 1 — y = ||b|| y' (two-pass: y_k, src/solvers.rs:169); 0 — y' itself (one-pass:
// the reconstruction multiplies by ||b||, src/solvers.rs:96-104); x * 1.0 is exact.
__global__ __launch_bounds__(kTPB) void k_ftk_inv(DevState S, int scale) {
  extern __shared__ double sh[];
  __shared__ double last[3];
  const int n = S.flags[2];
  if (S.flags[1] || n < 1) return;
  const size_t kc = (size_t)S.kcap;
  const int done = min(S.flags[5], max(n - 1, 0));  // rows eliminated during pass one
  double* D = sh;
  double* DU = sh + n;
  double* DU2 = sh + 2 * n;
  double* B = sh + 3 * n;
  double* R = sh + 4 * n;   // reciprocals of the pivots
  double* al = sh + 5 * n;  // alpha, beta of the rows still to eliminate
  double* be = sh + 6 * n;
  for (int i = threadIdx.x; i < n; i += kTPB) {
    if (i < done) {
      D[i] = S.lu[i];
      DU[i] = S.lu[kc + i];
      DU2[i] = S.lu[2 * kc + i];
      B[i] = S.lu[3 * kc + i];
    }
    al[i] = S.alphas[i];
    be[i] = i + 1 < n ? S.betas[i] : 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    LuRow cur = done == 0 ? LuRow{al[0], n > 1 ? be[0] : 0.0, 1.0}
                          : LuRow{S.lu[4 * kc], S.lu[4 * kc + 1], S.lu[4 * kc + 2]};
    for (int i = done; i + 1 < n; ++i)
      lu_row(i, i + 2 < n, be[i], al[i + 1], i + 2 < n ? be[i + 1] : 0.0, cur, D, DU, DU2, B);
    last[0] = cur.d;
    last[1] = cur.b;
  }
  __syncthreads();
  // Off the chain, on all lanes: the pivots' reciprocals, each row repacked as one
  // 32-B record {B, DU, DU2, D} (two 16-B LDS reads per row on the chain instead of four
  // 8-B ones), and div_rn's range test of every pivot and reciprocal.
  // 4 (n - 1) doubles from an even offset: 16-B aligned records for the 16-B LDS accesses
  // whatever the parity of n (at most 11 n - 3 <= 11 kcap doubles in all)
  double* P = sh + ((7 * n + 1) & ~1);
  bool pbad = false;
  for (int i = threadIdx.x; i + 1 < n; i += kTPB) {
    const double d = D[i], r = 1.0 / d;
    R[i] = r;
    typedef double d2v __attribute__((ext_vector_type(2)));
    reinterpret_cast<d2v*>(P)[2 * i] = d2v{B[i], DU[i]};
    reinterpret_cast<d2v*>(P)[2 * i + 1] = d2v{DU2[i], d};
    pbad = pbad || !(exp_in_range(d) && exp_in_range(r));
  }
  const bool any_pbad = __syncthreads_or(pbad);
  double* Y = D;   // x' of every row (D is read only through P from here on)
  double* T = DU;  // the numerator t of every row, for the deferred range test
  if (threadIdx.x == 0) {
    // back substitution with U = (D, DU, DU2): x_i = ((B_i - DU_i x_{i+1}) - DU2_i x_{i+2}) / D_i
    const double xl = last[1] / last[0];  // b[n-1] / d[n-1]
    Y[n - 1] = xl;
    if (n >= 2) {
      double x1 = xl, x0;
      {
        const double t = B[n - 2] - DU[n - 2] * x1;
        x0 = div_rn(t, D[n - 2], R[n - 2], !any_pbad);
        Y[n - 2] = x0;
        T[n - 2] = 0.0;  // row n - 2 took div_rn's own checks
      }
      // the fast chain: Markstein's correction with every operand read one row ahead; the
      // range tests of t and the quotient are deferred to all lanes after the loop
      typedef double d2v __attribute__((ext_vector_type(2)));
      const d2v* PR = reinterpret_cast<const d2v*>(P);
      d2v p0 = {0.0, 0.0}, p1 = {0.0, 1.0};
      double r_n = 1.0;
      if (n >= 3) {
        p0 = PR[2 * (n - 3)]; p1 = PR[2 * (n - 3) + 1]; r_n = R[n - 3];
      }
      for (int ii = n - 3; ii >= 0; --ii) {
        const double bi = p0.x, dui = p0.y, du2i = p1.x, di = p1.y, ri = r_n;
        if (ii > 0) {
          p0 = PR[2 * (ii - 1)]; p1 = PR[2 * (ii - 1) + 1]; r_n = R[ii - 1];
        }
        const double t = bi - dui * x0 - du2i * x1;
        const double q0 = t * ri;
        const double qm = fma(fma(-di, q0, t), ri, q0);
        const double xi = t == 0.0 ? q0 : qm;  // +-0: q0 carries the quotient's sign
        Y[ii] = xi;
        T[ii] = t;
        x1 = x0;
        x0 = xi;
      }
    }
  }
  __syncthreads();
  // deferred: a row whose numerator or quotient left div_rn's range (t == 0 is exact)
  bool bad = any_pbad && n >= 2;
  for (int i = threadIdx.x; i + 2 < n; i += kTPB) {
    const double t = T[i];
    bad = bad || !(t == 0.0 || (exp_in_range(t) && exp_in_range(Y[i])));
  }
  if (__syncthreads_or(bad)) {
    // an operand outside div_rn's range (singular or badly scaled T_k): IEEE divisions
    if (threadIdx.x == 0) {
      const double* PD = P;
      double x1 = Y[n - 1];
      double x0 = (PD[4 * (n - 2)] - PD[4 * (n - 2) + 1] * x1) / PD[4 * (n - 2) + 3];
      Y[n - 2] = x0;
      for (int ii = n - 3; ii >= 0; --ii) {
        const double xi = (PD[4 * ii] - PD[4 * ii + 1] * x0 - PD[4 * ii + 2] * x1) / PD[4 * ii + 3];
        Y[ii] = xi;
        x1 = x0;
        x0 = xi;
      }
    }
    __syncthreads();
  }
  const double bnorm = scale ? S.norms[0] : 1.0;
  for (int i = threadIdx.x; i < n; i += kTPB) S.y[i] = Y[i] * bnorm;
}

// f(T_k) = exp(T_k) on the device: y = ||b|| exp(T_k) e_1 (src/bin/stability.rs:175-193
// forms Q exp(Lambda) Q^T e_1 from a dense EVD; the host built-in tpl_ftk_exp runs QL).
// A QL sweep is one long chain of dependent rotations (1.2 ms at k = 200 on the host, worse
// on one GPU lane), so the device evaluates the same function with a parallel method: the
// Chebyshev expansion of exp on an interval [a, b] holding the spectrum,
//   exp(c + r x) = e^c (I_0(r) + 2 sum_m I_m(r) T_m(x)),  c = (a+b)/2, r = (b-a)/2,
// applied to e_1 with x = (T - c)/r by Clenshaw's recurrence (every row of the tridiagonal
// product on its own thread, one LDS exchange and barrier per term), the modified Bessel
// coefficients generated alongside by Miller's backward recurrence I_{m-1} = I_{m+1} +
// (2m/r) I_m and normalised by e^r = I_0 + 2 sum I_m — no coefficient table, no EVD, and
// no clusters to resolve (eigenvectors never appear). [a, b]: one round of 512-shift Sturm
// multisection of the Gershgorin interval (a count is exact for a matrix within a few ulps
// of T, so the bracket holds the spectrum up to the added margin; the bracket's excess,
// at most 1/513 of the Gershgorin width, only scales the error bound by its exponential). Accuracy is the
// EVD's class: the error is a small multiple of eps * exp(lambda_max) (the coefficients sum
// to e^b), against the tolerance the host QL itself meets; the terms run until the
// coefficients fall below 1e-22 of e^b (Debye asymptotics of I_m(r)). Falls back to the host
// (flags[4] = 1, y = 0) when T is not finite, when the expansion needs more than
// kExpMaxTerms terms (|lambda_max - lambda_min| above ~2e4), or when ||y|| < 1e-3 e^b
// (the absolute error bound would not be small against ||y||). Dynamic LDS: 4 kcap + 4 doubles
// and 256 ints.
constexpr int kExpRows = 8;          // rows per thread: n <= 2048 (the LDS bound is lower)
constexpr int kExpMaxTerms = 16384;
constexpr double kExpMinRatio = 1e-3;  // ||exp(T - b I) e_1|| below this: host (see the end)
constexpr int kExpShifts = 2 * kTPB;   // Sturm shifts per end of the spectrum (one round)
// Reciprocal for the Sturm pivots: v_rcp_f64 and one Newton step (a Sturm count tolerates
// the last-bit difference from a division; the bracket carries a margin far above it)
__device__ __forceinline__ double rcp_nr(double q) {
  const double r = __builtin_amdgcn_rcp(q);
  return fma(fma(-q, r, 1.0), r, r);
}
// ln(e^-r I_m(r)), uniform asymptotic (Debye) form; used only to size the expansion
__device__ __forceinline__ double log_scaled_bessel_i(double m, double r) {
  const double s = sqrt(m * m + r * r);
  return -r + s - m * asinh(m / r) - 0.9189385332046727 - 0.25 * log(s * s);
}
__global__ __launch_bounds__(kTPB) void k_ftk_exp(DevState S, int scale) {
  extern __shared__ double sh[];
  __shared__ double red[2][kTPB];
  __shared__ int cnt[2 * kExpShifts];  // Sturm counts: [min end | max end]
  __shared__ int first[2];
  TPL_MARK(0);
  const int n = S.flags[2];
  if (S.flags[1] || n < 1) return;
  const int t = threadIdx.x;
  double* al = sh;            // alpha (n)
  double* b2 = sh + n;        // beta^2 (n - 1), b2[n-1] = 0
  double* buf0 = sh + 2 * n;  // Clenshaw exchange buffers: row i at [i + 1], zeros at both ends
  double* buf1 = buf0 + (n + 2);
  const double bnorm = scale ? S.norms[0] : 1.0;
  // this thread's rows: alpha, the betas on both sides (registers for the whole expansion)
  const int R = (n + kTPB - 1) / kTPB;
  double ra[kExpRows], rbl[kExpRows], rbr[kExpRows];
  double glo = INFINITY, ghi = -INFINITY, bmax = 0.0;
  bool finite = true;
#pragma unroll
  for (int u = 0; u < kExpRows; ++u) {
    const int i = t + u * kTPB;
    ra[u] = rbl[u] = rbr[u] = 0.0;
    if (u < R && i < n) {
      ra[u] = S.alphas[i];
      rbl[u] = i > 0 ? S.betas[i - 1] : 0.0;
      rbr[u] = i + 1 < n ? S.betas[i] : 0.0;
      al[i] = ra[u];
      b2[i] = rbr[u] * rbr[u];
      finite = finite && isfinite(ra[u]) && isfinite(rbr[u]);
      const double rad = fabs(rbl[u]) + fabs(rbr[u]);
      glo = fmin(glo, ra[u] - rad);
      ghi = fmax(ghi, ra[u] + rad);
      bmax = fmax(bmax, rbr[u] * rbr[u]);
    }
  }
  for (int i = t; i < n + 2; i += kTPB) buf0[i] = buf1[i] = 0.0;
  red[0][t] = glo;
  red[1][t] = ghi;
  cnt[t] = finite ? 0 : 1;
  if (t < 2) first[t] = kExpShifts;
  __syncthreads();
  for (int h = kTPB / 2; h > 0; h >>= 1) {
    if (t < h) {
      red[0][t] = fmin(red[0][t], red[0][t + h]);
      red[1][t] = fmax(red[1][t], red[1][t + h]);
      cnt[t] |= cnt[t + h];
    }
    __syncthreads();
  }
  glo = red[0][0];
  ghi = red[1][0];
  const bool bad = cnt[0] != 0;
  __syncthreads();
  red[0][t] = bmax;
  __syncthreads();
  for (int h = kTPB / 2; h > 0; h >>= 1) {
    if (t < h) red[0][t] = fmax(red[0][t], red[0][t + h]);
    __syncthreads();
  }
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, red[0][0]);
  auto fallback = [&]() {
    for (int i = t; i < n; i += kTPB) S.y[i] = 0.0;
    if (t == 0) S.flags[4] = 1;
  };
  if (bad) {
    fallback();
    return;
  }
  if (n == 1) {
    if (t == 0) S.y[0] = exp(al[0]) * bnorm;
    return;
  }
  TPL_MARK(1);
  // One round of Sturm multisection over the Gershgorin interval [glo, ghi]: 512 shifts
  // serve both ends, two independent LDL^T pivot chains per thread (ILP: each chain is a
  // dependent sequence of n reciprocals). lambda_min lies in the bracket ending at the
  // first shift with a count >= 1, lambda_max in the one ending at the first count == n.
  {
    const double w = (ghi - glo) / (double)(kExpShifts + 1);
    double sg[2], q[2];
    int c[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      sg[u] = glo + w * (double)(u * kTPB + t + 1);  // shift s = u * 256 + t
      q[u] = al[0] - sg[u];
      if (fabs(q[u]) < pivmin) q[u] = -pivmin;
      c[u] = q[u] < 0.0;
    }
    for (int i = 1; i < n; ++i) {
      const double ai = al[i], bb = b2[i - 1];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        q[u] = (ai - sg[u]) - bb * rcp_nr(q[u]);
        if (fabs(q[u]) < pivmin) q[u] = -pivmin;
        c[u] += q[u] < 0.0;
      }
    }
    cnt[t] = c[0];
    cnt[t + kTPB] = c[1];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int sidx = u * kTPB + t;
      if (cnt[sidx] >= 1) atomicMin(&first[0], sidx);
      if (cnt[sidx] >= n) atomicMin(&first[1], sidx);
    }
    __syncthreads();
  }
  TPL_MARK(2);
  // [a, b] holds the spectrum: below the shift before lambda_min's first count, above the
  // first shift counting all n, widened by a margin far above a count's backward error
  const double wsh = (ghi - glo) / (double)(kExpShifts + 1);
  const double gmag = fmax(fabs(glo), fabs(ghi));
  const double a = (first[0] > 0 ? glo + wsh * (double)first[0] : glo) - 1e-9 * (1.0 + gmag);
  const double b = (first[1] < kExpShifts ? glo + wsh * (double)(first[1] + 1) : ghi) +
                   1e-9 * (1.0 + gmag);
  const double c = 0.5 * (a + b);
  const double r = fmax(0.5 * (b - a), 1e-30 * (1.0 + fabs(c)));
  const double inv_r = 1.0 / r;
  // terms: the smallest m with e^-r I_m(r) < 1e-22 (asymptotic form, decreasing in m),
  // found in two parallel passes: every thread tests m = 64 t, then the 64 candidates
  // below the first passing one
  {
    __syncthreads();  // every thread has read the brackets out of first[]
    if (t < 2) first[t] = kExpMaxTerms + 1;
    __syncthreads();
    const int m0 = 64 * t;
    if (m0 <= kExpMaxTerms && log_scaled_bessel_i((double)m0, r) < -50.66) atomicMin(&first[0], m0);
    __syncthreads();
    const int hi = first[0];
    if (hi <= kExpMaxTerms && t < 64) {
      const int m1 = hi - 63 + t;
      if (m1 >= 0 && log_scaled_bessel_i((double)m1, r) < -50.66) atomicMin(&first[1], m1);
    }
    __syncthreads();
  }
  if (first[0] > kExpMaxTerms) {
    fallback();
    return;
  }
  const int N = min(first[0], first[1]) + 8;
  TPL_MARK(3);
  // Clenshaw: b_m = a_m e_1 + 2 x b_{m+1} - b_{m+2} (m = N .. 1), x = (T - c I) / r; the
  // result is a_0 e_1 + x b_1 - b_2 with a_0 = I_0, a_m = 2 I_m (unnormalised Miller values)
  double b1[kExpRows], b2v[kExpRows], dia[kExpRows];
#pragma unroll
  for (int u = 0; u < kExpRows; ++u) {
    b1[u] = b2v[u] = 0.0;
    dia[u] = ra[u] - c;
  }
  double Ip1 = 0.0, Im = 1.0, Ssum = 0.0;  // I_{m+1}, I_m (Miller seed), 2 sum_{m'>=m} I_m'
  double* cur = buf0;
  double* nxt = buf1;
  if (n <= 4 * 64) {
    // T_k of at most 256 rows (configs[1]: k = 200): ONE wave runs the recurrence, four
    // consecutive rows per lane, the neighbour rows across lanes by DPP wave shifts — no
    // LDS exchange and no barrier per term. The same operations on the same operands as
    // the general loop below, row by row (zero neighbours at both ends), so the same bits.
    if (t < 64) {
      double f1[4], f2[4], fd[4], fl[4], fr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * t + j;
        const bool ok = i < n;
        fd[j] = ok ? al[i] - c : 0.0;
        fl[j] = (ok && i > 0) ? S.betas[i - 1] : 0.0;
        fr[j] = (ok && i + 1 < n) ? S.betas[i] : 0.0;
        f1[j] = f2[j] = 0.0;
      }
      for (int m = N; m >= 1; --m) {
        const double left = dpp_f64<0x138>(f1[3]);   // wave_shr:1 -> row 4t - 1 (0 at lane 0)
        const double right = dpp_f64<0x130>(f1[0]);  // wave_shl:1 -> row 4t + 4 (0 at lane 63)
        const double am = 2.0 * Im;
        double nv[4];
        nv[0] = ((fl[0] * left + fd[0] * f1[0]) + fr[0] * f1[1]) * inv_r;
        nv[1] = ((fl[1] * f1[0] + fd[1] * f1[1]) + fr[1] * f1[2]) * inv_r;
        nv[2] = ((fl[2] * f1[1] + fd[2] * f1[2]) + fr[2] * f1[3]) * inv_r;
        nv[3] = ((fl[3] * f1[2] + fd[3] * f1[3]) + fr[3] * right) * inv_r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          double v = 2.0 * nv[j] - f2[j];
          if (t == 0 && j == 0) v = v + am;
          f2[j] = f1[j];
          f1[j] = v;
        }
        Ssum = Ssum + am;
        const double Inext = Ip1 + (2.0 * (double)m * inv_r) * Im;
        Ip1 = Im;
        Im = Inext;
        if (fabs(Im) > 1e200) {
          Im *= 1e-200; Ip1 *= 1e-200; Ssum *= 1e-200;
#pragma unroll
          for (int j = 0; j < 4; ++j) { f1[j] *= 1e-200; f2[j] *= 1e-200; }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * t + j;
        if (i < n) {
          cur[i + 1] = f1[j];
          nxt[i + 1] = f2[j];
        }
      }
      if (t == 0) {
        red[1][0] = Im;
        red[1][1] = Ssum;
      }
    }
    __syncthreads();
    Im = red[1][0];
    Ssum = red[1][1];
#pragma unroll
    for (int u = 0; u < kExpRows; ++u) {
      const int i = t + u * kTPB;
      if (u < R && i < n) {
        b1[u] = cur[i + 1];
        b2v[u] = nxt[i + 1];
      }
    }
    __syncthreads();  // every lane has its rows before the tail rewrites cur
  } else
  for (int m = N; m >= 1; --m) {
    // publish b_{m+1}, then every row forms b_m from its neighbours
#pragma unroll
    for (int u = 0; u < kExpRows; ++u) {
      const int i = t + u * kTPB;
      if (u < R && i < n) cur[i + 1] = b1[u];
    }
    __syncthreads();
    const double am = 2.0 * Im;
#pragma unroll
    for (int u = 0; u < kExpRows; ++u) {
      const int i = t + u * kTPB;
      if (u < R && i < n) {
        const double xb = ((rbl[u] * cur[i] + dia[u] * cur[i + 1]) + rbr[u] * cur[i + 2]) * inv_r;
        double v = 2.0 * xb - b2v[u];
        if (i == 0) v = v + am;
        b2v[u] = b1[u];
        b1[u] = v;
      }
    }
    Ssum = Ssum + am;
    const double Inext = Ip1 + (2.0 * (double)m * inv_r) * Im;
    Ip1 = Im;
    Im = Inext;
    if (fabs(Im) > 1e200) {  // Miller's values grow towards m = 0: rescale the whole state
      Im *= 1e-200; Ip1 *= 1e-200; Ssum *= 1e-200;
#pragma unroll
      for (int u = 0; u < kExpRows; ++u) { b1[u] *= 1e-200; b2v[u] *= 1e-200; }
    }
    double* sw = cur; cur = nxt; nxt = sw;  // double buffer: one barrier per term
  }
  TPL_MARK(4);
  // y' = e^b (I_0 e_1 + x b_1 - b_2) / (I_0 + 2 sum I_m)
#pragma unroll
  for (int u = 0; u < kExpRows; ++u) {
    const int i = t + u * kTPB;
    if (u < R && i < n) cur[i + 1] = b1[u];
  }
  __syncthreads();
  const double norm = Ssum + Im;
  const double eb = exp(b);
  double yv[kExpRows];
  double sq = 0.0;
#pragma unroll
  for (int u = 0; u < kExpRows; ++u) {
    const int i = t + u * kTPB;
    yv[u] = 0.0;
    if (u < R && i < n) {
      const double xb = ((rbl[u] * cur[i] + dia[u] * cur[i + 1]) + rbr[u] * cur[i + 2]) * inv_r;
      double v = xb - b2v[u];
      if (i == 0) v = v + Im;
      yv[u] = v / norm;  // exp(T - b I) e_1
      sq = fma(yv[u], yv[u], sq);
    }
  }
  // The expansion's error is a few eps * (terms) in units of e^b; when ||exp(T - bI) e_1||
  // is far below 1 (e_1 nearly orthogonal to the top of the spectrum) that is no longer
  // small against ||y||, while the EVD keeps its relative accuracy: hand such cases back.
  __syncthreads();
  red[0][t] = sq;
  __syncthreads();
  for (int h = kTPB / 2; h > 0; h >>= 1) {
    if (t < h) red[0][t] = red[0][t] + red[0][t + h];
    __syncthreads();
  }
  if (!(red[0][0] >= kExpMinRatio * kExpMinRatio)) {
    fallback();
    return;
  }
#pragma unroll
  for (int u = 0; u < kExpRows; ++u) {
    const int i = t + u * kTPB;
    if (u < R && i < n) S.y[i] = (eb * yv[u]) * bnorm;
  }
  TPL_MARK(5);
  TPL_STAMP_TERMS(N);
}

// Row permutation at the boundary (locality order, tpl_layout.h): out[i] = in[idx[i]] for
// each of `cols` columns (leading dimensions ldo / ldi).
__global__ __launch_bounds__(kTPB) void k_permute(int64_t n, int cols, double* __restrict__ out,
                                                  int64_t ldo, const double* __restrict__ in,
                                                  int64_t ldi, const int32_t* __restrict__ idx) {
  const int c = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kTPB)
    out[(int64_t)c * ldo + i] = in[(int64_t)c * ldi + idx[i]];
}

// ---------------------------------------- replicated long rows (partitioned solve)
// Long row l = sum over ranks, in rank order, of the R partials all-gathered into
// yall[r * y_ld + l]; every rank then runs the row's epilogue (identical bits on all
// ranks). Local index of long row l: A.n - A.n_long + l. Alpha partial (pass one):
// thread t accumulates fma(v, w) over rows t + 256q of its workgroup's range, tree256.
// One row per thread (kLongEpiRows = kTPB). Every load of the launch — the row's own
// vector entries, its R partials (8 in flight at a time, at clamped rows, so every lane
// loads and the adds keep rank order) — is issued before the DevState scalars are read:
// one round trip behind the boundary instead of a scalar one first (round 3).
struct LongSum {
  double t[8];
};
// the first 8 ranks' partials of long row lc (clamped: every lane loads) ...
__device__ __forceinline__ void long_sum_issue(const CsrDev& A, const double* __restrict__ yall,
                                               int R, int lc, LongSum& q) {
#pragma unroll
  for (int u = 0; u < 8; ++u) q.t[u] = yall[(size_t)clampi(u, R - 1) * A.y_ld + lc];
}
// ... summed in rank order; more ranks in batches of 8 loads in flight
__device__ __forceinline__ double long_sum_finish(const CsrDev& A, const double* __restrict__ yall,
                                                  int R, int lc, const LongSum& q) {
  double y = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (u < R) y = y + q.t[u];
  for (int r0 = 8; r0 < R; r0 += 8) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = yall[(size_t)clampi(r0 + u, R - 1) * A.y_ld + lc];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (r0 + u < R) y = y + t[u];
  }
  return y;
}

// Pass one after the exchange: the long rows' epilogue (w, alpha partials) and, in R more
// workgroups, each rank's short-chunk alpha total from its all-gathered chunk partials —
// finish_partials over yall[r * y_ld + n_long ..], the tree k_reorth_reduce applies, so
// the totals are bitwise those a separate rank-total launch before the all-gather made
// (r02/r03; that launch is gone). Pa_long[-R .. -1]: the R totals; Pa_long[b]: block b.
__global__ __launch_bounds__(kTPB) void k_long_epi_p1(CsrDev A, DevState S,
                                                      const double* __restrict__ yall, int R,
                                                      const double* __restrict__ r_cur,
                                                      const double* __restrict__ r_prev,
                                                      double* __restrict__ W,
                                                      double* __restrict__ Vcol,
                                                      double* __restrict__ Pa_long, int j) {
  __shared__ double red[4];
  const int nbl = (A.n_long + kLongEpiRows - 1) / kLongEpiRows;
  if ((int)blockIdx.x >= nbl) {  // rank total (uniform per workgroup)
    const int r = blockIdx.x - nbl;
    const double* P = yall + (size_t)r * A.y_ld + A.n_long;
    const int N = A.nch[r];
    double tot = 0.0;  // a rank without short rows (N == 0, uniform): nothing to load
    if (N > 0) {
      PartialRegs<8> pr;
      load_partials(P, N, pr);
      tot = finish_partials(P, N, pr, red);
    }
    if (threadIdx.x == 0) Pa_long[r - R] = tot;
    return;
  }
  EpiPass1 epi;
  epi.r_cur = r_cur;
  epi.r_prev = (j >= 2) ? r_prev : r_cur;
  epi.has_prev = j >= 2;
  epi.W = W;
  epi.Vcol = Vcol;
  epi.Pa_long = nullptr;
  const int l = blockIdx.x * kLongEpiRows + threadIdx.x;
  const int lc = l < A.n_long ? l : A.n_long - 1;
  const int row = (int)(A.n - A.n_long) + lc;
  const Pre1 pre = epi.pre(row);
  LongSum q;
  long_sum_issue(A, yall, R, lc, q);
  __builtin_amdgcn_sched_barrier(0);
  const int stop = S.flags[0];
  const double beta = S.norms[j - 1];
  const double beta_prev = S.norms[j >= 2 ? j - 2 : 0];
  const double y = long_sum_finish(A, yall, R, lc, q);
  if (stop) return;  // stopped / breakdown (uniform)
  epi.invN_cur = 1.0 / beta;
  epi.invN_prev = (j >= 2) ? 1.0 / beta_prev : 0.0;
  epi.beta_sub = (j >= 2) ? beta : 0.0;
  double acc = 0.0;
  if (l < A.n_long) epi.apply(row, y, pre, acc);
  const double p = block_sum_tail(acc, red);
  if (threadIdx.x == 0) Pa_long[blockIdx.x] = p;
}

__global__ __launch_bounds__(kTPB) void k_long_epi_y(CsrDev A, const double* __restrict__ yall,
                                                     int R, double* __restrict__ y) {
  const int l = blockIdx.x * kLongEpiRows + threadIdx.x;
  const int lc = l < A.n_long ? l : A.n_long - 1;
  LongSum q;
  long_sum_issue(A, yall, R, lc, q);
  const double s = long_sum_finish(A, yall, R, lc, q);
  if (l < A.n_long) st_out(y + (A.n - A.n_long) + l, s);
}

// Pass two after the exchange: the coefficients come from the step's record, loaded
// lane-wise with the row's own entries (EpiPass2R), so nothing waits for a scalar load.
__global__ __launch_bounds__(kTPB) void k_long_epi_p2(CsrDev A, const double* __restrict__ rec,
                                                      const double* __restrict__ yall, int R,
                                                      const double* __restrict__ v_cur,
                                                      const double* __restrict__ v_prev,
                                                      double* __restrict__ v_next,
                                                      double* __restrict__ x,
                                                      double* __restrict__ Vcol, int j,
                                                      int nflush) {
  EpiPass2R epi;
  epi.v_cur = v_cur;
  epi.v_prev = (j >= 2) ? v_prev : v_cur;
  epi.rec = rec;
  epi.has_prev = j >= 2;
  epi.nflush = nflush;
  epi.v_next = v_next;
  epi.x = x;
  epi.Vcol = Vcol;
  const int l = blockIdx.x * kLongEpiRows + threadIdx.x;
  const int lc = l < A.n_long ? l : A.n_long - 1;
  const int row = (int)(A.n - A.n_long) + lc;
  const Pre2R pre = epi.pre(row);
  LongSum q;
  long_sum_issue(A, yall, R, lc, q);
  const double y = long_sum_finish(A, yall, R, lc, q);
  double acc = 0.0;
  if (l < A.n_long) epi.apply(row, y, pre, acc);
}

// One-pass reconstruction x = ||b|| (V_k y') (src/solvers.rs:96-104); V column-major, ld = n.
// steps < 0: steps_taken from the device state (the device-f path, no host round trip).
__global__ __launch_bounds__(kTPB) void k_gemv_recon(int64_t n, int steps, DevState S,
                                                     const double* __restrict__ V,
                                                     double* __restrict__ x) {
  if (steps < 0) {
    if (S.flags[1] || S.flags[4]) return;  // zero b / f handed back to the host
    steps = S.flags[2];
  }
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
constexpr int kReorthCols = 16; // columns per workgroup in the h = V^T r kernel

// h partials: grid (G2, ceil(cols/16)); workgroup (b, g) owns rows [bE, min(n,(b+1)E))
// and columns [16g, 16g+16). P[c*G2 + b] = tree256 of the thread accumulators (thread
// t: acc = fma(V[c][i], r[i], acc) over i = bE + t + 256q, q ascending). Every column's
// load is issued unconditionally (columns past cols re-read column 16g, unused) so the
// 17 loads of an iteration are all in flight; the 16 trees share one barrier.
// skip (selective variant): the second pass is not needed (k_reorth_decide).
__global__ __launch_bounds__(kTPB) void k_reorth_dot(int64_t n, int cols,
                                                     const double* __restrict__ V,
                                                     const double* __restrict__ r,
                                                     double* __restrict__ P, int G, int64_t E,
                                                     const int* __restrict__ skip) {
  __shared__ double red[kReorthCols * 4];
  if (skip && *skip) return;
  const int c0 = blockIdx.y * kReorthCols;
  const int nc = cols - c0 < kReorthCols ? cols - c0 : kReorthCols;
  const int64_t beg = (int64_t)blockIdx.x * E;
  const int64_t end = beg + E < n ? beg + E : n;
  double acc[kReorthCols];
#pragma unroll
  for (int u = 0; u < kReorthCols; ++u) acc[u] = 0.0;
#pragma unroll 2
  for (int64_t i = beg + threadIdx.x; i < end; i += kTPB) {
    const double ri = r[i];
    double v[kReorthCols];
#pragma unroll
    for (int u = 0; u < kReorthCols; ++u) v[u] = V[(int64_t)(c0 + (u < nc ? u : 0)) * n + i];
#pragma unroll
    for (int u = 0; u < kReorthCols; ++u) acc[u] = u < nc ? fma(v[u], ri, acc[u]) : acc[u];
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < kReorthCols; ++u) {
    const double sw = wave_sum(acc[u]);
    if ((threadIdx.x & 63) == 0) red[u * 4 + w] = sw;
  }
  __syncthreads();
  const int u = threadIdx.x;
  if (u < nc)
    P[(int64_t)(c0 + u) * G + blockIdx.x] =
        (red[u * 4 + 0] + red[u * 4 + 1]) + (red[u * 4 + 2] + red[u * 4 + 3]);
}

// h[c] = sum of the G partials of column c (one workgroup per column).
__global__ __launch_bounds__(kTPB) void k_reorth_reduce(const double* __restrict__ P, int G,
                                                        double* __restrict__ h,
                                                        const int* __restrict__ skip) {
  __shared__ double red[4];
  if (skip && *skip) return;
  PartialRegs<8> pr;
  const double* Pc = P + (int64_t)blockIdx.x * G;
  load_partials(Pc, G, pr);
  const double s = finish_partials(Pc, G, pr, red);
  if (threadIdx.x == 0) h[blockIdx.x] = s;
}

// r -= V h ; optional ||r||^2 partials in the canonical norm order (E partition).
// Thread t owns the pairs (i0, i0 + 1), i0 = bE + 2t + 512q, as the norm order does;
// per element s = 0; s = fma(V[c][i], h[c], s) for c ascending. The columns are taken
// kUpdCols at a time with all 2 kUpdCols loads in flight before the ordered FMAs: the
// sweep is a pure HBM stream (V_j does not fit the Infinity Cache at k = 500), so bytes
// in flight per CU, not arithmetic, set its rate.
constexpr int kUpdCols = 16;
__global__ __launch_bounds__(kTPB) void k_reorth_update(int64_t n, int cols,
                                                        const double* __restrict__ V,
                                                        double* __restrict__ r,
                                                        const double* __restrict__ h,
                                                        double* __restrict__ Pnorm, int64_t E,
                                                        const int* __restrict__ skip) {
  __shared__ double red[4];
  if (skip && *skip) return;
  const int64_t beg = (int64_t)blockIdx.x * E;
  const int64_t end = beg + E < n ? beg + E : n;
  double acc = 0.0;
  for (int64_t i0 = beg + 2 * threadIdx.x; i0 < end; i0 += 2 * kTPB) {
    const bool has1 = i0 + 1 < end;
    const int64_t i1 = has1 ? i0 + 1 : i0;
    const double r0 = r[i0], r1 = r[i1];
    double s0 = 0.0, s1 = 0.0;
    int c = 0;
    for (; c + kUpdCols <= cols; c += kUpdCols) {
      double v0[kUpdCols], v1[kUpdCols];
#pragma unroll
      for (int u = 0; u < kUpdCols; ++u) {
        const double* col = V + (int64_t)(c + u) * n;
        v0[u] = col[i0];
        v1[u] = col[i1];
      }
#pragma unroll
      for (int u = 0; u < kUpdCols; ++u) {
        s0 = fma(v0[u], h[c + u], s0);
        s1 = fma(v1[u], h[c + u], s1);
      }
    }
    for (; c < cols; ++c) {
      const double* col = V + (int64_t)c * n;
      s0 = fma(col[i0], h[c], s0);
      s1 = fma(col[i1], h[c], s1);
    }
    const double q0 = r0 - s0;
    r[i0] = q0;
    acc = fma(q0, q0, acc);
    if (has1) {
      const double q1 = r1 - s1;
      r[i1] = q1;
      acc = fma(q1, q1, acc);
    }
  }
  if (Pnorm) {
    const double p = block_sum(acc, red);
    if (threadIdx.x == 0) Pnorm[blockIdx.x] = p;
  }
}

// Selective re-orthogonalisation (Kahan–Parlett "twice is enough"): after the first
// projection r' = r - V h, the second one is needed only when it removed more than half
// of r's squared norm. n0 = ||r||^2 (the partials k_p1_axpy left in S.Pb), n1 = ||r'||^2
// (Pb1, written by the first update), both reduced in the canonical norm order; if
// n1 >= n0 / 2 the second pass is skipped and r' is the result — its partials become the
// ones k_p1_spmv reduces for beta — else S.flags[3] counts a second pass. rec: this
// step's slot of the per-step record (1: a second pass ran), so the host can count only
// the steps a caller keeps (a step callback may stop before the device's last step).
// One workgroup.
__global__ __launch_bounds__(kTPB) void k_reorth_decide(DevState S, const double* __restrict__ Pb1,
                                                        int G2, int* __restrict__ skip,
                                                        int* __restrict__ rec) {
  __shared__ double red[4];
  PartialRegs<4> p0, p1;  // G2 <= 1024
  load_partials(S.Pb, G2, p0);
  load_partials(Pb1, G2, p1);
  const double n0 = finish_partials(S.Pb, G2, p0, red);
  const double n1 = finish_partials(Pb1, G2, p1, red);
  const bool sk = n1 >= 0.5 * n0;
  if (sk)
    for (int i = threadIdx.x; i < G2; i += kTPB) S.Pb[i] = Pb1[i];
  if (threadIdx.x == 0) {
    *skip = sk ? 1 : 0;
    *rec = sk ? 0 : 1;
    if (!sk) S.flags[3] = S.flags[3] + 1;
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
// chunk part: 8 XCDs x the largest eighth of the row blocks x chunks per row block
static inline int spmv_grid(const CsrDev& A) {
  return A.n_slice_blocks + 8 * ((A.G2 + 7) / 8) * (int)(A.E / kChunkRows);
}
// element-wise kernels over the G2 row blocks (elem_block)
static inline int g2_grid(const CsrDev& A) { return 8 * ((A.G2 + 7) / 8); }
// dynamic LDS of the SpMV-shaped kernels: a bin's staged products + piece starts
static inline size_t spmv_lds_bytes(const CsrDev& A) {
  const size_t bins = A.n_slice_blocks > 0
             ? (size_t)A.bin_cap * sizeof(double) + kTPB * sizeof(int) + kTPB * sizeof(double)
             : 0;
  const size_t win = (size_t)A.s_win * sizeof(double);  // short-chunk column window
  return bins > win ? bins : win;
}
// Launch the SpMV-shaped kernel specialised for the layout's uniform chunk width.
#define TPL_LAUNCH_CASE(KERNEL, F)                                                          \
  case F: hipLaunchKernelGGL(KERNEL<F>, grid_, block_, shm_, s_, args_...); break
// Launch the SpMV-shaped kernel specialised for the layout (chunk width, value format).
#define TPL_LAUNCH_CW(KERNEL, A, s, ...)                                                    \
  [&](auto... args_) {                                                                     \
    const dim3 grid_(spmv_grid(A)), block_(kTPB);                                           \
    const size_t shm_ = spmv_lds_bytes(A);                                                  \
    hipStream_t s_ = (s);                                                                   \
    const int cw_ = (A).s_width >= 1 && (A).s_width <= 4 ? (A).s_width : 0;                \
    switch (cw_ | ((A).val_i8 ? 8 : 0) | ((A).s_col16 ? 16 : 0) | ((A).b_col16 ? 32 : 0) |  \
            ((A).s_win > 0 && cw_ > 0 && (A).s_col16 ? 64 : 0)) {                            \
      TPL_LAUNCH_CASE(KERNEL, 0); TPL_LAUNCH_CASE(KERNEL, 32); TPL_LAUNCH_CASE(KERNEL, 16); TPL_LAUNCH_CASE(KERNEL, 48);\
      TPL_LAUNCH_CASE(KERNEL, 8); TPL_LAUNCH_CASE(KERNEL, 40); TPL_LAUNCH_CASE(KERNEL, 24); TPL_LAUNCH_CASE(KERNEL, 56);\
      TPL_LAUNCH_CASE(KERNEL, 1); TPL_LAUNCH_CASE(KERNEL, 33); TPL_LAUNCH_CASE(KERNEL, 17); TPL_LAUNCH_CASE(KERNEL, 49);\
      TPL_LAUNCH_CASE(KERNEL, 9); TPL_LAUNCH_CASE(KERNEL, 41); TPL_LAUNCH_CASE(KERNEL, 25); TPL_LAUNCH_CASE(KERNEL, 57);\
      TPL_LAUNCH_CASE(KERNEL, 2); TPL_LAUNCH_CASE(KERNEL, 34); TPL_LAUNCH_CASE(KERNEL, 18); TPL_LAUNCH_CASE(KERNEL, 50);\
      TPL_LAUNCH_CASE(KERNEL, 10); TPL_LAUNCH_CASE(KERNEL, 42); TPL_LAUNCH_CASE(KERNEL, 26); TPL_LAUNCH_CASE(KERNEL, 58);\
      TPL_LAUNCH_CASE(KERNEL, 3); TPL_LAUNCH_CASE(KERNEL, 35); TPL_LAUNCH_CASE(KERNEL, 19); TPL_LAUNCH_CASE(KERNEL, 51);\
      TPL_LAUNCH_CASE(KERNEL, 11); TPL_LAUNCH_CASE(KERNEL, 43); TPL_LAUNCH_CASE(KERNEL, 27); TPL_LAUNCH_CASE(KERNEL, 59);\
      TPL_LAUNCH_CASE(KERNEL, 4); TPL_LAUNCH_CASE(KERNEL, 36); TPL_LAUNCH_CASE(KERNEL, 20); TPL_LAUNCH_CASE(KERNEL, 52);\
      TPL_LAUNCH_CASE(KERNEL, 12); TPL_LAUNCH_CASE(KERNEL, 44); TPL_LAUNCH_CASE(KERNEL, 28); TPL_LAUNCH_CASE(KERNEL, 60);\
      TPL_LAUNCH_CASE(KERNEL, 81); TPL_LAUNCH_CASE(KERNEL, 82); TPL_LAUNCH_CASE(KERNEL, 83); TPL_LAUNCH_CASE(KERNEL, 84);\
      TPL_LAUNCH_CASE(KERNEL, 89); TPL_LAUNCH_CASE(KERNEL, 90); TPL_LAUNCH_CASE(KERNEL, 91); TPL_LAUNCH_CASE(KERNEL, 92);\
      TPL_LAUNCH_CASE(KERNEL, 113); TPL_LAUNCH_CASE(KERNEL, 114); TPL_LAUNCH_CASE(KERNEL, 115); TPL_LAUNCH_CASE(KERNEL, 116);\
      TPL_LAUNCH_CASE(KERNEL, 121); TPL_LAUNCH_CASE(KERNEL, 122); TPL_LAUNCH_CASE(KERNEL, 123); TPL_LAUNCH_CASE(KERNEL, 124);\
      default: return hipErrorInvalidConfiguration; /* no instance for this layout */    \
    }                                                                                       \
    return hipGetLastError();                                                               \
  }(__VA_ARGS__)

hipError_t spmv(const CsrDev& A, const double* x, double* y, hipStream_t s) {
  if (spmv_grid(A) > 0) return TPL_LAUNCH_CW(k_spmv, A, s, A, x, y);
  return hipGetLastError();
}
hipError_t p1_init(const CsrDev& A, const DevState& S, const double* b, hipStream_t s) {
  hipLaunchKernelGGL(k_p1_init, dim3(g2_grid(A)), dim3(kTPB), 0, s, A, S, b);
  return hipGetLastError();
}
hipError_t p1_spmv(const CsrDev& A, const DevState& S, const double* xsrc, const double* r_cur,
                   const double* r_prev, double* W, double* Vcol, int j, hipStream_t s,
                   unsigned long long* stamp) {
  if (spmv_grid(A) <= 0) return hipGetLastError();
  if (A.pb_ld > 0)
    return TPL_LAUNCH_CW(k_p1_spmv_gp, A, s, A, S, xsrc, r_cur, r_prev, W, Vcol, j, stamp);
  if (A.G2_r <= kTPB)
    return TPL_LAUNCH_CW(k_p1_spmv, A, s, A, S, xsrc, r_cur, r_prev, W, Vcol, j, stamp);
  return TPL_LAUNCH_CW(k_p1_spmv_wide, A, s, A, S, xsrc, r_cur, r_prev, W, Vcol, j, stamp);
  return hipGetLastError();
}
hipError_t p1_axpy(const CsrDev& A, const DevState& S, const double* W, const double* r_cur,
                   double* r_next, int j, int k, int elim, hipStream_t s,
                   unsigned long long* st) {
  const dim3 g(g2_grid(A) + (elim ? 1 : 0)), b(kTPB);
  if (A.NA_r <= 2 * kTPB)
    hipLaunchKernelGGL(k_p1_axpy<2>, g, b, 0, s, A, S, W, r_cur, r_next, j, k, elim, st);
  else if (A.NA_r <= 4 * kTPB)
    hipLaunchKernelGGL(k_p1_axpy<4>, g, b, 0, s, A, S, W, r_cur, r_next, j, k, elim, st);
  else if (A.NA_r <= 8 * kTPB)
    hipLaunchKernelGGL(k_p1_axpy<8>, g, b, 0, s, A, S, W, r_cur, r_next, j, k, elim, st);
  else
    hipLaunchKernelGGL(k_p1_axpy<12>, g, b, 0, s, A, S, W, r_cur, r_next, j, k, elim, st);
  return hipGetLastError();
}
hipError_t p2_init(int64_t n, const DevState& S, const double* b, double* v1, double* x,
                   double* Vcol, int dyn, hipStream_t s) {
  hipLaunchKernelGGL(k_p2_init, dim3(elem_grid(n)), dim3(kTPB), 0, s, n, S, b, v1, x, Vcol, dyn);
  return hipGetLastError();
}
hipError_t permute(int64_t n, int cols, double* out, int64_t ldo, const double* in, int64_t ldi,
                   const int32_t* idx, hipStream_t s) {
  for (int c0 = 0; n > 0 && c0 < cols; c0 += 65535) {
    const int c = std::min(cols - c0, 65535);
    hipLaunchKernelGGL(k_permute, dim3(elem_grid(n), c), dim3(kTPB), 0, s, n, c,
                       out + (int64_t)c0 * ldo, ldo, in + (int64_t)c0 * ldi, ldi, idx);
  }
  return hipGetLastError();
}
hipError_t p2_tail(int64_t n, const DevState& S, double* x, double* const V[3], hipStream_t s) {
  hipLaunchKernelGGL(k_p2_tail, dim3(elem_grid(n)), dim3(kTPB), 0, s, n, S, x, V[0], V[1], V[2]);
  return hipGetLastError();
}
hipError_t ftk_inv(const DevState& S, int kcap, int scale, hipStream_t s) {
  hipLaunchKernelGGL(k_ftk_inv, dim3(1), dim3(kTPB), (size_t)11 * kcap * sizeof(double), s, S, scale);
  return hipGetLastError();
}
hipError_t ftk_exp(const DevState& S, int kcap, int scale, hipStream_t s) {
  hipLaunchKernelGGL(k_ftk_exp, dim3(1), dim3(kTPB), (size_t)(4 * kcap + 4) * sizeof(double), s, S,
                     scale);
  return hipGetLastError();
}
hipError_t p2_spmv(const CsrDev& A, const DevState& S, const double* xsrc, const double* v_cur,
                   const double* v_prev, double* v_next, double* x, double* Vcol, int j,
                   int nflush, hipStream_t s) {
  if (spmv_grid(A) > 0)
    return TPL_LAUNCH_CW(k_p2_spmv, A, s, A, S.p2c + 8 * (size_t)j, xsrc, v_cur, v_prev, v_next,
                         x, Vcol, j, nflush);
  return hipGetLastError();
}
hipError_t p2_coefs(const DevState& S, int k, int dyn, hipStream_t s) {
  if (k > 1)
    hipLaunchKernelGGL(k_p2_coefs, dim3((k + kTPB - 1) / kTPB), dim3(kTPB), 0, s, S, k, dyn);
  return hipGetLastError();
}
int long_epi_blocks(const CsrDev& A) { return (A.n_long + kLongEpiRows - 1) / kLongEpiRows; }
hipError_t long_epi_p1(const CsrDev& A, const DevState& S, const double* yall, int R,
                       const double* r_cur, const double* r_prev, double* W, double* Vcol,
                       double* Pa_long, int j, hipStream_t s) {
  // the long rows' blocks, then one workgroup per rank for the short-chunk alpha totals
  hipLaunchKernelGGL(k_long_epi_p1, dim3(long_epi_blocks(A) + R), dim3(kTPB), 0, s, A, S, yall,
                     R, r_cur, r_prev, W, Vcol, Pa_long, j);
  return hipGetLastError();
}
hipError_t long_epi_y(const CsrDev& A, const double* yall, int R, double* y, hipStream_t s) {
  if (A.n_long > 0)
    hipLaunchKernelGGL(k_long_epi_y, dim3(long_epi_blocks(A)), dim3(kTPB), 0, s, A, yall, R, y);
  return hipGetLastError();
}
hipError_t long_epi_p2(const CsrDev& A, const DevState& S, const double* yall, int R,
                       const double* v_cur, const double* v_prev, double* v_next, double* x,
                       double* Vcol, int j, int nflush, hipStream_t s) {
  if (A.n_long > 0)
    hipLaunchKernelGGL(k_long_epi_p2, dim3(long_epi_blocks(A)), dim3(kTPB), 0, s, A,
                       S.p2c + 8 * (size_t)j, yall, R, v_cur, v_prev, v_next, x, Vcol, j, nflush);
  return hipGetLastError();
}
hipError_t gemv_recon(int64_t n, int steps, const DevState& S, const double* V, double* x,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_gemv_recon, dim3(elem_grid(n)), dim3(kTPB), 0, s, n, steps, S, V, x);
  return hipGetLastError();
}
hipError_t reorth_dot(int64_t n, int cols, const double* V, const double* r, double* P, int G,
                      int64_t E, const int* skip, hipStream_t s) {
  dim3 grid(G, (cols + kReorthCols - 1) / kReorthCols);
  hipLaunchKernelGGL(k_reorth_dot, grid, dim3(kTPB), 0, s, n, cols, V, r, P, G, E, skip);
  return hipGetLastError();
}
hipError_t reorth_reduce(int cols, const double* P, int G, double* h, const int* skip,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_reorth_reduce, dim3(cols), dim3(kTPB), 0, s, P, G, h, skip);
  return hipGetLastError();
}
hipError_t reorth_update(int64_t n, int cols, const double* V, double* r, const double* h,
                         double* Pnorm, int G, int64_t E, const int* skip, hipStream_t s) {
  hipLaunchKernelGGL(k_reorth_update, dim3(G), dim3(kTPB), 0, s, n, cols, V, r, h, Pnorm, E,
                     skip);
  return hipGetLastError();
}
hipError_t reorth_decide(const DevState& S, const double* Pb1, int G2, int* skip, int* rec,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_reorth_decide, dim3(1), dim3(kTPB), 0, s, S, Pb1, G2, skip, rec);
  return hipGetLastError();
}

} // namespace launch
} // namespace tpl
