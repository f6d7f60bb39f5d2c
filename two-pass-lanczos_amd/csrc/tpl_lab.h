// tpl_lab.h — diagnostic instrumentation of the kernels, compiled in only by the stamp
// build (scripts/diag.sh: -DTPL_STAMP=1). In the product build every hook is empty.
#pragma once
#include <hip/hip_runtime.h>

namespace tpl {

#ifndef TPL_STAMP
#define TPL_STAMP 0
#endif
#if TPL_STAMP
// Diagnostic builds only: per-workgroup s_memrealtime (100 MHz) marks of the most
// recent SpMV-shaped launch — [0] start, [1] scale known, [2] products staged /
// row sums done, [3] piece sums staged, [4] publish drained, [5] end — read back
// by tpl_debug_stamps().
constexpr int kMarks = 9;  // marks 0..5, the workgroup's HW_ID / XCC_ID in slot 6, marks 7..8
__device__ unsigned long long g_stamps[kMarks * 65536];
__device__ int g_stamps_n;  // k_ftk_exp: the expansion's term count of the last launch
#define TPL_MARK(k)                                                          \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 65536)                              \
      g_stamps[kMarks * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TPL_MARK_ID()                                                        \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 65536) {                            \
      unsigned hw_, xcc_;                                                    \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));     \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc_)); \
      g_stamps[kMarks * blockIdx.x + 6] = ((unsigned long long)xcc_ << 32) | hw_; \
    }                                                                        \
  } while (0)
// marks of a kernel that runs beside an SpMV-shaped one (k_p1_axpy): its own rows of the
// table, kAxpyMarkBase on
constexpr int kAxpyMarkBase = 60000;
#define TPL_MARK_AT(base, k)                                                 \
  do {                                                                       \
    if (threadIdx.x == 0 && (base) + blockIdx.x < 65536)                     \
      g_stamps[kMarks * ((base) + blockIdx.x) + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// the workgroup's very first instruction (before any kernel-argument load): tells a late
// dispatch from a late start of the marked code
__device__ unsigned long long g_first[65536];
#define TPL_MARK_FIRST()                                                     \
  do {                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();          \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_first[blockIdx.x] = t_;    \
    __builtin_amdgcn_sched_barrier(0);                                       \
  } while (0)
#else
#define TPL_MARK(k) do {} while (0)
#define TPL_MARK_ID() do {} while (0)
#define TPL_MARK_AT(base, k) do {} while (0)
#define TPL_MARK_FIRST() do {} while (0)
#endif

// k_ftk_exp: record the expansion's term count (stamp build only)
#if TPL_STAMP
#define TPL_STAMP_TERMS(N)       \
  do {                           \
    if (threadIdx.x == 0) g_stamps_n = (N); \
  } while (0)
#else
#define TPL_STAMP_TERMS(N) do {} while (0)
#endif

} // namespace tpl

#if TPL_STAMP
extern "C" int tpl_debug_stamps(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tpl::g_stamps),
                                  sizeof(unsigned long long) * tpl::kMarks * n);
}
extern "C" int tpl_debug_first(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tpl::g_first), sizeof(unsigned long long) * n);
}
extern "C" int tpl_debug_exp_terms(int* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tpl::g_stamps_n), sizeof(int));
}
#endif
