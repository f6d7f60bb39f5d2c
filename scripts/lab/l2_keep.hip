// Does an XCD's L2 keep lines written by the previous kernel on that XCD? (dev lab)
// K_write: block b writes piece b (PIECE doubles) of B, plain or sc1 stores, and records
// its XCC id. K_read: block b reads the pieces written on XCD (own + shift) % 8 — its own
// XCD's pieces (shift 0) or another XCD's (shift 1). Times K_read over many rounds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int NB = 1024, TPB = 256, PIECE = 4096;  // 1024 x 32 KB = 32 MB (4 MB per XCD)
__device__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}
template <int WT>
__global__ void k_write(double* B, int* xcc, double val) {
  const int b = blockIdx.x;
  if (threadIdx.x == 0) xcc[b] = xcc_id();
  for (int i = threadIdx.x; i < PIECE; i += TPB) {
    double* p = B + (size_t)b * PIECE + i;
    if (WT) __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(val + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = val + i;
  }
}
// Block b reads the (b / 8)-th piece written on XCD (own + shift) % 8 in the most
// recent k_write (its xcc[] record), found by wave 0 with ballots.
__global__ void k_read(const double* B, const int* xcc, int shift, double* out) {
  __shared__ int src_s;
  const int x = (xcc_id() + shift) & 7;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int v[NB / 64];
    for (int c = 0; c < NB / 64; ++c) v[c] = xcc[c * 64 + lane];
    int target = blockIdx.x / 8, count = 0, src = 0;
    bool done = false;
    for (int c = 0; c < NB / 64 && !done; ++c) {
      const unsigned long long m = __ballot((v[c] & 7) == x);
      const int pc = __popcll(m);
      if (count + pc > target) {
        unsigned long long mm = m;
        for (int k = 0; k < target - count; ++k) mm &= mm - 1;
        src = c * 64 + __ffsll((long long)mm) - 1;
        done = true;
      }
      count += pc;
    }
    if (lane == 0) src_s = done ? src : 0;
  }
  __syncthreads();
  double s = 0.0;
  const double* p = B + (size_t)src_s * PIECE;
  for (int i = threadIdx.x; i < PIECE; i += TPB) s += p[i];
  if (s == 12345.678) out[blockIdx.x] = s;
}
int main() {
  double *B, *out; int *xcc;
  CHK(hipMalloc(&B, (size_t)NB * PIECE * 8)); CHK(hipMalloc(&out, NB * 8));
  CHK(hipMalloc(&xcc, NB * 4));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (int wt = 0; wt < 2; ++wt) {
    for (int shift = 0; shift < 2; ++shift) {
      float tot = 0.f; int rounds = 200;
      for (int r = 0; r < rounds + 5; ++r) {
        if (wt) hipLaunchKernelGGL(k_write<1>, dim3(NB), dim3(TPB), 0, 0, B, xcc, (double)r);
        else hipLaunchKernelGGL(k_write<0>, dim3(NB), dim3(TPB), 0, 0, B, xcc, (double)r);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_read, dim3(NB), dim3(TPB), 0, 0, B, xcc, shift, out);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 5) tot += ms;
      }
      printf("wt=%d shift=%d  read 32 MB: %.2f us avg\n", wt, shift, 1000.f * tot / rounds);
    }
  }
  return 0;
}
