// Lab: how long does a workgroup wait for its kernel arguments while the memory system is
// busy? One launch of 1,536 workgroups: the first 544 stream 256 MB (the bins' role), the
// other 992 (the chunks' role) stamp s_memrealtime at their first instruction and again
// once a 384-B argument struct is in SGPRs — read (S) from the kernarg segment, as the
// SpMV kernels take CsrDev, or (D) from a __device__ variable (ordinary device memory,
// no kernel argument at all). Prints
// the percentiles of the wait in us. Graph-launched, as the pass graphs are.
//   hipcc -O3 --offload-arch=gfx950 kernarg_load_lab.hip -o kernarg_load_lab
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big {
  const double* src;
  double* dst;
  unsigned long long* out;
  long n;
  long f[44];
};

__device__ __forceinline__ void busy(const double* src, double* dst, long n) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += 544L * 256) s += src[i];
  if (s == 12345.0) dst[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_arg(Big b) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::"s"(b.src), "s"(b.dst), "s"(b.out), "s"(b.n), "s"(b.f[0]), "s"(b.f[20]), "s"(b.f[43]));
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x < 544) { busy(b.src, b.dst, b.n); return; }
  if (threadIdx.x == 0) b.out[blockIdx.x - 544] = t1 - t0 + (unsigned long long)(b.f[0] + b.f[20] + b.f[43]);
}

__device__ Big g_big;  // ordinary device memory, addressed without any kernel argument
__global__ __launch_bounds__(256) void k_ptr() {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_sched_barrier(0);
  const Big b = g_big;
  unsigned long long* out = b.out;
  asm volatile("" ::"s"(b.src), "s"(b.dst), "s"(b.out), "s"(b.n), "s"(b.f[0]), "s"(b.f[20]), "s"(b.f[43]));
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x < 544) { busy(b.src, b.dst, b.n); return; }
  if (threadIdx.x == 0) out[blockIdx.x - 544] = t1 - t0 + (unsigned long long)(b.f[0] + b.f[20] + b.f[43]);
}

static void pct(const char* name, std::vector<unsigned long long>& v) {
  std::sort(v.begin(), v.end());
  auto at = [&](double q) { return v[(size_t)(q * (v.size() - 1))] / 100.0; };
  std::printf("%s wait us: p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", name, at(0), at(0.5), at(0.9), at(1.0));
}

int main() {
  const long n = 32L << 20;  // 256 MB of doubles
  double *src, *dst;
  unsigned long long* out;
  CK(hipMalloc(&src, n * 8)); CK(hipMalloc(&dst, 4096)); CK(hipMalloc(&out, 992 * 8));
  CK(hipMemset(src, 0, n * 8));
  Big b{};
  b.src = src; b.dst = dst; b.out = out; b.n = n;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_big), &b, sizeof(Big)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipGraphExec_t ex[2];
  for (int v = 0; v < 2; ++v) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < 4; ++r) {
      if (v == 0) k_arg<<<1536, 256, 0, st>>>(b);
      else k_ptr<<<1536, 256, 0, st>>>();
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ex[v], g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
  }
  std::vector<unsigned long long> h(992);
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 2; ++v) {
      CK(hipGraphLaunch(ex[v], st));
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(h.data(), out, 992 * 8, hipMemcpyDeviceToHost));
      pct(v == 0 ? "kernarg struct " : "device pointer ", h);
    }
  return 0;
}
