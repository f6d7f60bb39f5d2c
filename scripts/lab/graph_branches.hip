// Lab: does a hipGraph run two independent branches (captured on forked streams)
// concurrently? Two kernels of 8 workgroups each busy-wait ~T us on the wall clock
// (s_memrealtime, 100 MHz); the graph takes ~T if the branches overlap, ~2T if not.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void spin(long ticks, int* out) {
  const long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;  // vector store
}
int main() {
  const long T = 5000;  // 50 us at 100 MHz
  int* d;
  CK(hipMalloc(&d, 1024 * sizeof(int)));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t fork, join, e0, e1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {  // 0: forked branches, 1: one stream
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
    for (int rep = 0; rep < 10; ++rep) {
      if (mode == 0) {
        CK(hipEventRecord(fork, a));
        CK(hipStreamWaitEvent(b, fork, 0));
        hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, T, d);
        hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, b, T, d + 512);
        CK(hipEventRecord(join, b));
        CK(hipStreamWaitEvent(a, join, 0));
      } else {
        hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, T, d);
        hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, T, d + 512);
      }
    }
    CK(hipStreamEndCapture(a, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, a));
    CK(hipStreamSynchronize(a));
    CK(hipEventRecord(e0, a));
    CK(hipGraphLaunch(ge, a));
    CK(hipEventRecord(e1, a));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s: %.1f us per pair of 50-us kernels\n", mode == 0 ? "forked branches" : "one stream", ms * 100.0);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
