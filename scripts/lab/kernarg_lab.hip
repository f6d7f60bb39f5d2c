// Lab: does kernarg preload (gfx950 user-SGPR preload, -mllvm
// -amdgpu-kernarg-preload-count=N) shorten a dependent kernel boundary? Two kernels
// alternate in one hipGraph, as k_p1_spmv / k_p1_axpy do: a 1,536-workgroup streaming
// kernel and a 245-workgroup element-wise one. Variant S passes a 384-B struct by value
// (no preload possible: the runtime's CsrDev shape); variant P passes the same pointers and
// sizes as leading scalar arguments (preloaded into SGPRs at dispatch). Time per pair over
// 2,000 pairs, HIP events, alternated 5 times.
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=16 kernarg_lab.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big {
  double* a;
  double* b;
  double* c;
  long n;
  long pad[44];
};

__global__ __launch_bounds__(256) void k_stream_s(Big s) {
  const long i0 = (long)blockIdx.x * 512 + threadIdx.x;
  for (long i = i0; i < i0 + 512 && i < s.n; i += 256) s.b[i] = s.a[i] * 1.0000001 + s.c[i];
}
__global__ __launch_bounds__(256) void k_elem_s(Big s) {
  const long i0 = (long)blockIdx.x * 2048 + threadIdx.x;
  for (long i = i0; i < i0 + 2048 && i < s.n; i += 256) s.c[i] = s.b[i] - 0.5 * s.a[i];
}
__global__ __launch_bounds__(256) void k_stream_p(double* a, double* b, double* c, long n) {
  const long i0 = (long)blockIdx.x * 512 + threadIdx.x;
  for (long i = i0; i < i0 + 512 && i < n; i += 256) b[i] = a[i] * 1.0000001 + c[i];
}
__global__ __launch_bounds__(256) void k_elem_p(double* a, double* b, double* c, long n) {
  const long i0 = (long)blockIdx.x * 2048 + threadIdx.x;
  for (long i = i0; i < i0 + 2048 && i < n; i += 256) c[i] = b[i] - 0.5 * a[i];
}

int main() {
  const long n = 501155;
  double *a, *b, *c;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&c, n * 8));
  CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8)); CK(hipMemset(c, 0, n * 8));
  Big s{};
  s.a = a; s.b = b; s.c = c; s.n = n;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int g1 = (int)((n + 511) / 512), g2 = (int)((n + 2047) / 2048), pairs = 2000;
  hipGraphExec_t ex[2];
  for (int v = 0; v < 2; ++v) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int p = 0; p < pairs; ++p) {
      if (v == 0) {
        k_stream_s<<<g1, 256, 0, st>>>(s);
        k_elem_s<<<g2, 256, 0, st>>>(s);
      } else {
        k_stream_p<<<g1, 256, 0, st>>>(a, b, c, n);
        k_elem_p<<<g2, 256, 0, st>>>(a, b, c, n);
      }
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ex[v], g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int v = 0; v < 2; ++v) CK(hipGraphLaunch(ex[v], st));
  CK(hipStreamSynchronize(st));
  for (int rep = 0; rep < 5; ++rep)
    for (int v = 0; v < 2; ++v) {
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ex[v], st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("%s pair %.3f us\n", v == 0 ? "struct " : "scalars", 1000.0 * ms / pairs);
    }
  return 0;
}
