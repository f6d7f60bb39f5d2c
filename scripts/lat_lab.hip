// lat_lab.hip — per-kernel fixed costs and dependent-load round trips on MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void k_empty(double* y) { if (threadIdx.x == 1023) y[0] = 1; }
__global__ void k_copy(int n, const double* __restrict__ x, double* __restrict__ y) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i < n) y[i] = x[i] * 2.0; }
// chain of D dependent loads (index chasing through idx), then store
template <int D>
__global__ void k_chain(int n, const int* __restrict__ idx, const double* __restrict__ x, double* __restrict__ y) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
  int j = i;
#pragma unroll
  for (int d = 0; d < D; ++d) j = idx[j];
  y[i] = x[j];
}
// SELL width-2 short rows: entry k of row i at k*n + i (column-major), gather, store
__global__ void k_sell2(int n, const int* __restrict__ c, const double* __restrict__ v, const double* __restrict__ x, double* __restrict__ y) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
  int c0 = c[i], c1 = c[n + i]; double a0 = v[i], a1 = v[n + i];
  double s = 0.0; s = s + a0 * x[c0]; s = s + a1 * x[c1]; y[i] = s; }
// same + epilogue-style extra loads (2 vectors) and a 2nd store
__global__ void k_sell2_epi(int n, const int* __restrict__ c, const double* __restrict__ v, const double* __restrict__ x,
                            const double* __restrict__ r1, const double* __restrict__ r2, double* __restrict__ y, double* __restrict__ p, int* __restrict__ flag) {
  int i = blockIdx.x * 256 + threadIdx.x;
  int f = flag[0];
  if (i >= n) return;
  int c0 = c[i], c1 = c[n + i]; double a0 = v[i], a1 = v[n + i];
  double q1 = r1[i], q2 = r2[i];
  double s = 0.0; s = s + a0 * x[c0]; s = s + a1 * x[c1];
  if (f) return;
  double w = s - 0.5 * q2; y[i] = w; if ((i & 255) == 0) p[i >> 8] = w * q1; }

int main() {
  const int n = 500000, m = 1155;
  std::vector<int> idx(n), c(2 * n); std::vector<double> x(n, 1.0);
  for (int i = 0; i < n; ++i) { idx[i] = (int)((i * 2654435761u) % n); c[i] = n - m + (i * 7) % m; c[n + i] = n - m + (i * 13 + 5) % m; }
  int *d_idx, *d_c, *d_flag; double *d_x, *d_y, *d_v, *d_r1, *d_r2, *d_p;
  CK(hipMalloc(&d_idx, 4 * n)); CK(hipMalloc(&d_c, 8 * n)); CK(hipMalloc(&d_x, 8 * n)); CK(hipMalloc(&d_y, 8 * n));
  CK(hipMalloc(&d_v, 16 * n)); CK(hipMalloc(&d_r1, 8 * n)); CK(hipMalloc(&d_r2, 8 * n)); CK(hipMalloc(&d_p, 8 * n)); CK(hipMalloc(&d_flag, 64));
  CK(hipMemset(d_flag, 0, 64));
  CK(hipMemcpy(d_idx, idx.data(), 4 * n, hipMemcpyHostToDevice)); CK(hipMemcpy(d_c, c.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_x, x.data(), 8 * n, hipMemcpyHostToDevice)); CK(hipMemcpy(d_v, x.data(), 8 * n, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto bench = [&](const char* name, auto launch) {
    for (int r = 0; r < 5; ++r) launch();
    CK(hipDeviceSynchronize());
    const int iters = 300; CK(hipEventRecord(e0)); for (int r = 0; r < iters; ++r) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-32s %8.2f us/launch (events, back-to-back)\n", name, 1000.0 * ms / iters); };
  int g = (n + 255) / 256;
  bench("empty g=1", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, d_y); });
  bench("empty g=1956", [&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, d_y); });
  bench("copy 4MB", [&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, n, d_x, d_y); });
  bench("chain D=1", [&] { hipLaunchKernelGGL(k_chain<1>, dim3(g), dim3(256), 0, 0, n, d_idx, d_x, d_y); });
  bench("chain D=2", [&] { hipLaunchKernelGGL(k_chain<2>, dim3(g), dim3(256), 0, 0, n, d_idx, d_x, d_y); });
  bench("chain D=4", [&] { hipLaunchKernelGGL(k_chain<4>, dim3(g), dim3(256), 0, 0, n, d_idx, d_x, d_y); });
  bench("chain D=8", [&] { hipLaunchKernelGGL(k_chain<8>, dim3(g), dim3(256), 0, 0, n, d_idx, d_x, d_y); });
  bench("sell2 arc rows", [&] { hipLaunchKernelGGL(k_sell2, dim3(g), dim3(256), 0, 0, n, d_c, d_v, d_x, d_y); });
  bench("sell2 arc rows + epilogue", [&] { hipLaunchKernelGGL(k_sell2_epi, dim3(g), dim3(256), 0, 0, n, d_c, d_v, d_x, d_r1, d_r2, d_y, d_p, d_flag); });
  // two different kernels alternating (as in a real chain)
  bench("copy + empty alternating (per pair)", [&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, n, d_x, d_y);
                                                     hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, d_y); });
  // graph of 100 copies
  hipStream_t s; CK(hipStreamCreate(&s)); hipGraph_t gr; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int r = 0; r < 100; ++r) hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s, n, d_x, d_y);
  CK(hipStreamEndCapture(s, &gr)); CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s)); for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s)); CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); printf("%-32s %8.2f us/launch (graph of 100)\n", "copy 4MB graph", 1000.0 * ms / 1000);
  hipGraph_t gr2; hipGraphExec_t ge2;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int r = 0; r < 100; ++r) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, s, d_y);
  CK(hipStreamEndCapture(s, &gr2)); CK(hipGraphInstantiate(&ge2, gr2, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge2, s)); CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s)); for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge2, s)); CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1)); printf("%-32s %8.2f us/launch (graph of 100)\n", "empty graph", 1000.0 * ms / 1000);
  return 0;
}
