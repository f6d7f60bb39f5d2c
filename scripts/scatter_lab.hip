#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
__global__ void k_gather(int n, const int* __restrict__ idx, const double* __restrict__ x, double* __restrict__ y) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i < n) y[i] = x[idx[i]]; }
__global__ void k_scatter(int n, const int* __restrict__ idx, const double* __restrict__ x, double* __restrict__ y) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i < n) y[idx[i]] = x[i]; }
__global__ void k_copy(int n, const double* __restrict__ x, double* __restrict__ y) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i < n) y[i] = x[i]; }
int main() {
  const int N = 1 << 20;            // 1M entries (8 MB)
  std::vector<int> perm(N); for (int i = 0; i < N; ++i) perm[i] = i;
  std::mt19937 rng(1); std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<int> half(N); for (int i = 0; i < N; ++i) half[i] = (i & 1) ? perm[i] : i;  // half random
  int *d_p, *d_h; double *d_x, *d_y;
  CK(hipMalloc(&d_p, 4 * N)); CK(hipMalloc(&d_h, 4 * N)); CK(hipMalloc(&d_x, 8 * N)); CK(hipMalloc(&d_y, 8 * N));
  CK(hipMemcpy(d_p, perm.data(), 4 * N, hipMemcpyHostToDevice)); CK(hipMemcpy(d_h, half.data(), 4 * N, hipMemcpyHostToDevice));
  CK(hipMemset(d_x, 0, 8 * N));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto bench = [&](const char* name, auto launch) {
    for (int r = 0; r < 5; ++r) launch(); CK(hipDeviceSynchronize());
    const int iters = 300; CK(hipEventRecord(e0)); for (int r = 0; r < iters; ++r) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-40s %8.2f us\n", name, 1000.0 * ms / iters); };
  int g = N / 256;
  bench("copy 8MB", [&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, N, d_x, d_y); });
  bench("gather 1M random", [&] { hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, 0, N, d_p, d_x, d_y); });
  bench("scatter 1M random", [&] { hipLaunchKernelGGL(k_scatter, dim3(g), dim3(256), 0, 0, N, d_p, d_x, d_y); });
  bench("gather 1M half-random", [&] { hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, 0, N, d_h, d_x, d_y); });
  bench("scatter 1M half-random", [&] { hipLaunchKernelGGL(k_scatter, dim3(g), dim3(256), 0, 0, N, d_h, d_x, d_y); });
  bench("gather 500k random", [&] { hipLaunchKernelGGL(k_gather, dim3(g / 2), dim3(256), 0, 0, N / 2, d_p, d_x, d_y); });
  bench("scatter 500k random", [&] { hipLaunchKernelGGL(k_scatter, dim3(g / 2), dim3(256), 0, 0, N / 2, d_p, d_x, d_y); });
  return 0;
}
