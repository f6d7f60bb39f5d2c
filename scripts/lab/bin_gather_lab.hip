// Lab: the long-row bins' gathers at 500k arcs, in the canonical position order vs
// sorted by column inside each bin (the same gathers; 25.8 vs 7.1 distinct 128-B lines
// per wave-instruction, scripts/lab/bin_profile.py DUMP=...). One workgroup per bin, block
// b = 8 m + s (slice s on XCD s, as the SpMV places them); thread t gathers positions
// t + 256 u, u < 8. Back-to-back launches timed with HIP events, alternated.
//   hipcc -O3 --offload-arch=gfx950 bin_gather_lab.hip -o bin_gather_lab
//   ./bin_gather_lab lab_bin/bins.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_gather(const int* __restrict__ cols, int cap,
                                                const double* __restrict__ x,
                                                double* __restrict__ out) {
  const int* c = cols + (size_t)blockIdx.x * cap;
  int ci[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) ci[u] = c[threadIdx.x + 256 * u];
  double xv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) xv[u] = x[ci[u] < 0 ? 0 : ci[u]];
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += ci[u] < 0 ? 0.0 : xv[u];
  out[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  FILE* f = std::fopen(argc > 1 ? argv[1] : "lab_bin/bins.bin", "rb");
  if (!f) { std::printf("no data\n"); return 1; }
  int hdr[3];
  if (std::fread(hdr, 4, 3, f) != 3) return 1;
  const int nb = hdr[0], cap = hdr[1], n = hdr[2];
  if (cap != 2048) { std::printf("cap %d: this lab assumes 2048\n", cap); return 1; }
  std::vector<int> canon((size_t)nb * cap), srt((size_t)nb * cap);
  if (std::fread(canon.data(), 4, canon.size(), f) != canon.size()) return 1;
  if (std::fread(srt.data(), 4, srt.size(), f) != srt.size()) return 1;
  std::fclose(f);
  for (int v : canon) if (v >= n) { std::printf("bad column\n"); return 1; }
  int *dc, *ds;
  double *x, *out;
  CK(hipMalloc(&dc, canon.size() * 4)); CK(hipMalloc(&ds, srt.size() * 4));
  CK(hipMalloc(&x, (size_t)n * 8)); CK(hipMalloc(&out, (size_t)nb * 256 * 8));
  CK(hipMemcpy(dc, canon.data(), canon.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, srt.data(), srt.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(x, 0, (size_t)n * 8));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 2000;
  for (int rep = 0; rep < 4; ++rep)
    for (int v = 0; v < 2; ++v) {
      const int* cols = v == 0 ? dc : ds;
      k_gather<<<nb, 256, 0, st>>>(cols, cap, x, out);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) k_gather<<<nb, 256, 0, st>>>(cols, cap, x, out);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("%s %.3f us per launch (%d bins)\n", v == 0 ? "canonical" : "sorted   ",
                  1000.0 * ms / iters, nb);
    }
  return 0;
}
