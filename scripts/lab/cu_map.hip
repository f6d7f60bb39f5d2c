// Which CU does workgroup b of a fully resident grid land on? (dev lab) Every workgroup
// holds the SpMV kernels' LDS footprint and stays resident ~30 us, so the placement is
// the dispatcher's initial one. Prints, for the blocks of XCD 0 (b % 8 == 0) in order,
// the (SE, SH, CU) of each, and how many workgroups each CU of that XCD received.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void k_where(unsigned* out, int spin_ticks) {
  extern __shared__ double lds[];
  long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    lds[0] = (double)hw;
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(2);
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 1560;
  const size_t lds = argc > 2 ? (size_t)atoi(argv[2]) : 19968;
  unsigned* d;
  hipMalloc(&d, grid * 2 * sizeof(unsigned));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_where, dim3(grid), dim3(256), lds, 0, d, 3000);
    hipDeviceSynchronize();
  }
  std::vector<unsigned> h(grid * 2);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  printf("grid %d lds %zu\n", grid, lds);
  for (int x = 0; x < 2; ++x) {
    std::map<int, int> per_cu;
    printf("XCD-group %d, block b = 8 i + %d: i -> se.sh.cu (xcc)\n", x, x);
    for (int b = x, i = 0; b < grid; b += 8, ++i) {
      const unsigned hw = h[2 * b], xcc = h[2 * b + 1];
      const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const int key = se * 32 + sh * 16 + cu;
      per_cu[key]++;
      printf("%d:%d.%d.%d(%u) ", i, se, sh, cu, xcc & 15);
      if (i % 16 == 15) printf("\n");
    }
    printf("\nper CU:");
    for (auto& kv : per_cu) printf(" %d.%d.%d=%d", kv.first / 32, (kv.first / 16) & 1, kv.first & 15, kv.second);
    printf("\n");
  }
  return 0;
}
