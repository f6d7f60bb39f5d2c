// Is the block -> XCD dealing offset stable across launches? (dev lab) Launches a
// sequence of kernels with grids that are / are not multiples of 8 and prints, per
// launch, the XCC id of block 0 and whether every block b sits on (b + off) % 8.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k_rec(int* xcc) {
  if (threadIdx.x == 0) {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    xcc[blockIdx.x] = v;
  }
}
int main() {
  const int grids[] = {1024, 1024, 1555, 1024, 490, 1555, 490, 1560, 496, 1560, 496, 1560, 496, 1560, 496};
  int* d; hipMalloc(&d, 4096 * 4);
  for (int rep = 0; rep < 2; ++rep) {
    for (int g : grids) {
      hipLaunchKernelGGL(k_rec, dim3(g), dim3(256), 0, 0, d);
      std::vector<int> h(g);
      hipMemcpy(h.data(), d, g * 4, hipMemcpyDeviceToHost);
      const int off = h[0] & 7;
      int bad = 0;
      for (int b = 0; b < g; ++b) bad += ((h[b] & 7) != ((b + off) & 7));
      printf("grid %5d  block0 on XCD %d  blocks off the round-robin: %d\n", g, off, bad);
    }
  }
  // back-to-back without host sync in between (as in a graph), recorded into slices
  int* d2; hipMalloc(&d2, 16 * 4096 * 4);
  const int seq[] = {1560, 496, 1560, 496, 1560, 496, 1560, 496};
  for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_rec, dim3(seq[i]), dim3(256), 0, 0, d2 + i * 4096);
  hipDeviceSynchronize();
  std::vector<int> h(8 * 4096);
  hipMemcpy(h.data(), d2, 8 * 4096 * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < 8; ++i) {
    const int* x = h.data() + i * 4096;
    const int off = x[0] & 7;
    int bad = 0;
    for (int b = 0; b < seq[i]; ++b) bad += ((x[b] & 7) != ((b + off) & 7));
    printf("stream seq %d grid %d block0 XCD %d off-rr %d\n", i, seq[i], off, bad);
  }
  return 0;
}
