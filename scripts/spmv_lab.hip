// spmv_lab.hip — standalone ablation bench for the SpMV core on a dumped CSR matrix.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o spmv_lab spmv_lab.hip
// Run:   ./spmv_lab /tmp/csr_500k.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

constexpr int TPB = 256;
struct Item { int row0, row1, nz0, kind; };

__device__ __forceinline__ double wave_sum(double v) {
  v = v + __shfl_xor(v, 32); v = v + __shfl_xor(v, 16); v = v + __shfl_xor(v, 8);
  v = v + __shfl_xor(v, 4); v = v + __shfl_xor(v, 2); v = v + __shfl_xor(v, 1);
  return v;
}

// ---- pure stream: read val, col, rowptr once, write n doubles (the byte roof)
__global__ __launch_bounds__(256) void k_stream(int n, int nnz, const int* __restrict__ rp, const int* __restrict__ col,
                                                const double* __restrict__ val, double* __restrict__ y) {
  double s = 0; int acc = 0;
  int tid = blockIdx.x * 256 + threadIdx.x, nt = gridDim.x * 256;
  for (int q = tid; q < nnz; q += nt) { s += val[q]; acc += col[q]; }
  for (int i = tid; i <= n; i += nt) acc += rp[i];
  for (int i = tid; i < n; i += nt) y[i] = s + acc;
}

// ---- current design (item walk), mode bits: 1 = skip stream items, 2 = skip wave items, 4 = no gather
template <int MODE>
__global__ __launch_bounds__(256) void k_items(int n_items, int G, const Item* __restrict__ items, const int* __restrict__ rp,
                                               const int* __restrict__ col, const double* __restrict__ val,
                                               const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double prod[2048];
  const int t = threadIdx.x;
  for (int it = blockIdx.x; it < n_items; it += G) {
    const Item item = items[it];
    if (item.kind == 0) {
      if (MODE & 1) continue;
      const int nz0 = item.nz0, cnt = rp[item.row1] - nz0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = t + u * 256;
        if (q < cnt) { const int c = col[nz0 + q]; prod[q] = val[nz0 + q] * x[(MODE & 4) ? (c & 63) : c]; }
      }
      __syncthreads();
      for (int i = item.row0 + t; i < item.row1; i += 256) {
        const int b = rp[i] - nz0, e = rp[i + 1] - nz0;
        double s = 0.0;
        for (int q = b; q < e; ++q) s = s + prod[q];
        y[i] = s;
      }
      __syncthreads();
    } else {
      if (MODE & 2) continue;
      const int w = t >> 6, lane = t & 63, i = item.row0 + w;
      double s = 0.0;
      if (i < item.row1) {
        const int e = rp[i + 1];
        int q = rp[i] + lane;
        for (; q + 192 < e; q += 256) {
          const int c0 = col[q], c1 = col[q + 64], c2 = col[q + 128], c3 = col[q + 192];
          const double a0 = val[q], a1 = val[q + 64], a2 = val[q + 128], a3 = val[q + 192];
          const double p0 = a0 * x[(MODE & 4) ? (c0 & 63) : c0], p1 = a1 * x[(MODE & 4) ? (c1 & 63) : c1];
          const double p2 = a2 * x[(MODE & 4) ? (c2 & 63) : c2], p3 = a3 * x[(MODE & 4) ? (c3 & 63) : c3];
          s = s + p0; s = s + p1; s = s + p2; s = s + p3;
        }
        for (; q < e; q += 64) s = s + val[q] * x[(MODE & 4) ? (col[q] & 63) : col[q]];
      }
      s = wave_sum(s);
      if (i < item.row1 && lane == 0) y[i] = s;
    }
  }
}

// ---- CSR-vector, one wave per row, all rows (baseline reference design)
__global__ __launch_bounds__(256) void k_vector(int n, const int* __restrict__ rp, const int* __restrict__ col,
                                                const double* __restrict__ val, const double* __restrict__ x, double* __restrict__ y) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n) return;
  double s = 0.0;
  for (int q = rp[row] + lane; q < rp[row + 1]; q += 64) s = s + val[q] * x[col[q]];
  s = wave_sum(s);
  if (lane == 0) y[row] = s;
}

// ---- scalar CSR: one thread per row (short rows only, long rows handled by a 2nd kernel)
__global__ __launch_bounds__(256) void k_scalar_short(int n, const int* __restrict__ rp, const int* __restrict__ col,
                                                      const double* __restrict__ val, const double* __restrict__ x, double* __restrict__ y, int maxlen) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int b = rp[i], e = rp[i + 1];
  if (e - b > maxlen) return;
  double s = 0.0;
  for (int q = b; q < e; ++q) s = s + val[q] * x[col[q]];
  y[i] = s;
}
// long rows listed explicitly: one block per row
__global__ __launch_bounds__(256) void k_block_rows(const int* __restrict__ rows, const int* __restrict__ rp, const int* __restrict__ col,
                                                    const double* __restrict__ val, const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double red[4];
  const int i = rows[blockIdx.x];
  double s = 0.0;
  for (int q = rp[i] + threadIdx.x; q < rp[i + 1]; q += 256) s = s + val[q] * x[col[q]];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) y[i] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- long rows split into S column slices; block b handles slice b % S of a 4-row group
// (blocks b, b+8, ... share an XCD under round-robin dispatch -> each XCD's L2 only
// sees 1/8 of x). Writes partials P[r*S + s].
template <int S>
__global__ __launch_bounds__(256) void k_node_slices(int ngroups, const int* __restrict__ rows, int nrows,
    const int* __restrict__ off, const int* __restrict__ col, const double* __restrict__ val,
    const double* __restrict__ x, double* __restrict__ P) {
  const int s = blockIdx.x % S, g = blockIdx.x / S;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ri = g * 4 + w;
  if (ri >= nrows) return;
  const int b = off[ri * (S + 1) + s], e = off[ri * (S + 1) + s + 1];
  double acc = 0.0;
  int q = b + lane;
  for (; q + 64 < e; q += 128) { const int c0 = col[q], c1 = col[q + 64]; const double a0 = val[q], a1 = val[q + 64];
    const double p0 = a0 * x[c0], p1 = a1 * x[c1]; acc = acc + p0; acc = acc + p1; }
  for (; q < e; q += 64) acc = acc + val[q] * x[col[q]];
  acc = wave_sum(acc);
  if (lane == 0) P[ri * S + s] = acc;
}
// combine: y[row] = sum_s P[r][s]
template <int S>
__global__ void k_node_combine(const int* __restrict__ rows, int nrows, const double* __restrict__ P, double* __restrict__ y) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < S; ++k) s = s + P[r * S + k];
  y[rows[r]] = s;
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  long long hdr[2];
  fread(hdr, 8, 2, f);
  int n = (int)hdr[0], nnz = (int)hdr[1];
  std::vector<int> rp(n + 1), col(nnz);
  std::vector<double> val(nnz), x(n);
  fread(rp.data(), 4, n + 1, f); fread(col.data(), 4, nnz, f); fread(val.data(), 8, nnz, f);
  fclose(f);
  for (int i = 0; i < n; ++i) x[i] = 1.0 / (1 + i % 97);
  // items like the product (stream 2048/1024, wave 4 rows)
  std::vector<Item> items;
  { int i = 0; while (i < n) { int L = rp[i + 1] - rp[i];
      if (L <= 32) { int r0 = i, nz0 = rp[i], rows = 0; while (i < n && rp[i+1]-rp[i] <= 32 && rp[i+1]-nz0 <= 2048 && rows < 1024) { ++i; ++rows; } items.push_back({r0, i, nz0, 0}); }
      else { int r0 = i; while (i < n && i - r0 < 4 && rp[i+1]-rp[i] > 32) ++i; items.push_back({r0, i, rp[r0], 1}); } } }
  std::vector<int> longrows; for (int i = 0; i < n; ++i) if (rp[i+1]-rp[i] > 32) longrows.push_back(i);
  int *d_rp, *d_col, *d_long; double *d_val, *d_x, *d_y; Item* d_items;
  CK(hipMalloc(&d_rp, 4 * (n + 1))); CK(hipMalloc(&d_col, 4 * nnz)); CK(hipMalloc(&d_val, 8 * (size_t)nnz));
  CK(hipMalloc(&d_x, 8 * n)); CK(hipMalloc(&d_y, 8 * n)); CK(hipMalloc(&d_items, sizeof(Item) * items.size()));
  CK(hipMalloc(&d_long, 4 * longrows.size() + 4));
  CK(hipMemcpy(d_rp, rp.data(), 4 * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_col, col.data(), 4 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_val, val.data(), 8 * (size_t)nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_x, x.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_items, items.data(), sizeof(Item) * items.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_long, longrows.data(), 4 * longrows.size(), hipMemcpyHostToDevice));
  int ni = items.size(), G = ni;
  double bytes = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
  printf("n=%d nnz=%d items=%d longrows=%zu algo_bytes=%.0f\n", n, nnz, ni, longrows.size(), bytes);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto bench = [&](const char* name, auto launch) {
    for (int r = 0; r < 5; ++r) launch();
    CK(hipDeviceSynchronize());
    const int iters = 200;
    CK(hipEventRecord(e0));
    for (int r = 0; r < iters; ++r) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double us = 1000.0 * ms / iters;
    printf("%-28s %8.2f us  %7.1f GB/s (algo)\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  bench("empty-ish stream 256blk", [&] { hipLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, 0, 0, 0, d_rp, d_col, d_val, d_y); });
  for (int g : {512, 1024, 2048, 4096})
    bench((std::string("stream roof g=") + std::to_string(g)).c_str(), [&] { hipLaunchKernelGGL(k_stream, dim3(g), dim3(256), 0, 0, n, nnz, d_rp, d_col, d_val, d_y); });
  bench("items full", [&] { hipLaunchKernelGGL(k_items<0>, dim3(G), dim3(256), 0, 0, ni, G, d_items, d_rp, d_col, d_val, d_x, d_y); });
  bench("items stream-only", [&] { hipLaunchKernelGGL(k_items<2>, dim3(G), dim3(256), 0, 0, ni, G, d_items, d_rp, d_col, d_val, d_x, d_y); });
  bench("items wave-only", [&] { hipLaunchKernelGGL(k_items<1>, dim3(G), dim3(256), 0, 0, ni, G, d_items, d_rp, d_col, d_val, d_x, d_y); });
  bench("items nogather", [&] { hipLaunchKernelGGL(k_items<4>, dim3(G), dim3(256), 0, 0, ni, G, d_items, d_rp, d_col, d_val, d_x, d_y); });
  bench("items wave-only nogather", [&] { hipLaunchKernelGGL(k_items<5>, dim3(G), dim3(256), 0, 0, ni, G, d_items, d_rp, d_col, d_val, d_x, d_y); });
  bench("vector (wave/row, all)", [&] { hipLaunchKernelGGL(k_vector, dim3((n + 3) / 4), dim3(256), 0, 0, n, d_rp, d_col, d_val, d_x, d_y); });
  bench("scalar short only", [&] { hipLaunchKernelGGL(k_scalar_short, dim3((n + 255) / 256), dim3(256), 0, 0, n, d_rp, d_col, d_val, d_x, d_y, 32); });
  // slice tables
  int m = 0; for (int i = 0; i < n; ++i) if (rp[i+1]-rp[i] > 32) { m = i; break; }   // first long row index ~ num arcs
  auto mk = [&](int S) { std::vector<int> off(longrows.size() * (S + 1));
    for (size_t r = 0; r < longrows.size(); ++r) { int i = longrows[r];
      for (int s2 = 0; s2 <= S; ++s2) { long long bound = (long long)m * s2 / S; int q = rp[i];
        while (q < rp[i+1] && col[q] < bound) ++q; if (s2 == S) q = rp[i+1]; off[r*(S+1)+s2] = q; } }
    int* d; CK(hipMalloc(&d, 4 * off.size())); CK(hipMemcpy(d, off.data(), 4 * off.size(), hipMemcpyHostToDevice)); return d; };
  int* off8 = mk(8); int* off16 = mk(16); int* off4 = mk(4); int* off1 = mk(1);
  double* d_P; CK(hipMalloc(&d_P, 8 * longrows.size() * 16));
  int nl = longrows.size(), ng = (nl + 3) / 4;
  bench("node slices S=1", [&] { hipLaunchKernelGGL(k_node_slices<1>, dim3(ng * 1), dim3(256), 0, 0, ng, d_long, nl, off1, d_col, d_val, d_x, d_P); });
  bench("node slices S=4", [&] { hipLaunchKernelGGL(k_node_slices<4>, dim3(ng * 4), dim3(256), 0, 0, ng, d_long, nl, off4, d_col, d_val, d_x, d_P); });
  bench("node slices S=8", [&] { hipLaunchKernelGGL(k_node_slices<8>, dim3(ng * 8), dim3(256), 0, 0, ng, d_long, nl, off8, d_col, d_val, d_x, d_P); });
  bench("node slices S=16", [&] { hipLaunchKernelGGL(k_node_slices<16>, dim3(ng * 16), dim3(256), 0, 0, ng, d_long, nl, off16, d_col, d_val, d_x, d_P); });
  bench("node combine S=8", [&] { hipLaunchKernelGGL(k_node_combine<8>, dim3((nl + 255) / 256), dim3(256), 0, 0, d_long, nl, d_P, d_y); });
  bench("block long rows only", [&] { hipLaunchKernelGGL(k_block_rows, dim3(longrows.size()), dim3(256), 0, 0, d_long, d_rp, d_col, d_val, d_x, d_y); });
  return 0;
}
