// Store-pattern microbenchmark for the SELL value layout (tools/micro, not part of the product).
// A: each 64-row chunk written by one wave, slot by slot, NV=7 values per (row, slot) in the
//    pair-interleaved layout (4 store instructions per slot), like k_assemble.
// B: the same bytes as a linear streaming write (dwordx4 per lane).
// C: like A but the wave writes its whole chunk region linearly (dwordx4, contiguous).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kRows = 64, NV = 7;

template <int MINW>
__global__ __launch_bounds__(256, MINW) void k_sell(double *vals, const int *chunk_off,
                                                    const int *chunk_len, int nrows, double v) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= nrows) return;
  const int chunk = row / kRows, lane = row % kRows;
  double *vc = vals + size_t(chunk_off[chunk]) * NV;
  const int len = chunk_len[chunk];
  for (int s = 0; s < len; s++) {
    double *sb = vc + size_t(s) * NV * kRows;
#pragma unroll
    for (int q = 0; q + 1 < NV; q += 2)
      reinterpret_cast<double2 *>(sb + (q >> 1) * 2 * kRows)[lane] = make_double2(v + s, v + q);
    sb[(NV - 1) * kRows + lane] = v;
  }
}

__global__ void k_linear(double2 *out, size_t n2, double v) {
  for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n2; i += size_t(gridDim.x) * 256)
    out[i] = make_double2(v, v + 1);
}

int main() {
  const int nrows = 738033, nchunks = (nrows + 63) / 64;
  std::vector<int> off(nchunks + 1), len(nchunks);
  off[0] = 0;
  for (int c = 0; c < nchunks; c++) {
    len[c] = 7;
    off[c + 1] = off[c] + 64 * len[c];
  }
  size_t nvals = size_t(off[nchunks]) * NV;
  double *vals;
  int *doff, *dlen;
  hipMalloc(&vals, nvals * 8);
  hipMalloc(&doff, off.size() * 4);
  hipMalloc(&dlen, len.size() * 4);
  hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dlen, len.data(), len.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char *name, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    hipEventRecord(e0);
    for (int i = 0; i < 20; i++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double us = ms * 1e3 / 20;
    std::printf("%-28s %8.2f us  %6.2f TB/s (%.1f MB)\n", name, us, nvals * 8 / us / 1e6,
                nvals * 8 / 1e6);
  };
  dim3 g((nrows + 255) / 256);
  timeit("sell chunk-per-wave MINW=3", [&] { hipLaunchKernelGGL(k_sell<3>, g, dim3(256), 0, 0, vals, doff, dlen, nrows, 1.0); });
  timeit("sell chunk-per-wave MINW=8", [&] { hipLaunchKernelGGL(k_sell<8>, g, dim3(256), 0, 0, vals, doff, dlen, nrows, 1.0); });
  timeit("linear dwordx4 2048 WG", [&] { hipLaunchKernelGGL(k_linear, dim3(2048), dim3(256), 0, 0, (double2 *)vals, nvals / 2, 1.0); });
  timeit("linear dwordx4 8192 WG", [&] { hipLaunchKernelGGL(k_linear, dim3(8192), dim3(256), 0, 0, (double2 *)vals, nvals / 2, 1.0); });
  return 0;
}
