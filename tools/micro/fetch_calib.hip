// FETCH_SIZE / WRITE_SIZE calibration for the access widths of the hot-path kernels (tools/micro,
// not part of the product).  MI355X_MICROARCH.md (HBM section) establishes FETCH_SIZE = half the
// bytes only for 16-B-per-lane streaming reads and calls every other width uncalibrated; the
// sweeps and the SpMV gather 8-B values and 24-B / 28-B records.  Each kernel below reads a KNOWN
// number of distinct 128-B lines of a 2 GiB buffer (8x the Infinity Cache, every line touched
// once per launch so nothing is served on-die), so rocprofv3's per-dispatch FETCH_SIZE divided by
// the known bytes is the factor to apply to that access pattern:
//   s16  streaming, 16 B per lane (dwordx4)                    -- the guide's calibrated case
//   s8   streaming, 8 B per lane (dwordx2)
//   s4   streaming, 4 B per lane (dword): column indices
//   g8   8-B gathers, one per 128-B line, lines in a random order (one line per lane): the bytes
//        the fabric moves per partial-line miss (64 or 128), not a known-byte case
//   g8h  8-B gathers, two per line from different waves (halves 64 B apart): partial lines too
//   g8f  8-B gathers covering whole lines: the 16 elements of a line read by 16 lanes of one wave
//        in a permuted lane order, lines in a random order -- known bytes = the lines' bytes
//   g24f 24-B records (3 doubles) covering whole lines: groups of 16 records (384 B = 3 lines)
//        taken by 16 lanes in a permuted order, groups in a random order -- known bytes exact
//   g28f 28-B records (7 floats, the packed f32 ILU factor block): groups of 32 records (896 B =
//        7 lines) taken by 32 lanes in a permuted order, groups in a random order
//   g24 / g28: records in a fully random order (each line is needed by ~5 records far apart in
//        time, so it is fetched up to ~5 times): an upper-bound case, reported, not a factor
//   w16  streaming 16-B stores; w8 streaming 8-B stores (plane stores of the SELL k-form values)
// The program prints the known bytes per kernel; tools/fetch_calib_summary.py joins them with the
// counter CSVs.  usage: fetch_calib [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

constexpr size_t kBytes = size_t(2) << 30;  // 2 GiB
constexpr int kB = 256;

__global__ void s16(const double2 *a, size_t n, double *sink) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < n; i += size_t(gridDim.x) * kB) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) sink[0] = s;
}
__global__ void s8(const double *a, size_t n, double *sink) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < n; i += size_t(gridDim.x) * kB)
    s += a[i];
  if (s == 12345.678) sink[0] = s;
}
__global__ void s4(const int *a, size_t n, double *sink) {
  long long s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < n; i += size_t(gridDim.x) * kB)
    s += a[i];
  if (s == 123456789) sink[0] = double(s);
}
// idx: element offsets (in doubles) to gather, one per thread-iteration
__device__ void b_g8(const double *a, const long long *idx, size_t m, double *sink) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < m; i += size_t(gridDim.x) * kB)
    s += a[idx[i]];
  if (s == 12345.678) sink[0] = s;
}
// idx: record indices; a record of 24 B = 3 doubles at 24 r (8-B aligned: dwordx2 x 3 as the
// compiler splits it) / of 28 B = 7 floats at 28 r
__device__ void b_g24(const double *a, const int *idx, size_t m, double *sink) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < m; i += size_t(gridDim.x) * kB) {
    const double *r = a + size_t(idx[i]) * 3;
    s += r[0] + r[1] + r[2];
  }
  if (s == 12345.678) sink[0] = s;
}
__device__ void b_g28(const float *a, const int *idx, size_t m, double *sink) {
  float s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < m; i += size_t(gridDim.x) * kB) {
    const float *r = a + size_t(idx[i]) * 7;
    for (int q = 0; q < 7; q++) s += r[q];
  }
  if (s == 12345.678f) sink[0] = s;
}
__global__ void g8f(const double *a, const int *idx, size_t m, double *sink) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < m; i += size_t(gridDim.x) * kB)
    s += a[idx[i]];
  if (s == 12345.678) sink[0] = s;
}
// same bodies under their own names, so the profiler's per-kernel rows separate the patterns
__global__ void g8(const double *a, const long long *idx, size_t m, double *sink) { b_g8(a, idx, m, sink); }
__global__ void g8h(const double *a, const long long *idx, size_t m, double *sink) { b_g8(a, idx, m, sink); }
__global__ void g24(const double *a, const int *idx, size_t m, double *sink) { b_g24(a, idx, m, sink); }
__global__ void g24f(const double *a, const int *idx, size_t m, double *sink) { b_g24(a, idx, m, sink); }
__global__ void g28(const float *a, const int *idx, size_t m, double *sink) { b_g28(a, idx, m, sink); }
__global__ void g28f(const float *a, const int *idx, size_t m, double *sink) { b_g28(a, idx, m, sink); }
__global__ void w16(double2 *a, size_t n) {
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < n; i += size_t(gridDim.x) * kB)
    a[i] = make_double2(double(i), 1.0);
}
__global__ void w8(double *a, size_t n) {
  for (size_t i = blockIdx.x * size_t(kB) + threadIdx.x; i < n; i += size_t(gridDim.x) * kB)
    a[i] = double(i);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  void *buf;
  double *sink;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, kBytes));
  const size_t lines = kBytes / 128;
  std::mt19937_64 rng(20261017);
  // g8: one 8-B element per line, lines in random order (half the lines, to bound the index array)
  const size_t m8 = lines / 2;
  std::vector<long long> i8(m8);
  {
    std::vector<long long> L(lines);
    std::iota(L.begin(), L.end(), 0);
    std::shuffle(L.begin(), L.end(), rng);
    for (size_t i = 0; i < m8; i++) i8[i] = L[i] * 16 + (L[i] % 16);
  }
  // g8h: the same m8 / 2 lines, each hit at offsets 0 and 64 B by elements far apart in the order
  std::vector<long long> i8h(m8);
  for (size_t i = 0; i < m8 / 2; i++) {
    i8h[i] = (i8[i] / 16) * 16;
    i8h[i + m8 / 2] = (i8[i] / 16) * 16 + 8;
  }
  // g24 / g28: every record of the first 1 GiB once, random order
  const size_t r24 = (kBytes / 2) / 24, r28 = (kBytes / 2) / 28;
  std::vector<int> i24(r24), i28(r28);
  std::iota(i24.begin(), i24.end(), 0);
  std::iota(i28.begin(), i28.end(), 0);
  std::shuffle(i24.begin(), i24.end(), rng);
  std::shuffle(i28.begin(), i28.end(), rng);
  // whole-line groups: a group of g consecutive items (elements / records) spans whole lines; the
  // groups are visited in a random order, the items of a group by g consecutive lanes in a
  // permuted order (g divides 64, so a group never straddles two waves)
  auto grouped = [&](size_t items, int g) {
    std::vector<int> out(items - items % g);
    std::vector<int> G(out.size() / g);
    std::iota(G.begin(), G.end(), 0);
    std::shuffle(G.begin(), G.end(), rng);
    std::vector<int> P(g);
    for (size_t q = 0; q < G.size(); q++) {
      std::iota(P.begin(), P.end(), 0);
      std::shuffle(P.begin(), P.end(), rng);
      for (int k = 0; k < g; k++) out[q * g + k] = G[q] * g + P[k];
    }
    return out;
  };
  const std::vector<int> i8f = grouped((kBytes / 4) / 8, 16);   // 512 MiB of doubles
  const std::vector<int> i24f = grouped((kBytes / 2) / 24, 16);  // 1 GiB of 24-B records
  const std::vector<int> i28f = grouped((kBytes / 2) / 28, 32);  // 1 GiB of 28-B records
  long long *d8, *d8h;
  int *d24, *d28, *d8f, *d24f, *d28f;
  CK(hipMalloc(&d8, m8 * 8));
  CK(hipMalloc(&d8h, m8 * 8));
  CK(hipMalloc(&d24, r24 * 4));
  CK(hipMalloc(&d28, r28 * 4));
  CK(hipMalloc(&d8f, i8f.size() * 4));
  CK(hipMalloc(&d24f, i24f.size() * 4));
  CK(hipMalloc(&d28f, i28f.size() * 4));
  CK(hipMemcpy(d8, i8.data(), m8 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d8h, i8h.data(), m8 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d24, i24.data(), r24 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d28, i28.data(), r28 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d8f, i8f.data(), i8f.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d24f, i24f.data(), i24f.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d28f, i28f.data(), i28f.size() * 4, hipMemcpyHostToDevice));
  const dim3 G(8192), Bk(kB);
  // known bytes: data lines moved (128 B per distinct line touched) + index array bytes streamed
  std::printf("{\"kernel\": \"s16\", \"known_bytes\": %zu}\n", kBytes);
  std::printf("{\"kernel\": \"s8\", \"known_bytes\": %zu}\n", kBytes);
  std::printf("{\"kernel\": \"s4\", \"known_bytes\": %zu}\n", kBytes);
  std::printf("{\"kernel\": \"g8\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              m8 * 128 + m8 * 8, m8 * 128, m8 * 8);
  std::printf("{\"kernel\": \"g8h\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              (m8 / 2) * 128 + m8 * 8, (m8 / 2) * 128, m8 * 8);
  std::printf("{\"kernel\": \"g24\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              r24 * 24 + r24 * 4, r24 * 24, r24 * 4);
  std::printf("{\"kernel\": \"g28\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              r28 * 28 + r28 * 4, r28 * 28, r28 * 4);
  std::printf("{\"kernel\": \"g8f\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              i8f.size() * 12, i8f.size() * 8, i8f.size() * 4);
  std::printf("{\"kernel\": \"g24f\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              i24f.size() * 28, i24f.size() * 24, i24f.size() * 4);
  std::printf("{\"kernel\": \"g28f\", \"known_bytes\": %zu, \"data_lines_bytes\": %zu, \"index_bytes\": %zu}\n",
              i28f.size() * 32, i28f.size() * 28, i28f.size() * 4);
  std::printf("{\"kernel\": \"w16\", \"known_write_bytes\": %zu}\n", kBytes);
  std::printf("{\"kernel\": \"w8\", \"known_write_bytes\": %zu}\n", kBytes);
  std::fflush(stdout);
  for (int r = 0; r < reps; r++) {
    hipLaunchKernelGGL(s16, G, Bk, 0, 0, (const double2 *)buf, kBytes / 16, sink);
    hipLaunchKernelGGL(s8, G, Bk, 0, 0, (const double *)buf, kBytes / 8, sink);
    hipLaunchKernelGGL(s4, G, Bk, 0, 0, (const int *)buf, kBytes / 4, sink);
    hipLaunchKernelGGL(g8, G, Bk, 0, 0, (const double *)buf, d8, m8, sink);
    hipLaunchKernelGGL(g8h, G, Bk, 0, 0, (const double *)buf, d8h, m8, sink);
    hipLaunchKernelGGL(g24, G, Bk, 0, 0, (const double *)buf, d24, r24, sink);
    hipLaunchKernelGGL(g28, G, Bk, 0, 0, (const float *)buf, d28, r28, sink);
    hipLaunchKernelGGL(g8f, G, Bk, 0, 0, (const double *)buf, d8f, i8f.size(), sink);
    hipLaunchKernelGGL(g24f, G, Bk, 0, 0, (const double *)buf, d24f, i24f.size(), sink);
    hipLaunchKernelGGL(g28f, G, Bk, 0, 0, (const float *)buf, d28f, i28f.size(), sink);
    hipLaunchKernelGGL(w16, G, Bk, 0, 0, (double2 *)buf, kBytes / 16);
    hipLaunchKernelGGL(w8, G, Bk, 0, 0, (double *)buf, kBytes / 8);
    CK(hipDeviceSynchronize());
  }
  CK(hipGetLastError());
  std::printf("done\n");
  return 0;
}
