// Measured HBM ceilings for the bench line (tools/micro, not part of the product): hand-written
// dwordx4 streaming kernels over buffers 6-8x the 256 MiB Infinity Cache, so every byte comes from
// or goes to HBM.  bench.py loads libstream.so and puts the four rates in `measured_stream_gbs`;
// every `frac_of_measured_*` of the line divides by one of them.
//   read   16 B per lane loads of a 2 GiB buffer, summed (a conditional sink store keeps them)
//   write  16 B per lane stores into a 2 GiB buffer
//   copy   16 B per lane load + store, 1 GiB -> 1 GiB (2 GiB moved)
//   mix    the assembly's read:write proportion (PMC at config 3: 79.7 MB read, 224.2 MB written
//          per launch = 26:74): each lane writes one 16-B element of a 1.5 GiB buffer and every
//          lane whose element index is 0..4 mod 14 also reads one 16-B element of a second buffer
//          (5:14 = 26.3:73.7), the reads contiguous in their buffer
// Each pattern runs in several shapes -- U = 1, 2, 4, 8 elements per lane with one workgroup per
// 256 x U elements, and a resident grid-stride form (8 workgroups per CU, U = 4 per pass) -- and the
// ceiling is the fastest shape: bytes moved / average launch time over `reps` launches, each timed
// with one HIP event pair after two untimed launches.
// C ABI: stream_measure(device, reps, out[4], shapes[20]) -> 0 or a HIP error code; out = {read,
// write, copy, mix} in GB/s (best shape), shapes[4 * s + k] = pattern k's rate in shape s (may be
// NULL).
#include <hip/hip_runtime.h>

#include <cstddef>

namespace {

constexpr int kB = 256;  // threads per workgroup
constexpr int kShapes = 5;

// this lane's first element and the stride between passes: blocks of 256 x U elements (one pass,
// GS = false), or a grid-stride loop over such blocks (GS = true)
template <int U, bool GS>
struct Walk {
  size_t n;
  __device__ size_t start() const { return size_t(blockIdx.x) * kB * U + threadIdx.x; }
  __device__ size_t step() const { return GS ? size_t(gridDim.x) * kB * U : n; }
};

template <int U, bool GS>
__global__ __launch_bounds__(kB) void k_read(const float4 *__restrict__ a, size_t n, float *sink) {
  const Walk<U, GS> w{n};
  float s = 0.f;
  for (size_t base = w.start(); base < n; base += w.step()) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + size_t(u) * kB;
      v[u] = i < n ? a[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; u++) s += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (s == 1234.5f) sink[threadIdx.x] = s;  // never true for the zero-filled buffer
}

template <int U, bool GS>
__global__ __launch_bounds__(kB) void k_write(float4 *__restrict__ a, size_t n, float c) {
  const Walk<U, GS> w{n};
  for (size_t base = w.start(); base < n; base += w.step()) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + size_t(u) * kB;
      if (i < n) a[i] = make_float4(c, c, c, c);
    }
  }
}

template <int U, bool GS>
__global__ __launch_bounds__(kB) void k_copy(const float4 *__restrict__ a, float4 *__restrict__ b,
                                             size_t n) {
  const Walk<U, GS> w{n};
  for (size_t base = w.start(); base < n; base += w.step()) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + size_t(u) * kB;
      if (i < n) v[u] = a[i];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + size_t(u) * kB;
      if (i < n) b[i] = v[u];
    }
  }
}

// writes n elements of wr; element i with i % 14 < 5 also reads r[(i / 14) * 5 + i % 14]
template <int U, bool GS>
__global__ __launch_bounds__(kB) void k_mix(const float4 *__restrict__ r, float4 *__restrict__ wr,
                                            size_t n) {
  const Walk<U, GS> w{n};
  for (size_t base = w.start(); base < n; base += w.step()) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + size_t(u) * kB;
      const unsigned m = unsigned(i % 14);
      v[u] = make_float4(1.f, 2.f, 3.f, 4.f);
      if (i < n && m < 5) v[u] = r[(i / 14) * 5 + m];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + size_t(u) * kB;
      if (i < n) wr[i] = v[u];
    }
  }
}

template <int U>
unsigned blocks(size_t n) {
  return unsigned((n + size_t(kB) * U - 1) / (size_t(kB) * U));
}

template <int U, bool GS>
hipError_t launch(int k, float4 *a, float4 *b, float *sink, size_t n2, size_t n1, size_t nmw,
                  unsigned resident, hipStream_t s) {
  auto g = [&](size_t n) { return GS ? resident : blocks<U>(n); };
  switch (k) {
    case 0: k_read<U, GS><<<g(n2), kB, 0, s>>>(a, n2, sink); break;
    case 1: k_write<U, GS><<<g(n2), kB, 0, s>>>(b, n2, 1.0f); break;
    case 2: k_copy<U, GS><<<g(n1), kB, 0, s>>>(a, b, n1); break;
    default: k_mix<U, GS><<<g(nmw), kB, 0, s>>>(a, b, nmw); break;
  }
  return hipGetLastError();
}

}  // namespace

extern "C" int stream_measure(int device, int reps, double *out, double *shapes) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return int(e);
  int cus = 0;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return int(e);
  const unsigned resident = unsigned(8 * (cus > 0 ? cus : 256));
  const size_t GiB = size_t(1) << 30;
  const size_t n2 = 2 * GiB / 16, n1 = GiB / 16;
  const size_t nmw = (3 * GiB / 2) / 16;
  const size_t nmr = nmw / 14 * 5 + (nmw % 14 < 5 ? nmw % 14 : 5);  // elements the mix reads
  const double bytes[4] = {double(n2) * 16, double(n2) * 16, 2.0 * double(n1) * 16,
                           double(nmw + nmr) * 16};
  float4 *a = nullptr, *b = nullptr;
  float *sink = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if ((e = hipMalloc(&a, n2 * 16)) != hipSuccess) return int(e);
  if ((e = hipMalloc(&b, n2 * 16)) != hipSuccess) {
    (void)hipFree(a);
    return int(e);
  }
  e = hipMalloc(&sink, kB * sizeof(float));
  if (e == hipSuccess) e = hipStreamCreate(&s);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipMemsetAsync(a, 0, n2 * 16, s);
  if (e == hipSuccess) e = hipMemsetAsync(b, 0, n2 * 16, s);
  for (int k = 0; k < 4; k++) out[k] = 0;
  for (int sh = 0; sh < kShapes && e == hipSuccess; sh++) {
    for (int k = 0; k < 4 && e == hipSuccess; k++) {
      auto go = [&]() {
        switch (sh) {
          case 0: return launch<1, false>(k, a, b, sink, n2, n1, nmw, resident, s);
          case 1: return launch<2, false>(k, a, b, sink, n2, n1, nmw, resident, s);
          case 2: return launch<4, false>(k, a, b, sink, n2, n1, nmw, resident, s);
          case 3: return launch<8, false>(k, a, b, sink, n2, n1, nmw, resident, s);
          default: return launch<4, true>(k, a, b, sink, n2, n1, nmw, resident, s);
        }
      };
      for (int w = 0; w < 2 && e == hipSuccess; w++) e = go();
      double ms_tot = 0;
      for (int r = 0; r < reps && e == hipSuccess; r++) {
        e = hipEventRecord(e0, s);
        if (e == hipSuccess) e = go();
        if (e == hipSuccess) e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        ms_tot += ms;
      }
      if (e != hipSuccess) break;
      const double gbs = bytes[k] * reps / (ms_tot * 1e-3) / 1e9;
      if (shapes) shapes[4 * sh + k] = gbs;
      if (gbs > out[k]) out[k] = gbs;
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (s) (void)hipStreamDestroy(s);
  (void)hipFree(sink);
  (void)hipFree(a);
  (void)hipFree(b);
  return e == hipSuccess ? 0 : int(e);
}
