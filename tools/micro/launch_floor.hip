// Launch floor of a colour-launch-shaped kernel on MI355X (measurement helper, not product):
// what K back-to-back launches of ~800 workgroups of 256 threads cost per launch on one stream
// when each does (0) nothing, (1) one coalesced 24-B load + store per thread (a colour launch's
// own-row traffic), (2) that plus one dependent gather through an index array (the staging chain's
// list -> gather step), (3) that plus a workgroup barrier and an LDS round trip.  The ILU(0)
// colour launches fit  time = 4.6 us + traffic / 7.9 TB/s  (DESIGN.md §0.8); this says how much of
// the 4.6 us a launch of that shape pays before any of the sweep's own work.
// usage: ./launch_floor [wgs=800] [reps=200]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k_shape(int n, const int *__restrict__ idx,
                                               const double *__restrict__ a,
                                               double *__restrict__ b) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if constexpr (MODE == 0) return;
  __shared__ double s[256 * 3];
  if (t >= n) return;
  double v0 = a[3 * size_t(t)], v1 = a[3 * size_t(t) + 1], v2 = a[3 * size_t(t) + 2];
  if constexpr (MODE >= 2) {
    const int j = idx[t];
    v0 += a[3 * size_t(j)];
    v1 += a[3 * size_t(j) + 1];
    v2 += a[3 * size_t(j) + 2];
  }
  if constexpr (MODE >= 3) {
    s[3 * threadIdx.x] = v0;
    s[3 * threadIdx.x + 1] = v1;
    s[3 * threadIdx.x + 2] = v2;
    __syncthreads();
    const int o = (threadIdx.x * 37) & 255;
    v0 += s[3 * o];
    v1 += s[3 * o + 1];
    v2 += s[3 * o + 2];
  }
  b[3 * size_t(t)] = v0;
  b[3 * size_t(t) + 1] = v1;
  b[3 * size_t(t) + 2] = v2;
}

int main(int argc, char **argv) {
  const int wgs = argc > 1 ? std::atoi(argv[1]) : 800, reps = argc > 2 ? std::atoi(argv[2]) : 200;
  const int n = wgs * 256;
  std::vector<int> hidx(n);
  unsigned s = 12345;
  for (int i = 0; i < n; i++) {  // neighbour-like: within +-4096 rows
    s = s * 1664525u + 1013904223u;
    int j = i + int(s % 8192) - 4096;
    hidx[i] = j < 0 ? -j : (j >= n ? 2 * n - 2 - j : j);
  }
  int *idx;
  double *a, *b;
  CK(hipMalloc(&idx, sizeof(int) * n));
  CK(hipMalloc(&a, sizeof(double) * 3 * n));
  CK(hipMalloc(&b, sizeof(double) * 3 * n));
  CK(hipMemcpy(idx, hidx.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  CK(hipMemset(a, 0, sizeof(double) * 3 * n));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int mode) {
    auto go = [&] {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_shape<0>, dim3(wgs), dim3(256), 0, st, n, idx, a, b); break;
        case 1: hipLaunchKernelGGL(k_shape<1>, dim3(wgs), dim3(256), 0, st, n, idx, a, b); break;
        case 2: hipLaunchKernelGGL(k_shape<2>, dim3(wgs), dim3(256), 0, st, n, idx, a, b); break;
        default: hipLaunchKernelGGL(k_shape<3>, dim3(wgs), dim3(256), 0, st, n, idx, a, b); break;
      }
    };
    for (int i = 0; i < 20; i++) go();
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; i++) go();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / reps;
  };
  // the same launches captured once into a hipGraph and replayed (per launch inside the replay)
  auto run_graph = [&](int mode) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < reps; i++) {
      if (mode == 0)
        hipLaunchKernelGGL(k_shape<0>, dim3(wgs), dim3(256), 0, st, n, idx, a, b);
      else
        hipLaunchKernelGGL(k_shape<2>, dim3(wgs), dim3(256), 0, st, n, idx, a, b);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 1e3 * ms / reps;
  };
  const char *names[4] = {"empty", "own load+store", "+ dependent gather", "+ barrier + LDS"};
  std::printf("{\"workgroups\": %d, \"threads\": %d, \"reps\": %d", wgs, n, reps);
  for (int m = 0; m < 4; m++) std::printf(", \"%s_us\": %.3f", names[m], run(m));
  std::printf(", \"graph empty_us\": %.3f, \"graph + dependent gather_us\": %.3f", run_graph(0),
              run_graph(2));
  std::printf("}\n");
  CK(hipFree(idx));
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
