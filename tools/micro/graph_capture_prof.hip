// Minimal stream capture of many kernel launches, for the rocprofv3 --kernel-trace crash of round 3
// (profiles/r03/amg_graph/rocprof_segv_r4b.log: SIGSEGV inside the runtime on the first capture of
// an AMG BiCGSTAB block of ~1,000 nodes).  Captures N launches of a trivial kernel (distinct
// arguments, a memset node every 16 launches as the BiCGSTAB blocks have), instantiates, replays
// three times, checks the result.  Run plain and under rocprofv3 --kernel-trace; if only the
// profiled run fails, the fault is the profiler's handling of large captures, not the library's.
// usage: graph_capture_prof N[:R] ...   (R replays, default 3; tools/micro, not part of the product)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void k_add(double *a, int n, double v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] += v;
}

int main(int argc, char **argv) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = 1 << 16;
  double *a, *b;
  CK(hipMalloc(&a, n * sizeof(double)));
  CK(hipMalloc(&b, n * sizeof(double)));
  for (int ai = 1; ai < argc; ai++) {
    const int N = std::atoi(argv[ai]);
    const char *colon = std::strchr(argv[ai], ':');
    const int R = colon ? std::atoi(colon + 1) : 3;
    CK(hipMemsetAsync(a, 0, n * sizeof(double), s));
    hipGraph_t g;
    hipGraphExec_t x;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < N; k++) {
      if (k % 16 == 15) hipMemsetAsync(b, 0, 64, s);
      hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, s, a, n, 1.0);
    }
    CK(hipStreamEndCapture(s, &g));
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    for (int r = 0; r < R; r++) CK(hipGraphLaunch(x, s));
    CK(hipStreamSynchronize(s));
    double h = 0;
    CK(hipMemcpy(&h, a + n - 1, sizeof(double), hipMemcpyDeviceToHost));
    std::printf("{\"launches\": %d, \"replays\": %d, \"nodes\": %zu, \"result\": %.1f, \"expect\": %.1f, \"ok\": %s}\n",
                N, R, nodes, h, double(R) * N, h == double(R) * N ? "true" : "false");
    std::fflush(stdout);
    CK(hipGraphExecDestroy(x));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
