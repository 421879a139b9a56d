// What the first stream query after finished work costs (the ~20 us of tools/run_timeline.py's
// sync_first), against the number of kernels launched since the last query, and with the same
// kernels as one graph launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/query_cost.hip -o tools/probes/query_cost
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void tiny(int* p, int v) {
  if (threadIdx.x == 0) p[blockIdx.x] = v;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}
static void spin_us(double t) {
  const auto t0 = clk::now();
  while (us(t0, clk::now()) < t) {
  }
}

int main() {
  int* buf;
  CK(hipMalloc(&buf, 4096));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int n : {1, 2, 6, 12}) {
    // graph of the same n launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < n; ++k) hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s, buf, k);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int mode = 0; mode < 2; ++mode) {
      std::vector<double> launch, query, again;
      for (int it = 0; it < 300; ++it) {
        const auto t0 = clk::now();
        if (mode == 0)
          for (int k = 0; k < n; ++k) hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s, buf, k);
        else
          CK(hipGraphLaunch(ge, s));
        const auto t1 = clk::now();
        spin_us(2000);   // the work is long finished
        const auto t2 = clk::now();
        const hipError_t q = hipStreamQuery(s);
        const auto t3 = clk::now();
        (void)hipStreamQuery(s);
        const auto t4 = clk::now();
        if (q != hipSuccess) printf("query %d\n", (int)q);
        if (it >= 20) {
          launch.push_back(us(t0, t1));
          query.push_back(us(t2, t3));
          again.push_back(us(t3, t4));
        }
      }
      for (auto* v : {&launch, &query, &again}) std::sort(v->begin(), v->end());
      printf("%2d kernels %s: enqueue %6.1f us, first query %6.1f us, next query %5.1f us (medians)\n",
             n, mode ? "as one graph" : "launched    ", launch[launch.size() / 2],
             query[query.size() / 2], again[again.size() / 2]);
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamDestroy(s));
  CK(hipFree(buf));
  return 0;
}
