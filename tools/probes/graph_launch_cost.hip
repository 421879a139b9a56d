// Host cost of launching a chain of small kernels: stream launches vs one hipGraph launch
// (captured from the same stream), and the device time of the chain both ways.
// hipcc --offload-arch=gfx950 -O2 tools/probes/graph_launch_cost.hip -o /tmp/glc
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void tiny(int* p, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[i] += 1;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const int K = 12, R = 2000;
  int* d;
  CK(hipMalloc(&d, 64 * 4));
  CK(hipMemset(d, 0, 64 * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev[K];
  for (int i = 0; i < K; ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  auto chain = [&](bool events) {
    for (int i = 0; i < K; ++i) {
      hipLaunchKernelGGL(tiny, dim3(64), dim3(256), 0, s, d, i);
      if (events) (void)hipEventRecord(ev[i], s);
    }
  };
  for (int ev_on = 0; ev_on < 2; ++ev_on) {
    for (int i = 0; i < 200; ++i) chain(ev_on);
    CK(hipStreamSynchronize(s));
    double host = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < R; ++r) {
      auto h0 = std::chrono::steady_clock::now();
      chain(ev_on);
      host += std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();
    }
    CK(hipStreamSynchronize(s));
    double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("stream: %d kernels%s: host %.1f us per chain, wall %.1f us per chain\n", K,
           ev_on ? " + event records" : "", 1e6 * host / R, 1e6 * tot / R);
  }
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  chain(false);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 200; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  double host = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < R; ++r) {
    auto h0 = std::chrono::steady_clock::now();
    (void)hipGraphLaunch(ge, s);
    host += std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();
  }
  CK(hipStreamSynchronize(s));
  double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("graph: %d kernels: host %.1f us per launch, wall %.1f us per chain\n", K, 1e6 * host / R,
         1e6 * tot / R);
  int h[64];
  CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  printf("check %d\n", h[0]);
  return 0;
}
