// Probe: do same-address lanes of ONE ds_add_f32 apply in lane order?  Each trial adds a
// sequence whose float sum depends on the order (big/small/cancelling values), to 1, 2 or
// 8 addresses, and compares with the lane-order sequential sum computed on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

__global__ void probe(const float* vals, const int* addr, float* out, int nbins, int trials) {
  __shared__ float h[64];
  const int l = threadIdx.x;
  for (int t = 0; t < trials; ++t) {
    if (l < nbins) h[l] = 0.f;
    __syncthreads();
    atomicAdd(&h[addr[t * 64 + l]], vals[t * 64 + l]);
    __syncthreads();
    if (l < nbins) out[t * 64 + l] = h[l];
    __syncthreads();
  }
}

int main() {
  const int trials = 2000;
  std::vector<float> v(trials * 64);
  std::vector<int> a(trials * 64);
  srand(7);
  for (int t = 0; t < trials; ++t) {
    const int nb = t % 3 == 0 ? 1 : t % 3 == 1 ? 2 : 8;
    for (int l = 0; l < 64; ++l) {
      const int k = rand() % 4;
      v[t * 64 + l] = k == 0 ? 1.0e8f * (rand() % 2 ? 1 : -1) : k == 1 ? 1.0f + (rand() % 1000) * 1e-3f
                    : k == 2 ? 3.1e-5f * (rand() % 100) : 7.7e7f;
      a[t * 64 + l] = rand() % nb;
    }
  }
  float *dv, *dout; int* da;
  hipMalloc(&dv, v.size() * 4); hipMalloc(&da, a.size() * 4); hipMalloc(&dout, v.size() * 4);
  hipMemcpy(dv, v.data(), v.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dv, da, dout, 64, trials);
  std::vector<float> o(v.size());
  hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
  int lane_order = 0, differ = 0, diff_any = 0;
  for (int t = 0; t < trials; ++t) {
    float ref[64] = {0};
    for (int l = 0; l < 64; ++l) ref[a[t * 64 + l]] += v[t * 64 + l];
    bool ok = true;
    for (int b = 0; b < 64; ++b) ok = ok && (o[t * 64 + b] == ref[b]);
    // would another order give a different result?  (reverse lane order)
    float rev[64] = {0};
    for (int l = 63; l >= 0; --l) rev[a[t * 64 + l]] += v[t * 64 + l];
    bool sens = false;
    for (int b = 0; b < 64; ++b) sens = sens || (rev[b] != ref[b]);
    lane_order += ok;
    differ += sens;
    diff_any += sens && ok;
  }
  printf("trials %d: lane-order result %d, order-sensitive trials %d, of which lane-order %d\n",
         trials, lane_order, differ, diff_any);
  return 0;
}
