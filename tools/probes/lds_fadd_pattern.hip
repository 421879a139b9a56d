// LDS float-atomic cost by address pattern and by waves per CU on gfx950 (a follow-up to
// lds_fadd_rate.hip, for the SIFT descriptor's histogram adds).  Each wave of a work-group
// issues N return-less ds_add_f32 on its own 4 KiB region; cycles (s_memtime) per
// instruction, averaged over the waves.  Patterns:
//   0  64 lanes, 64 distinct banks
//   1  descriptor-like: lane 8s+e -> base(s) + off(e), base shared by 4 consecutive s
//      (4-way same address per e), off = {0,1,10,11,60,61,70,71}
//   2  as 1 with 36 % of the lanes masked off (lanes whose e is 2 or 6, and s odd for e 3)
//   3  32 active lanes (even lanes), distinct banks
//   4  as 1 with base shared by all 8 s (8-way same address per e)
// hipcc --offload-arch=gfx950 -O2 tools/probes/lds_fadd_pattern.hip -o tools/probes/lds_fadd_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int pattern, int n, unsigned long long* out, float* sink) {
  __shared__ float hh[16][1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* h = hh[wv];
  for (int i = lane; i < 1024; i += 64) h[i] = 0.f;
  __syncthreads();
  const int s = lane >> 3, e = lane & 7;
  const int offs[8] = {0, 1, 10, 11, 60, 61, 70, 71};
  int a = lane;
  bool act = true;
  if (pattern == 1 || pattern == 2) a = 100 + (s >> 2) + offs[e];
  if (pattern == 2) act = !(e == 2 || e == 6 || (e == 3 && (s & 1)));
  if (pattern == 3) act = !(lane & 1);
  if (pattern == 4) a = 100 + offs[e];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (act)
    for (int i = 0; i < n; ++i) atomicAdd(&h[(a + 128 * (i & 3)) & 1023], 1.0f);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * 16 + wv] = t1 - t0;
  if (lane == 0) sink[blockIdx.x * 16 + wv] = h[5];
}

int main() {
  unsigned long long* d;
  float* sk;
  hipMalloc(&d, 256 * 16 * 8);
  hipMalloc(&sk, 256 * 16 * 4);
  const int n = 2048;
  const char* names[] = {"64 distinct banks", "descriptor 4-way", "descriptor 4-way, 36% off",
                         "32 active lanes", "descriptor 8-way"};
  for (int waves = 1; waves <= 8; waves *= 2)
    for (int p = 0; p < 5; ++p) {
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe, dim3(256), dim3(64 * waves), 0, 0, p, n, d, sk);
        hipDeviceSynchronize();
      }
      static unsigned long long h[256 * 16];
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      double sum = 0;
      for (int b = 0; b < 256; ++b)
        for (int w = 0; w < waves; ++w) sum += (double)h[b * 16 + w];
      const double avg = sum / (256 * waves);
      printf("waves/CU %d  %-28s %7.1f cycles per instruction per wave\n", waves, names[p], avg / n);
    }
  return 0;
}
