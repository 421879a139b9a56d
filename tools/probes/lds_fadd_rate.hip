// LDS float-atomic throughput on gfx950: one wave per CU issues N return-less ds_add_f32
// (atomicAdd on __shared__ float) with a chosen address pattern; cycles from s_memtime around
// the loop (plus a final lgkmcnt(0) wait).  Patterns: 0 = 64 distinct banks, 1 = 8 groups of 8
// lanes on one address each (8-way same address), 2 = all 64 lanes on one address,
// 3 = 8 active lanes (distinct banks), 4 = ds_add_u32 on 64 distinct banks (integer).
// hipcc --offload-arch=gfx950 -O2 tools/probes/lds_fadd_rate.hip -o tools/probes/lds_fadd_rate
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int pattern, int n, unsigned long long* out, float* sink) {
  __shared__ float h[4096];
  __shared__ unsigned hu[4096];
  const int lane = threadIdx.x;
  for (int i = lane; i < 4096; i += 64) { h[i] = 0.f; hu[i] = 0u; }
  __syncthreads();
  int a = lane;
  if (pattern == 1) a = (lane >> 3) * 97;
  if (pattern == 2) a = 0;
  const bool act = pattern != 3 || lane < 8;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (act) {
    if (pattern == 4) {
      for (int i = 0; i < n; ++i) atomicAdd(&hu[(a + 64 * (i & 31)) & 4095], 1u);
    } else {
      for (int i = 0; i < n; ++i) atomicAdd(&h[(a + 64 * (i & 31)) & 4095], 1.0f);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x] = t1 - t0;
  if (lane == 0) sink[blockIdx.x] = h[5] + (float)hu[5];
}

int main() {
  unsigned long long* d;
  float* s;
  hipMalloc(&d, 1024 * 8);
  hipMalloc(&s, 1024 * 4);
  const int n = 4096;
  const char* names[] = {"64 distinct banks", "8-way same address", "64-way same address",
                         "8 active lanes", "ds_add_u32 64 banks"};
  for (int p = 0; p < 5; ++p) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(probe, dim3(256), dim3(64), 0, 0, p, n, d, s);
      hipDeviceSynchronize();
    }
    unsigned long long h[256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    unsigned long long mx = 0, sum = 0;
    for (int i = 0; i < 256; ++i) { sum += h[i]; mx = h[i] > mx ? h[i] : mx; }
    const double avg = (double)sum / 256;
    printf("%-22s %7.1f cycles per instruction (s_memtime units), %.2f per active lane\n", names[p],
           avg / n, avg / n / (p == 3 ? 8 : 64));
  }
  return 0;
}
