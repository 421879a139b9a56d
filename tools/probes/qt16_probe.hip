// Skeleton probe for VERDICT r5's C3 route "QT-16, one wave per SIMD": the matcher's hot
// block with its LDS fragment reads, sustained (~1.5 s back to back) on operand bytes from a
// file (SIFT-like, tools/probes/sift_operand_bytes.py), in these shapes:
//   QT 8, 8 waves (2 per SIMD)  -- the kernel's shape
//   QT 16, 4 waves (1 per SIMD) -- half the LDS fragment reads per MFMA, no partner wave
//                                  (256 accumulator + operand registers: accumulators in AGPRs)
//   QT 12, 4 waves              -- the largest one-wave shape whose registers stay in VGPRs
//   QT 8, 4 waves               -- the kernel's tile count without the partner wave
// Per wave and subtile: 2 QT MFMAs (a0 then a1 into one accumulator per tile), the previous
// subtile's prefilter (max3, max, compare -> ballot per tile, one branch), and the next
// subtile's two fragments + c words from LDS (8 subtile images cycled).  The QT-16 shape keeps
// two named accumulator banks (even / odd subtile) so no accumulator is copied.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/qt16_probe.hip -o tools/probes/qt16_probe
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) int i32x4;

template <int QT>
__device__ __forceinline__ void prefilter(const i32x4 (&acc)[QT], int thr, int& hits) {
  uint64_t any = 0;
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int m = max(max(acc[t][0], acc[t][1]), max(acc[t][2], acc[t][3]));
    any |= __builtin_amdgcn_ballot_w64(m >= thr);
  }
#pragma unroll
  for (int i = 0; i < 2 * QT; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);                          // MFMA
    if (i < 3 * QT / 2) __builtin_amdgcn_sched_group_barrier(0x2, 2, 0);     // VALU
    if (i >= 1 && i <= 4) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
  }
  if (__builtin_expect(any != 0, 0)) ++hits;
}

template <int QT>
__device__ __forceinline__ void body(const i32x4* __restrict__ in, int* out, int iters,
                                     unsigned long long* clk) {
  __shared__ i32x4 lds[8 * 3 * 64];   // 8 subtile images: a0, a1, c (per lane)
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 8 * 3 * 64; i += blockDim.x) lds[i] = in[(64 + i) % 4096];
  __syncthreads();
  i32x4 bq[QT][2];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    bq[t][0] = in[(2 * t) * 64 + lane];
    bq[t][1] = in[(2 * t + 1) * 64 + lane];
  }
  i32x4 a0 = lds[0 * 64 + lane], a1 = lds[1 * 64 + lane], c = lds[2 * 64 + lane];
  i32x4 accA[QT], accB[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) accB[t] = i32x4{INT_MIN, INT_MIN, INT_MIN, INT_MIN};
  int thr = INT_MAX - 1, hits = 0;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      // even subtile into bank A (prefilter of bank B), odd into bank B (prefilter of A)
#pragma unroll
      for (int t = 0; t < QT; ++t) accA[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq[t][0], c, 0, 0, 0);
      {
        const int nu = (u + 1) & 7;
        a0 = lds[(nu * 3) * 64 + lane];
        a1 = lds[(nu * 3 + 1) * 64 + lane];
        c = lds[(nu * 3 + 2) * 64 + (lane >> 4) * 16];
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) accA[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq[t][1], accA[t], 0, 0, 0);
      prefilter<QT>(accB, thr, hits);
#pragma unroll
      for (int t = 0; t < QT; ++t) accB[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq[t][0], c, 0, 0, 0);
      {
        const int nu = (u + 2) & 7;
        a0 = lds[(nu * 3) * 64 + lane];
        a1 = lds[(nu * 3 + 1) * 64 + lane];
        c = lds[(nu * 3 + 2) * 64 + (lane >> 4) * 16];
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) accB[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq[t][1], accB[t], 0, 0, 0);
      prefilter<QT>(accA, thr, hits);
    }
  }
  int s = hits;
#pragma unroll
  for (int t = 0; t < QT; ++t) s += accA[t][0] + accB[t][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// A: the compiler's register split (one wave per SIMD leaves it 512 registers and it puts the
// MFMA results in AGPRs, which the prefilter must copy out with v_accvgpr_read).  V: the
// same body held to 256 registers (two waves' budget), so accumulators stay in VGPRs.
template <int QT, int NW>
__global__ __launch_bounds__(NW * 64, 1) void probe(const i32x4* __restrict__ in, int* out, int iters,
                                                    unsigned long long* clk) {
  body<QT>(in, out, iters, clk);
}
template <int QT, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2)))
void probe_v(const i32x4* __restrict__ in, int* out, int iters, unsigned long long* clk) {
  body<QT>(in, out, iters, clk);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int QT, int NW, bool V = false>
int run(const i32x4* in, int* out, unsigned long long* clk) {
  const int iters = 16000 / QT, nwg = 256;   // equal MFMAs per wave for every shape
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> h(2 * nwg);
  const int nlaunch = 440;
  float ms = 0;
  double ghz = 0;
  for (int rep = 0; rep < nlaunch; ++rep) {
    if (rep == nlaunch - 20) CK(hipEventRecord(e0, 0));
    if (V)
      hipLaunchKernelGGL((probe_v<QT, NW>), dim3(nwg), dim3(NW * 64), 0, 0, in, out, iters, clk);
    else
      hipLaunchKernelGGL((probe<QT, NW>), dim3(nwg), dim3(NW * 64), 0, 0, in, out, iters, clk);
  }
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 20;
  CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  for (int b = 0; b < nwg; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1 / nwg;
  // MFMAs per launch: work-groups x waves x iterations x 8 subtiles x 2 QT
  const double ops = (double)nwg * NW * iters * 8 * 2 * QT * 32768.0;
  printf("QT %2d, %d waves per work-group%s: %.3f ms per launch = %.2f POP/s = %.1f %% of 5 POP/s; "
         "clock %.2f GHz\n", QT, NW, V ? " (VGPR accumulators)" : "", ms, ops / (ms * 1e-3) / 1e15, ops / (ms * 1e-3) / 5e15 * 100.0,
         ghz);
  return 0;
}

int main(int argc, char** argv) {
  const int nvec = 64 * 64;
  i32x4* in;
  int* out;
  unsigned long long* clk;
  CK(hipMalloc(&in, nvec * sizeof(i32x4)));
  CK(hipMalloc(&out, 256 * 512 * sizeof(int)));
  CK(hipMalloc(&clk, 512 * sizeof(unsigned long long)));
  std::vector<int> h(nvec * 4);
  FILE* f = argc > 1 ? fopen(argv[1], "rb") : nullptr;
  if (!f || fread(h.data(), 4, h.size(), f) != h.size()) {
    printf("usage: qt16_probe OPERAND_BYTES (64 KiB)\n");
    return 1;
  }
  fclose(f);
  CK(hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  if (run<8, 8>(in, out, clk) || run<16, 4>(in, out, clk) || run<12, 4>(in, out, clk) ||
      run<8, 4>(in, out, clk) || run<12, 4, true>(in, out, clk) || run<8, 4, true>(in, out, clk) ||
      run<8, 8>(in, out, clk))
    return 1;
  return 0;
}
