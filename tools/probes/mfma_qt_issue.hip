// Issue-rate probe for the ring matcher's hot block, registers only (no LDS, no memory in
// the loop): per wave and "subtile", QT tiles x 2 dependent v_mfma_i32_16x16x64_i8 (a0 then
// a1 into the same accumulator, as match_unit), optionally the previous subtile's prefilter
// (v_max + v_max3 + v_cmp per tile -> ballot) and its scalar branch.  8 waves per
// work-group (2 per SIMD), one work-group per CU, 256 work-groups; reports the whole chip's
// int8 rate from the launch's events against the 5 POP/s dense peak.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/mfma_qt_issue.hip -o /tmp/mqi
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>

typedef __attribute__((ext_vector_type(4))) int i32x4;

// MODE 0: MFMAs only; 1: + prefilter VALU; 2: + ballot / branch; 3: + the next subtile's A
// fragments and c words from LDS (3 ds_read_b128, as the ring kernel); 4: the same two
// subtiles ahead; 5: the two fragment reads only (c in registers); 6: 5 + the LDS-DMA refill
// at the kernel's bytes per subtile (the compiler then drains the LDS counter per read).  (Modes 3 / 4 also add the loaded c to the running c -- 4 v_add per subtile
// the ring kernel does not have -- so they overstate the reads' cost by that VALU.)
template <int QT, int MODE>
__global__ __launch_bounds__(512, 1) void probe(const i32x4* __restrict__ in, int* out, int iters,
                                                unsigned long long* clk, const uint8_t* __restrict__ g) {
  __shared__ i32x4 lds[8 * 3 * 64];
  __shared__ __attribute__((aligned(16))) uint8_t ring[16 * 1024];   // MODE 6: LDS-DMA target
  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 8 * 3 * 64; i += blockDim.x) lds[i] = in[i % (64 * 16)];
  __syncthreads();
  i32x4 bq[QT][2];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    bq[t][0] = in[(2 * t) * 64 + lane];
    bq[t][1] = in[(2 * t + 1) * 64 + lane];
  }
  i32x4 a0 = in[2 * QT * 64 + lane], a1 = in[(2 * QT + 1) * 64 + lane], c = in[(2 * QT + 2) * 64 + lane];
  i32x4 a0n = a0, a1n = a1, cn = c;   // (MODE 4: the operands one subtile ahead)
  i32x4 accp[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) accp[t] = i32x4{INT_MIN, INT_MIN, INT_MIN, INT_MIN};
  int thr = INT_MAX - 1, hits = 0;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      i32x4 acc[QT];
#pragma unroll
      for (int t = 0; t < QT; ++t)   // (mode 0: one chain per tile across subtiles, all live)
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq[t][0], MODE == 0 ? accp[t] : c, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq[t][1], acc[t], 0, 0, 0);
      if constexpr (MODE == 3) {   // next subtile's operands (8 subtiles' images, cycled)
        const int nu = (u + 1) & 7;
        a0 = lds[(nu * 3) * 64 + lane];
        a1 = lds[(nu * 3 + 1) * 64 + lane];
        c = lds[(nu * 3 + 2) * 64 + (lane >> 4) * 16] + c;
      } else if constexpr (MODE == 5) {   // the fragments only (c words held for the stage)
        const int nu = (u + 1) & 7;
        a0 = lds[(nu * 3) * 64 + lane];
        a1 = lds[(nu * 3 + 1) * 64 + lane];
        c[0] += 1;
      } else if constexpr (MODE == 6) {   // mode 5 + the ring's LDS-DMA refill rate: one 1 KiB
        const int nu = (u + 1) & 7;       // piece per wave on 2 of every 8 subtiles (2 KiB
        a0 = lds[(nu * 3) * 64 + lane];   // per subtile and CU, as the kernel's 64 KiB stage
        a1 = lds[(nu * 3 + 1) * 64 + lane];   // over 32 subtiles)
        c[0] += 1;
        if (u < 2) {
          const uint8_t* src = g + ((int64_t)blockIdx.x * 1024 + (it & 63) * 16 + wv * 2 + u) * 1024;
          __builtin_amdgcn_global_load_lds(src + lane * 16,
                                           (__attribute__((address_space(3))) void*)(ring + (wv * 2 + u) * 1024),
                                           16, 0, 0);
        }
        // (loads of three iterations ago must have landed: ~24 subtiles of prefetch window,
        // as the kernel's one 32-subtile stage)
        if (u == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else if constexpr (MODE == 4) {   // two subtiles ahead
        const int nu = (u + 2) & 7;
        a0 = a0n;
        a1 = a1n;
        c = cn + c;
        a0n = lds[(nu * 3) * 64 + lane];
        a1n = lds[(nu * 3 + 1) * 64 + lane];
        cn = lds[(nu * 3 + 2) * 64 + (lane >> 4) * 16];
      }
      if constexpr (MODE >= 1) {
        uint64_t any = 0;
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          const int m = max(max(accp[t][0], accp[t][1]), max(accp[t][2], accp[t][3]));
          any |= __builtin_amdgcn_ballot_w64(m >= thr);
        }
#pragma unroll
        for (int i = 0; i < 2 * QT; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
          if (i < 3 * QT / 2) __builtin_amdgcn_sched_group_barrier(0x2, 2, 0);
        }
        if constexpr (MODE >= 2) {
          if (__builtin_expect(any != 0, 0)) {   // never taken (thr is above every value)
            ++hits;
            thr = max(thr, accp[0][0]);
          }
        } else {
          hits += any != 0;
        }
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) accp[t] = acc[t];
      c[0] += 1;   // a different init per subtile: no two MFMAs alike (no CSE)
    }
  }
  int s = hits;
#pragma unroll
  for (int t = 0; t < QT; ++t) s += accp[t][0] + accp[t][1] + accp[t][2] + accp[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    clk[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int QT, int MODE>
int run(const i32x4* in, int* out, unsigned long long* clk, unsigned long long* hclk,
        const uint8_t* g) {
  const int iters = 2000, nwg = 256;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((probe<QT, MODE>), dim3(nwg), dim3(512), 0, 0, in, out, iters, clk, g);
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  CK(hipMemcpy(hclk, clk, nwg * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double cyc = 0, rt = 0;
  for (int b = 0; b < nwg; ++b) { cyc += hclk[2 * b]; rt += hclk[2 * b + 1]; }
  cyc /= nwg;
  rt /= nwg;
  const double mfma_per_simd = 2.0 * iters * 8 * 2 * QT;   // 2 waves per SIMD
  // whole-chip int8 rate from the launch's own events: every SIMD of every work-group's CU
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const double ops = (double)nwg * 4 * mfma_per_simd * 32768.0;
  // (wave 0's own s_memtime span covers only part of the launch: the SIMD's older wave gets
  // the MFMA pipe first, so only the launch's events give the rate)
  printf("QT %d mode %d: launch %.3f ms = %.2f POP/s int8 = %.1f %% of 5 (%d CUs, wave-0 clock "
         "%.2f GHz)\n", QT, MODE, ms, ops / (ms * 1e-3) / 1e15, ops / (ms * 1e-3) / 5e15 * 100.0,
         ncu, cyc / rt * 0.1);
  return 0;
}

int main() {
  i32x4* in;
  int* out;
  unsigned long long *clk, hclk[512];
  CK(hipMalloc(&in, 64 * 64 * sizeof(i32x4)));
  CK(hipMemset(in, 1, 64 * 64 * sizeof(i32x4)));
  CK(hipMalloc(&out, 256 * 512 * sizeof(int)));
  CK(hipMalloc(&clk, 512 * sizeof(unsigned long long)));
  uint8_t* g;   // 256 work-groups x 64 x 16 KiB of DMA source (256 MiB: streamed, past the caches)
  CK(hipMalloc(&g, (size_t)256 * 1024 * 1024));
  CK(hipMemset(g, 3, (size_t)256 * 1024 * 1024));
  if (run<2, 0>(in, out, clk, hclk, g) || run<2, 1>(in, out, clk, hclk, g) || run<2, 2>(in, out, clk, hclk, g) ||
      run<2, 3>(in, out, clk, hclk, g) || run<4, 0>(in, out, clk, hclk, g) || run<4, 2>(in, out, clk, hclk, g) ||
      run<2, 4>(in, out, clk, hclk, g) || run<2, 5>(in, out, clk, hclk, g) || run<4, 5>(in, out, clk, hclk, g) ||
      run<2, 6>(in, out, clk, hclk, g) || run<4, 6>(in, out, clk, hclk, g) ||
      run<2, 7>(in, out, clk, hclk, g) || run<4, 7>(in, out, clk, hclk, g) || run<4, 3>(in, out, clk, hclk, g) || run<4, 4>(in, out, clk, hclk, g) ||
      run<8, 0>(in, out, clk, hclk, g) || run<8, 2>(in, out, clk, hclk, g) || run<8, 3>(in, out, clk, hclk, g) ||
      run<8, 4>(in, out, clk, hclk, g))
    return 1;
  return 0;
}
