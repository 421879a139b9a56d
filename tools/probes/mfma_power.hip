// Sustained-clock probe for the int8 MFMA at C3's shape: is the matcher's clock drop under
// load (1.98-2.27 GHz in the PMC passes, against the 2.4 GHz the 5 POP/s peak is quoted at)
// a property of the MFMA pipe on real data, or of the VALU / LDS work around it?
// The hot block of match_unit at 8 query tiles per wave, registers only: per wave and
// "subtile" 8 tiles x 2 dependent v_mfma_i32_16x16x64_i8; MODE 1 adds the prefilter (max3,
// max, compare -> ballot per tile, one scalar branch).  8 waves per work-group, one
// work-group per CU, 256 work-groups.  Operands either all-ones (no toggling) or random
// bytes (the A operand rotates through 8 random subtile images per iteration, like a DB
// stream).  Each configuration runs back to back for ~1.5 s; the rate of the last launches
// is reported, with the clock from s_memtime / s_memrealtime of wave 0 of each work-group.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/mfma_power.hip -o /tmp/mfma_power
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) int i32x4;
constexpr int QT = 8;

template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(const i32x4* __restrict__ in, int* out, int iters,
                                                unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  i32x4 bq[QT][2];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    bq[t][0] = in[(2 * t) * 64 + lane];
    bq[t][1] = in[(2 * t + 1) * 64 + lane];
  }
  // 8 subtile images of A (2 fragments each) + c words, rotated per subtile
  i32x4 a[8][2];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    a[u][0] = in[(2 * QT + 2 * u) * 64 + lane];
    a[u][1] = in[(2 * QT + 2 * u + 1) * 64 + lane];
  }
  const i32x4 c = in[(2 * QT + 16) * 64 + lane];
  i32x4 accp[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) accp[t] = i32x4{INT_MIN, INT_MIN, INT_MIN, INT_MIN};
  int thr = INT_MAX - 1, hits = 0;
  [[maybe_unused]] int wmax[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) wmax[t] = INT_MIN;
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
      for (int t = 0; t < QT; ++t)
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u][0], bq[t][0], MODE == 0 ? accp[t] : c, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u][1], bq[t][1], acc[t], 0, 0, 0);
      if constexpr (MODE >= 2) {
        // prefilter windows of W = 2 (MODE 2) or 4 (MODE 3) subtiles: a running max per tile
        // (max3 folds two new values into it: 2 VALU per tile and subtile), one compare /
        // ballot / branch per tile at the window's last subtile
        constexpr int W = MODE == 2 ? 2 : 4;
        uint64_t any = 0;
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          const int m0 = (u % W == 0) ? max(max(accp[t][0], accp[t][1]), accp[t][2])
                                      : max(max(wmax[t], accp[t][0]), accp[t][1]);
          wmax[t] = (u % W == 0) ? max(m0, accp[t][3]) : max(max(m0, accp[t][2]), accp[t][3]);
          if (u % W == W - 1) any |= __builtin_amdgcn_ballot_w64(wmax[t] >= thr);
        }
#pragma unroll
        for (int i = 0; i < 2 * QT; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
          if (i < (u % W == W - 1 ? 3 * QT / 2 : QT)) __builtin_amdgcn_sched_group_barrier(0x2, 2, 0);
        }
        if (u % W == W - 1 && __builtin_expect(any != 0, 0)) ++hits;
      }
      if constexpr (MODE == 1) {
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
        if (__builtin_expect(any != 0, 0)) ++hits;
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) accp[t] = acc[t];
    }
  }
  int s = hits;
#pragma unroll
  for (int t = 0; t < QT; ++t) s += accp[t][0] + accp[t][1] + accp[t][2] + accp[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// the same for the 32x32x32 shape (impl i8w's): 4 tiles of 32 queries per wave (the ring's
// 128 queries), a 32-row "subtile" = 4 k-steps x 4 tiles = 16 MFMAs (twice the work of the
// 16x16x64 subtile), tile-major with the previous tile's prefilter beside the current tile's
// chain (two max3 chains over its 16 values + combine + compare: 8 VALU + ballot); MODE 1 adds
// that prefilter
typedef __attribute__((ext_vector_type(16))) int i32x16;
template <int MODE>
__global__ __launch_bounds__(512, 1) void probe_w(const i32x4* __restrict__ in, int* out, int iters,
                                                  unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  i32x4 bq[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int k = 0; k < 4; ++k) bq[t][k] = in[(4 * t + k) * 64 + lane];
  i32x4 a[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[u][k] = in[(16 + 4 * u + k) * 64 + lane];
  i32x16 c;
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = in[(32 + i / 4) * 64 + lane][i & 3];
  i32x16 accp = c;
  int thr = INT_MAX - 1, hits = 0;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[u & 3][0], bq[t][0], MODE ? c : accp, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[u & 3][1], bq[t][1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[u & 3][2], bq[t][2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[u & 3][3], bq[t][3], acc, 0, 0, 0);
        if constexpr (MODE == 1) {
          const int ma = max(max(max(max(max(max(accp[0], accp[1]), accp[2]), accp[3]), accp[4]), accp[5]), accp[6]);
          const int mb = max(max(max(max(max(max(accp[7], accp[8]), accp[9]), accp[10]), accp[11]), accp[12]), accp[13]);
          const int m = max(max(ma, mb), max(accp[14], accp[15]));
          if (__builtin_expect(__builtin_amdgcn_ballot_w64(m >= thr) != 0, 0)) ++hits;
        }
        accp = acc;
      }
    }
  }
  int s = hits;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += accp[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int MODE>
int run_w(const char* data, const i32x4* in, int* out, unsigned long long* clk);

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int MODE>
int run(const char* data, const i32x4* in, int* out, unsigned long long* clk) {
  const int iters = 2000, nwg = 256;   // ~3.4 ms per launch at 2.4 GHz
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> h(2 * nwg);
  const int nlaunch = 440;   // ~1.5 s back to back
  float last = 0;
  double ghz = 0;
  CK(hipEventRecord(e0, 0));
  for (int rep = 0; rep < nlaunch; ++rep) {
    if (rep == nlaunch - 20) CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((probe<MODE>), dim3(nwg), dim3(512), 0, 0, in, out, iters, clk);
  }
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventElapsedTime(&last, e0, e1));
  last /= 20;
  CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  for (int b = 0; b < nwg; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1 / nwg;
  const double ops = (double)nwg * 4 * (2.0 * iters * 8 * 2 * QT) * 32768.0;
  printf("%-14.14s data, mode %d (%s): %.3f ms per launch (last 20 of %d) = %.2f POP/s = %.1f %% of "
         "5 POP/s; last launch's clock %.2f GHz\n", data, MODE,
         MODE == 0 ? "MFMA only" : MODE == 1 ? "MFMA + prefilter" : MODE == 2 ? "MFMA + 2-subtile windows" : "MFMA + 4-subtile windows", last, nlaunch, ops / (last * 1e-3) / 1e15,
         ops / (last * 1e-3) / 5e15 * 100.0, ghz);
  return 0;
}

template <int MODE>
int run_w(const char* data, const i32x4* in, int* out, unsigned long long* clk) {
  const int iters = 1000, nwg = 256;   // same op count per launch as the 16x16x64 probe
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> h(2 * nwg);
  const int nlaunch = 440;
  float last = 0;
  double ghz = 0;
  for (int rep = 0; rep < nlaunch; ++rep) {
    if (rep == nlaunch - 20) CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((probe_w<MODE>), dim3(nwg), dim3(512), 0, 0, in, out, iters, clk);
  }
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventElapsedTime(&last, e0, e1));
  last /= 20;
  CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  for (int b = 0; b < nwg; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1 / nwg;
  const double ops = (double)nwg * 4 * (2.0 * iters * 8 * 16) * 65536.0;
  printf("%-14.14s data, 32x32x32 %s: %.3f ms per launch = %.2f POP/s = %.1f %% of 5 POP/s; "
         "clock %.2f GHz\n", data, MODE ? "MFMA + prefilter" : "MFMA only", last,
         ops / (last * 1e-3) / 1e15, ops / (last * 1e-3) / 5e15 * 100.0, ghz);
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
  for (auto& v : h) v = 0x01010101;
  CK(hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  if (run<0>("ones", in, out, clk) || run<1>("ones", in, out, clk) || run<3>("ones", in, out, clk)) return 1;
  if (argc > 1) {   // operand bytes from a file (e.g. SIFT-like descriptors shifted by -128)
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(h.data(), 4, h.size(), f) != h.size()) {
      printf("cannot read %s\n", argv[1]);
      return 1;
    }
    fclose(f);
    CK(hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    if (argc > 2 && argv[2][0] == 'w') {   // "w": the 32x32x32 shape against 16x16x64
      if (run<1>(argv[1], in, out, clk) || run_w<0>(argv[1], in, out, clk) ||
          run_w<1>(argv[1], in, out, clk))
        return 1;
      return 0;
    }
    if (run<0>(argv[1], in, out, clk) || run<1>(argv[1], in, out, clk)) return 1;
    if (argc > 2) return 0;   // (a second argument: the file's lines only)
  }
  srand(12345);
  for (auto& v : h) v = (rand() & 0xffff) | ((rand() & 0xffff) << 16);
  CK(hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  if (run<0>("random", in, out, clk) || run<1>("random", in, out, clk) ||
      run<2>("random", in, out, clk) || run<3>("random", in, out, clk) || run<1>("random", in, out, clk))
    return 1;
  return 0;
}
