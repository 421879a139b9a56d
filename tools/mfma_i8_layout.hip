// Verify the operand lane map of v_mfma_i32_16x16x64_i8 with exact, asymmetric integer
// data (cdna_hip_programming.md §3: "other dtypes: check the map with exact integer data").
// Hypothesis H: lane l holds A[row l&15][k = 16*(l>>4) + j] and B[k = 16*(l>>4) + j][col l&15],
// j = 0..15 (one byte each); D: col = l&15, row = 4*(l>>4) + reg.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_layout.hip -o /tmp/mfma_i8 && /tmp/mfma_i8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) int i32x4;

__global__ void k(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x;
  long a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  unsigned char av[16], bv[16];
  for (int j = 0; j < 16; ++j) {
    av[j] = (unsigned char)A[(l & 15) * 64 + 16 * (l >> 4) + j];   // A row-major [16][64]
    bv[j] = (unsigned char)B[(16 * (l >> 4) + j) * 16 + (l & 15)]; // B row-major [64][16]
  }
  for (int j = 0; j < 8; ++j) {
    a0 |= (long)av[j] << (8 * j);
    a1 |= (long)av[8 + j] << (8 * j);
    b0 |= (long)bv[j] << (8 * j);
    b1 |= (long)bv[8 + j] << (8 * j);
  }
  typedef __attribute__((ext_vector_type(4))) int iv4;
  iv4 a = {(int)(a0 & 0xffffffff), (int)(a0 >> 32), (int)(a1 & 0xffffffff), (int)(a1 >> 32)};
  iv4 b = {(int)(b0 & 0xffffffff), (int)(b0 >> 32), (int)(b1 & 0xffffffff), (int)(b1 >> 32)};
  i32x4 c = {0, 0, 0, 0};
  i32x4 d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = d[r];
}

// 32x32x32 i8: hypothesis lane l holds A[row l&31][k = 16*(l>>5) + j], B[k = 16*(l>>5) + j][col l&31];
// D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5) (dtype-independent C/D map)
typedef __attribute__((ext_vector_type(16))) int i32x16;
__global__ void k32(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x;
  unsigned av[4] = {0, 0, 0, 0}, bv[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16; ++j) {
    av[j >> 2] |= (unsigned)(unsigned char)A[(l & 31) * 32 + 16 * (l >> 5) + j] << (8 * (j & 3));
    bv[j >> 2] |= (unsigned)(unsigned char)B[(16 * (l >> 5) + j) * 32 + (l & 31)] << (8 * (j & 3));
  }
  typedef __attribute__((ext_vector_type(4))) int iv4;
  iv4 a = {(int)av[0], (int)av[1], (int)av[2], (int)av[3]};
  iv4 b = {(int)bv[0], (int)bv[1], (int)bv[2], (int)bv[3]};
  i32x16 c = {};
  i32x16 d = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = d[r];
}

static int test32() {
  signed char hA[32 * 32], hB[32 * 32];
  int ref[32 * 32], got[32 * 32];
  for (int i = 0; i < 32 * 32; ++i) hA[i] = (signed char)(rand() % 256 - 128);
  for (int i = 0; i < 32 * 32; ++i) hB[i] = (signed char)(rand() % 256 - 128);
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 32; ++c) {
      int s = 0;
      for (int k = 0; k < 32; ++k) s += hA[r * 32 + k] * hB[k * 32 + c];
      ref[r * 32 + c] = s;
    }
  signed char *dA, *dB;
  int* dD;
  if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dD, sizeof got)) return 2;
  if (hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice) ||
      hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice)) return 2;
  hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  if (hipMemcpy(got, dD, sizeof got, hipMemcpyDeviceToHost)) return 2;
  int bad = 0;
  for (int i = 0; i < 1024; ++i) bad += got[i] != ref[i];
  printf("i8 32x32x32 layout hypothesis: %s (%d/1024 mismatches)\n", bad ? "WRONG" : "OK", bad);
  return bad ? 1 : 0;
}

// v_permlane32_swap / v_permlane16_swap of a register with itself: the two results hold
// {x_l, x_(l^32)} / {x_l, x_(l^16)} (the shared-threshold reduction in match_i8.hip)
__global__ void kswap(int* o) {
  const unsigned x = threadIdx.x * 7u + 3u;
  const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  const auto q = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const unsigned l = threadIdx.x;
  const unsigned e32 = (l ^ 32) * 7u + 3u, e16 = (l ^ 16) * 7u + 3u;
  const bool ok32 = (p[0] == x && p[1] == e32) || (p[0] == e32 && p[1] == x);
  const bool ok16 = (q[0] == x && q[1] == e16) || (q[0] == e16 && q[1] == x);
  o[l] = (ok32 ? 0 : 1) | (ok16 ? 0 : 2);
}

static int test_swap() {
  int* d;
  int h[64];
  if (hipMalloc(&d, sizeof h)) return 2;
  hipLaunchKernelGGL(kswap, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost)) return 2;
  int b32 = 0, b16 = 0;
  for (int i = 0; i < 64; ++i) {
    b32 += h[i] & 1;
    b16 += (h[i] >> 1) & 1;
  }
  printf("permlane32_swap pair hypothesis: %s (%d/64)\n", b32 ? "WRONG" : "OK", b32);
  printf("permlane16_swap pair hypothesis: %s (%d/64)\n", b16 ? "WRONG" : "OK", b16);
  return (b32 || b16) ? 1 : 0;
}

int main() {
  signed char hA[16 * 64], hB[64 * 16];
  int ref[16 * 16], got[16 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (signed char)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (signed char)(rand() % 256 - 128);
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += hA[r * 64 + k] * hB[k * 16 + c];
      ref[r * 16 + c] = s;
    }
  signed char *dA, *dB;
  int* dD;
  if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dD, sizeof got)) return 2;
  if (hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice) ||
      hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice)) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  if (hipMemcpy(got, dD, sizeof got, hipMemcpyDeviceToHost)) return 2;
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += got[i] != ref[i];
  printf("i8 16x16x64 layout hypothesis H: %s (%d/256 mismatches)\n", bad ? "WRONG" : "OK", bad);
  return (bad ? 1 : 0) | test32() | test_swap();
}
