// match_i8.hip -- the brute-force k=2 matcher on the int8 MFMA (v_mfma_i32_16x16x64_i8),
// twice the bf16 MFMA rate, exact.
//
// SIFT values are integers 0..255; shifted by -128 they are int8, and the L2 distance is
// shift-invariant: ||q - d||^2 = ||q'||^2 + ||d'||^2 - 2 q'.d'  (q' = q - 128, d' = d - 128).
// The MFMA accumulates q'.d' exactly in i32 (|q'.d'| <= 2^21).  Minimising the distance
// is maximising y = 2 q'.d' - ||d'||^2; -2 does not fit the int8 operands, so the row
// norm is folded into the accumulator init as c = floor(-||d'||^2 / 2) (w = -||d'||^2 is
// stored per row as c = w >> 1 and its parity p = w & 1).  The MFMA then yields
// h = q'.d' + c and y = 2h + p:
// ordering by y is ordering by h with the parity bit as tiebreak, and max(h) >=
// floor(y2 / 2) is a NECESSARY condition for a row to beat the running second best y2 --
// so the fast path needs no per-element op (3 VALU per 16x16 tile, like the bf16 path).
// The two largest y per query (= two smallest distances) are tracked exactly;
// distance^2 = ||q'||^2 - y, exact in f32 (< 2^24).
//
// Layout (operand lane map verified on hardware, tools/mfma_i8_layout.hip): lane l holds
// A[row l&15][k 16(l>>4)..+15] and B[k ..][col l&15]; D: col l&15, rows 4(l>>4)+r.  A 16-row
// subtile is [kstep 2][lane 64][16 B] = 2 KiB (the LDS image is the HBM image).
// Structure (cf. match.hip): queries stationary in VGPRs (64 per lane for 128 queries per
// wave), DB streamed through a 2-slot LDS-DMA ring of 512-row stages (prefetch distance 1,
// one barrier per stage), c read per subtile (parity on the slow path).  The prefilter of subtile u runs while
// the MFMAs of subtile u+1 are in flight (software pipeline: no MFMA->VALU stall), with
// one ballot + scalar branch per subtile and per 16x16 tile.  Each lane keeps the exact
// top-2 of its own rows; the threshold is the query's second best over its four lane
// groups (permlane swaps), so a query's slow path fires about as often as its top-2 changes.
// Work-groups are ordered XCD-aware: each XCD's L2 serves one or two DB chunks.
// Measured and rejected (C3, same device): a persistent work-queue kernel (more chunks =
// more top-2 restarts), a seeded threshold pre-pass (gain eaten by the pass), other
// shifts than -128 (slower), the 32x32x32 shape (impl 2, below: 9 VALU per 1024 pairs
// instead of 12 and half the MFMA issue holds, but the chip holds ~2.03 GHz on it vs ~2.2 on
// 16x16x64: 4.7 vs 4.0-4.2 ms; kept as an option).
#include <climits>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "sod_internal.h"

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((address_space(3))) void lds_void;

namespace {

// QT = 16-query tiles per wave (a template parameter: 8 for large query sets, 4 / 2 so that
// small ones still fill every wave and get longer DB chunks; launch_match_i8 chooses)
#ifndef SOD_I8_NW
#define SOD_I8_NW 8
#endif
// 16x16x64 kernel: one work-group of NW16 waves per CU slot.  With 8 waves (2 per SIMD)
// in ONE work-group the stage barrier keeps the two waves of a SIMD in step; two 4-wave
// work-groups per CU instead let the older one take issue priority, finish ~30 % earlier
// and leave the other running alone (one wave per SIMD) for the tail (measured with
// in-kernel stamps).
constexpr int NW16 = SOD_I8_NW;
constexpr int NT16 = NW16 * 64;
#ifndef SOD_I8_SPS
#define SOD_I8_SPS 32    // 512-row stages: 64 KiB, two slots (measured +1 % over 256-row x 3)
#endif
constexpr int SPS = SOD_I8_SPS;   // subtiles per stage (one barrier per stage)
constexpr int kStageRows = SPS * 16;
constexpr int kSub = 2048;     // bytes per 16-row subtile
constexpr int kStageBytes = SPS * kSub;          // 64 KiB
// per stage (128 rows) and wave w (its 128/NW16 rows): [c: i32 each | p: i32 each]
constexpr int kStageNorm = 2 * SPS * kSubRows * 4;   // c and parity words
// the norm words live in a ring of their own, one entry deeper than the descriptor ring:
// the parity words of a stage are read only on the slow path of its LAST subtile, which
// runs (software pipeline) after the next stage's barrier -- when that stage's refill
// already targets the descriptor slot
#ifndef SOD_I8_RING
#define SOD_I8_RING 2      // LDS stage slots (prefetch distance = RING - 1 stages)
#endif
constexpr int kNormRing = SOD_I8_RING + 1 > 4 ? SOD_I8_RING + 1 : 4;
constexpr int kPiecesPerWave = kStageBytes / 1024 / NW16;   // 1 KiB LDS-DMA pieces
constexpr int kPadNormI = 1 << 30;                        // ||d'||^2 of padding rows (w = -2^30)
static_assert(kStageBytes / 1024 % NW16 == 0, "pieces split evenly");

// pack: one thread per (row, 16-dim chunk c = 0..7); int8 of (value - 128); exact i32 norm
template <typename TIn, bool kWide>
__global__ void pack_i8_kernel(const TIn* __restrict__ src, int64_t n, int64_t npad,
                               uint8_t* __restrict__ pack, int* __restrict__ norms, int padnorm,
                               uint32_t* __restrict__ flags, int max_slot) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t >> 3;
  const int c = (int)(t & 7);
  if (row >= npad) return;   // npad*8 threads is a multiple of 64
  int v[16];
  uint32_t bad = 0;
  if (row < n) {
    if constexpr (sizeof(TIn) == 1) {
      const uint4 raw = *reinterpret_cast<const uint4*>(src + row * kDim + c * 16);
      const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (int)((w[j >> 2] >> (8 * (j & 3))) & 0xFF);
    } else {
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float4 f = *reinterpret_cast<const float4*>(src + row * kDim + c * 16 + 4 * j4);
        const float ff[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x = ff[j];
          const bool finite = (__float_as_uint(x) & 0x7f800000u) != 0x7f800000u;
          const bool ok = finite && x >= 0.f && x <= 255.f && x == truncf(x);
          bad |= ok ? 0u : 1u;
          v[4 * j4 + j] = ok ? (int)x : 0;
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 128;   // shifted to 0
  }
  int ss = 0, raw = 0;
  uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int s = v[j] - 128;
    ss += s * s;
    raw += v[j] * v[j];
    o[j >> 2] |= ((uint32_t)(s & 0xFF)) << (8 * (j & 3));
  }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    ss += __shfl_xor(ss, m, 8);
    raw += __shfl_xor(raw, m, 8);
  }
  int64_t off;
  if constexpr (kWide) {   // 32-row subtiles for 32x32x32: [kstep 4][lane 64][16 B]
    off = (row >> 5) * 4096 + (c >> 1) * 1024 + ((row & 31) + 32 * (c & 1)) * 16;
  } else {                 // 16-row subtiles for 16x16x64: [kstep 2][lane 64][16 B]
    off = (row >> 4) * kSub + (c >> 2) * 1024 + ((row & 15) + 16 * (c & 3)) * 16;
  }
  *reinterpret_cast<uint4*>(pack + off) = make_uint4(o[0], o[1], o[2], o[3]);
  if (c == 0) {
    if (padnorm) {
      // DB rows: w = -||d'||^2 (padding: -2^30) as c = w >> 1 and p = w & 1 (npad apart)
      const int w = (row < n) ? -ss : -padnorm;
      norms[row] = w >> 1;
      norms[npad + row] = w & 1;
    } else {
      norms[row] = ss;   // queries: +||q'||^2 (padding: 0)
    }
    // raw ||v||^2 (as float bits, like match.hip) for sod_match_exact_order
    if (row < n) atomicMax(&flags[max_slot], __float_as_uint((float)raw));
  }
  if (bad) atomicAdd(&flags[0], 1u);
}

__device__ __forceinline__ void glds16(const void* g, uint8_t* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_base, 16, 0, 0);
}

// norms of the stage's 128 rows, wave w of NWx covering rows R*w .. R*w+R-1 (R = 128/NWx):
// lanes 0..R/4-1 fetch c, the next R/4 lanes parity -> one run [c: R x i32 | p: R x i32]
// per wave (global_load_lds writes lane i at M0 + 16 i)
template <int NWx, int kRows>
__device__ __forceinline__ void issue_norms(const int* __restrict__ dn, int64_t npad, int64_t row0,
                                            uint8_t* slot_norm, int wave, int lane) {
  constexpr int R = kRows / NWx, L = R / 4;
  static_assert(2 * L <= 64 && R % 4 == 0, "one glds per wave covers its norm rows");
  const int* src = dn + (lane < L ? 0 : npad) + row0 + wave * R + (lane % L) * 4;
  if (lane < 2 * L) glds16(src, slot_norm + wave * (8 * R));
}

#ifndef SOD_I8_XCHUNK
#define SOD_I8_XCHUNK 1    // thresholds shared between the DB chunks of a query (global max)
#endif
// buffer descriptor word 3 for CDNA (raw, untyped, 32-bit format field as the loads ignore it)
constexpr int kRsrcWord3 = 0x00020000;

// one 1 KiB piece of a stage: lane i's 16 B land at slot + 16 i (M0 = the LDS piece base)
__device__ __forceinline__ void issue_piece(__amdgpu_buffer_rsrc_t rs, uint8_t* lds_piece,
                                            uint32_t soff, int lane) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_piece, 16, (uint32_t)lane * 16u,
                                           soff, 0, 0);
}

__device__ __forceinline__ void issue_stage(const uint8_t* __restrict__ dbpack,
                                            const int* __restrict__ dn, int64_t npad, int64_t sub0,
                                            uint8_t* slot, uint8_t* norm_slot, int wave, int lane) {
  const uint8_t* src = dbpack + sub0 * kSub;
#pragma unroll
  for (int j = 0; j < kPiecesPerWave; ++j) {
    const int piece = wave * kPiecesPerWave + j;
    glds16(src + piece * 1024 + lane * 16, slot + piece * 1024);
  }
  issue_norms<NW16, kStageRows>(dn, npad, sub0 * kSubRows, norm_slot, wave, lane);
}

// offset (in a norm-ring entry) of a 16-row subtile's c for lane group g = lane >> 4 (its
// 4 rows 16u+4g..); the parity words follow at +kParOff
constexpr int kNormRows = kStageRows / NW16;
constexpr int kParOff = 4 * kNormRows;
__device__ __forceinline__ int norm_off(int u, int g) {
  const int row = 16 * u + 4 * g;
  return (row / kNormRows) * (8 * kNormRows) + (row % kNormRows) * 4;
}

#ifndef SOD_I8_ASMLDS
// 1: the ring's fragment / c reads as ds_read_b128 in inline asm with counted waits of our
// own.  The compiler tracks the LDS-DMA refill as an LDS event of another kind, so it can
// only drain the LDS counter completely before the first use of any read (lgkmcnt(0) at
// every subtile, the reads for the subtiles ahead included): prefetching further ahead
// gained nothing.  LDS returns in order, the refill counts on vmcnt only, so waiting for
// all but the reads issued after a subtile's own is exact.  2: at <= 2 query tiles per wave
// (one image: -4 %; C2 at 4 tiles +3 %, C3 at 8 +0.3 %, round 5)
#define SOD_I8_ASMLDS 2
#endif
// LDS byte address of a pointer into the work-group's LDS
__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
}
// ds_read_b128 at a base address + an immediate offset (a constant after unrolling)
__device__ __forceinline__ i32x4 lds_read16(uint32_t base, int off) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(off));
  return v;
}
// wait until at most n LDS operations are outstanding; a, b, c are then ready (tied, so no
// use of them is scheduled before the wait)
__device__ __forceinline__ void lds_wait3(i32x4& a, i32x4& b, i32x4& c, int n) {
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "i"(n));
}

// median of three (v_med3_i32): with y1 >= y2, med3(y1, y, y2) is the new second best
__device__ __forceinline__ int imed3(int a, int b, int c) {
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ void merge2i(int& y1, int& i1, int& y2, int o1, int oi, int o2) {
  // max on y (= min distance), ties -> lower trainIdx; second = max of the rest
  if (o1 > y1 || (o1 == y1 && oi < i1)) {
    y2 = max(y1, o2);
    y1 = o1;
    i1 = oi;
  } else {
    y2 = max(y2, o1);
  }
}

#ifndef SOD_I8_SLOTS
#define SOD_I8_SLOTS 1     // shared bound from the best rows of the even / odd DB chunks
#endif
// threshold words a wave exchanges per query: t2, plus the two best-row slots below 8 query
// tiles per wave (gthr layout: kThrWords regions of nq_pad words)
template <int QT>
constexpr int gwords() { return SOD_I8_SLOTS && QT <= 4 ? kThrWords : 1; }
#ifndef SOD_I8_SEEDSLOT
#define SOD_I8_SEEDSLOT 1  // the seed's best row goes out with the seed's t2
#endif
#ifndef SOD_I8_SEED
#define SOD_I8_SEED 1      // seed pass over a chunk's first stage instead of the dense phase
#endif
#ifndef SOD_I8_SEEDSUB
#define SOD_I8_SEEDSUB SPS // subtiles of the first stage the seed pass covers
#endif
#ifndef SOD_I8_SEEDSUB_QT2
#define SOD_I8_SEEDSUB_QT2 16   // ... at 2 query tiles per wave (one query image; round 5)
#endif
#ifndef SOD_I8_SEEDPUB
#define SOD_I8_SEEDPUB 1   // publish the seed thresholds to the other chunks right away
#endif
#ifndef SOD_I8_SEEDLOAD
#define SOD_I8_SEEDLOAD 1  // then read the other chunks' seeds before the stage's main pass
#endif
#ifndef SOD_I8_DENSE
#define SOD_I8_DENSE 32    // leading subtiles of a chunk updated without threshold exchange (C2: +8 %)
#endif
constexpr int64_t kDense = SOD_I8_DENSE;
// shared-threshold exchange points (subtiles of a stage, SOD_I8_XCHUNK): the DMA issued at
// kShareLoad[i] is applied at kShareApply[i] (the same stage when it is later, else the next)
#ifndef SOD_I8_PUB_EVERY
#define SOD_I8_PUB_EVERY 1   // 4 measured: 5 % less L2-miss traffic, time unchanged
#endif
#ifndef SOD_I8_XEVERY
// stages between threshold exchanges (load + publish) after a chunk's first 4: every stage's
// load of the wave's 128 global values (served past L2) was ~70 MB of a launch's L2-miss
// traffic; every 4th: 541 -> 469 MB and -0.8 % time at C3, C2 equal (16th: 416 MB, C2 +4 %)
#define SOD_I8_XEVERY 4
#endif
constexpr int64_t kPublishDense = 4, kPublishEvery = SOD_I8_PUB_EVERY;
#ifndef SOD_I8_XDENSE
#define SOD_I8_XDENSE 8    // leading stages that exchange thresholds every stage (4: C2 +1.8 %)
#endif
constexpr int64_t kXDense = SOD_I8_XDENSE, kXEvery = SOD_I8_XEVERY;
#ifndef SOD_I8_SHARE_AT
#define SOD_I8_SHARE_AT 4, 20   // subtile of the threshold load, of its application (8, 24: C3 +0.2 %)
#endif
constexpr int kShareAt[2] = {SOD_I8_SHARE_AT};
__device__ __forceinline__ constexpr bool share_load(int u) { return u == kShareAt[0]; }
__device__ __forceinline__ constexpr bool share_apply(int u) { return u == kShareAt[1]; }

constexpr int kRing = SOD_I8_RING;
constexpr int kLoadsPerStage = kPiecesPerWave + 1;   // vm instructions per wave per stage

// Top-2 VALUES of {a, partner lane's a} for the lane pairs (l, l^32) / (l, l^16):
// v_permlane32_swap / v_permlane16_swap of a register with itself leaves {x_l, x_partner}
// in the two results (in some order), so max / min of the pair need no lane select.
__device__ __forceinline__ void top2_xor32(int& y1, int& y2) {
  const auto p = __builtin_amdgcn_permlane32_swap((unsigned)y1, (unsigned)y1, false, false);
  const auto q = __builtin_amdgcn_permlane32_swap((unsigned)y2, (unsigned)y2, false, false);
  const int a = (int)p[0], b = (int)p[1];
  y1 = max(a, b);
  y2 = max(max(min(a, b), (int)q[0]), (int)q[1]);
}
__device__ __forceinline__ void top2_xor16(int& y1, int& y2) {
  const auto p = __builtin_amdgcn_permlane16_swap((unsigned)y1, (unsigned)y1, false, false);
  const auto q = __builtin_amdgcn_permlane16_swap((unsigned)y2, (unsigned)y2, false, false);
  const int a = (int)p[0], b = (int)p[1];
  y1 = max(a, b);
  y2 = max(max(min(a, b), (int)q[0]), (int)q[1]);
}
// max of a over the lane quadruple (l, l^16, l^32, l^48): one query's four lane groups
__device__ __forceinline__ int max_xor3216(int a) {
  auto p = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)a, false, false);
  a = max((int)p[0], (int)p[1]);
  p = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)a, false, false);
  return max((int)p[0], (int)p[1]);
}

#define PARITY_T const uint8_t*   // LDS address of the lane's 4 parity words

// max of N values as a v_max3 tree (ceil((N-1)/2) VALU), fully unrolled
template <int N>
struct MaxTree {
  static __device__ __forceinline__ int f(const int* v) {
    if constexpr (N == 1) {
      return v[0];
    } else if constexpr (N == 2) {
      return max(v[0], v[1]);
    } else {
      constexpr int M = N / 3 + (N % 3 != 0);
      int w[M];
#pragma unroll
      for (int i = 0; i < N / 3; ++i) w[i] = max(max(v[3 * i], v[3 * i + 1]), v[3 * i + 2]);
      if constexpr (N % 3 == 2) w[M - 1] = max(v[N - 2], v[N - 1]);
      if constexpr (N % 3 == 1) w[M - 1] = v[N - 1];
      return MaxTree<M>::f(w);
    }
  }
};


// prefilter + exact top-2 update of one 16x16 tile set (see the file comment).  Each lane
// keeps the exact top-2 (with index) of ITS rows; the prefilter threshold is the query's
// second-best value over all four lane groups (lanes l, l^16, l^32, l^48), which every
// row of the final top-2 reaches (>=, so ties keep their lowest-index winner).
// mode (wave-uniform): 0 = prefilter; 1 = dense (the chunk's first subtiles, where
// t2 is still -inf and every tile takes the exact update: the threshold exchange is
// skipped); 2 = the last dense subtile (the exchange then sets every tile's t2).
template <int QT, bool kAsm>
__device__ __forceinline__ void tile_update(const i32x4 (&acc)[QT], PARITY_T pin, int rowb,
                                            int (&y1)[QT], int (&y2)[QT], int (&t2)[QT],
                                            int (&id)[QT], int mode = 0, bool vmem = false) {
  uint64_t hit[QT];
  uint64_t any = 0;
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int m = max(max(acc[t][0], acc[t][1]), max(acc[t][2], acc[t][3]));
    hit[t] = __builtin_amdgcn_ballot_w64(m >= t2[t]);
    any |= hit[t];
  }
  // interleave this block (the subtile's 16 MFMAs, next-subtile LDS reads, the previous
  // subtile's prefilter) as MFMA, 2 VALU, MFMA, 2 VALU, ...
#pragma unroll
  for (int i = 0; i < 2 * QT; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);                            // MFMA
    if (i < 3 * QT / 2) __builtin_amdgcn_sched_group_barrier(0x2, 2, 0);       // VALU
    if (!kAsm && i >= 1 && i <= 4)
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                        // DS read
    if (vmem && i == 6) __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);      // refill piece
  }
  if (__builtin_expect(any != 0, 0)) {   // slow path laid out away from the hot loop
    i32x4 p;
    if constexpr (kAsm) {
      // (an LDS read the compiler tracked here would make it drain the counter before every
      // later fragment read that reuses its registers)
      p = lds_read16(lds_addr(pin), 0);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(p));
    } else {
      p = *reinterpret_cast<const i32x4*>(pin);
    }
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      if (hit[t]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int y = 2 * acc[t][r] | p[r];
          const bool gt = y > y1[t];
          y2[t] = imed3(y1[t], y, y2[t]);
          id[t] = gt ? rowb + r : id[t];
          y1[t] = gt ? y : y1[t];
        }
        if (mode == 0) {
          int g1 = y1[t], g2 = y2[t];
          top2_xor32(g1, g2);
          top2_xor16(g1, g2);
          t2[t] = max(t2[t], g2 >> 1);   // never below a shared bound already applied
        }
      }
    }
    if (mode == 2) {
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        int g1 = y1[t], g2 = y2[t];
        top2_xor32(g1, g2);
        top2_xor16(g1, g2);
        t2[t] = max(t2[t], g2 >> 1);
      }
    }
  }
}

// One work unit: query block qb (NW16*QT tiles) against DB chunk sp (sub_per_split subtiles),
// writing the chunk's partial top-2 of every query to slot sp of pd1/pidx/pd2.
// PF = subtiles whose A fragments / norm words are read from LDS ahead of their MFMAs: 1
// hides the LDS latency behind one subtile's MFMAs, which at 2-4 query tiles per wave (8-16
// MFMAs per wave and subtile) is too short.
// PAIR = waves per query slice: with 2, waves w and w + NW16/2 (the same SIMD) hold the same
// queries and take the even / odd subtiles of every stage, so each 2 KiB subtile is read
// from LDS by half the waves for twice the MFMAs (small query sets, where the 8 waves'
// fragment reads keep the LDS array busy most of the MFMA time); their two partial top-2
// lists merge through LDS at the end.
template <int QT, int PF, int PAIR>
__device__ __forceinline__ void match_unit(
    uint8_t* lds, int sp, int qb, const uint8_t* __restrict__ dbpack, const int* __restrict__ dn,
    int64_t nsub, const uint8_t* __restrict__ qpack, const int* __restrict__ qn, int nqt,
    int64_t nq_pad, int64_t sub_per_split, int row_offset, float* __restrict__ pd1,
    int* __restrict__ pidx, float* __restrict__ pd2, int* __restrict__ gthr, int seedload) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NQW = NW16 / PAIR;                  // query slices per work-group
  constexpr int SUBS = SPS / PAIR;                  // subtiles per stage and wave
  static_assert(PAIR == 1 || (PAIR == 2 && kNormRows % 32 == 0 && kShareAt[0] % 2 == 0 &&
                              kShareAt[1] % 2 == 0 && kPiecesPerWave <= SUBS),
                "paired waves: odd subtiles sit 64 B after the even ones in the norm ring");
  const int qwave = wave % NQW, par = wave / NQW;   // query slice, subtile phase
  constexpr bool kAsm = SOD_I8_ASMLDS == 1 || (SOD_I8_ASMLDS == 2 && QT <= 2);
  const int qt0 = (qb * NQW + qwave) * QT;
  const int64_t s_lo = (int64_t)sp * sub_per_split;
  const int64_t s_hi = min(nsub, s_lo + sub_per_split);
  const int64_t nst = (s_hi - s_lo) / SPS;
  const int64_t npad = nsub * kSubRows;

  uint8_t* const nring = lds + kRing * kStageBytes;
#pragma unroll
  for (int j = 0; j < kRing - 1; ++j)
    if (j < nst)
      issue_stage(dbpack, dn, npad, s_lo + j * SPS, lds + j * kStageBytes, nring + j * kStageNorm,
                  wave, lane);
  static_assert(kRing == 2, "spread refill: the slot refilled during stage s is stage s-1's");
  // the chunk's descriptors as one buffer (< 2 GiB: launch_match_i8 sizes the chunks)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dbpack + s_lo * kSub), (short)0, (int)((s_hi - s_lo) * kSub), kRsrcWord3);

  i32x4 bq[QT][2];
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int qt = qt0 + t;
      bq[t][k] = qt < nqt ? *reinterpret_cast<const i32x4*>(qpack + ((int64_t)qt * 2 + k) * 1024 + lane * 16)
                          : i32x4{0, 0, 0, 0};
    }
  int y1[QT], y2[QT], t2[QT], id[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    y1[t] = INT_MIN;
    y2[t] = INT_MIN;
    t2[t] = INT_MIN >> 1;
    id[t] = 0x7fffffff;
  }
  const int rowl = row_offset + (int)(s_lo * kSubRows) + (lane >> 4) * 4 + par * kSubRows;
#if SOD_I8_XCHUNK
  // Chunks of the same queries share their prefilter thresholds: gthr[q] = max over chunks of
  // the t2 (= query-wide second best >> 1) they published.  A chunk holding t2 has two rows
  // with y >= 2 t2, so a row below it can never be in the query's global top-2 (ties pass the
  // >= test): any chunk may skip it.  At each stage boundary a wave publishes its tiles' t2
  // (buffer atomic max, lanes of one lane group, only where above the last value read) and
  // DMAs the current global values of its 128 queries into LDS, which the next boundary
  // applies -- a value one stage old, or stale across XCDs, is still a valid bound, so
  // nothing waits for it.  The chunk's own top-2 stays exact over the rows it keeps.
  // SOD_I8_SLOTS: every chunk also publishes its query-wide best h (the value of one of its
  // rows) into word 1 + (chunk & 1) by atomic max.  The two words then hold rows of two
  // different chunks, so min(even best, odd best) has two distinct rows at or above it and
  // is a valid bound too -- close to the second best over ALL rows the chunks have seen so
  // far, where the max of the chunks' own second bests lags far behind with many chunks.
  // Layout: gthr[r * nq_pad + q], r = 0: t2, 1: even best, 2: odd best (h units).  The
  // kernel at 8 query tiles per wave (C3) leaves the slots out: no time gained there, three
  // times the exchange loads (gwords<QT>).
  constexpr int GW = gwords<QT / PAIR>();
  constexpr bool kSlots = GW > 1;
  const int wq = __builtin_amdgcn_readfirstlane(wave);
  const int qwq = wq % NQW;
  const int ntile = max(0, min(QT, nqt - (qb * NQW + qwq) * QT));   // real tiles of the wave
  const int64_t qw0 = (int64_t)(qb * NQW + qwq) * QT * 16;   // the wave's first query
  int* const gw = gthr + qw0;
  // one descriptor over the three words of the slot (a padding tile's load reads the next
  // queries' words or, past the end, 0; its bound is never used)
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)gthr, (short)0, (int)(kThrWords * nq_pad * 4), kRsrcWord3);
  uint8_t* const gl =
      lds + kRing * kStageBytes + kNormRing * kStageNorm + wq * (QT * 64 * GW);
  [[maybe_unused]] const int oslot = 1 + (sp & 1);   // this chunk's best-row word
#endif
  // accumulators, norms and first row of the subtile whose prefilter is pending; the
  // initial "previous subtile" is empty (h = INT_MIN can never pass t2)
  i32x4 accp[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) accp[t] = i32x4{INT_MIN, INT_MIN, INT_MIN, INT_MIN};
  const uint8_t* pp = nring;   // never read before it is set (accp cannot pass t2)
  int rowp = 0;

  int slot = 0;
  for (int64_t s = 0; s < nst; ++s) {
    // the wave's loads of stage s are complete when at most the later prefetched stages'
    // loads remain in flight (vector memory returns in order)
    const int64_t younger = min<int64_t>(kRing - 2, nst - 1 - s);   // stages issued after s
    if (kRing >= 4 && younger >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kLoadsPerStage) : "memory");
    else if (kRing >= 3 && younger >= 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLoadsPerStage) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // every wave has finished stage s-1, so its slot takes stage s+kRing-1
    // (descriptor pieces spread over this stage's first subtiles below; norms now)
    if (s + 1 < nst)
      issue_norms<NW16, kStageRows>(dn, npad, (s_lo + (s + 1) * SPS) * kSubRows,
                                    nring + ((s + 1) % kNormRing) * kStageNorm, wave, lane);
    // the last stage re-reads itself into the free slot (never read again): the pieces stay
    // unconditional, so no branch splits the subtile blocks
    const int wv = __builtin_amdgcn_readfirstlane(wave);   // wave-uniform: SGPR offsets
    uint8_t* const refill = lds + (slot == 0 ? 1 : 0) * kStageBytes + wv * kPiecesPerWave * 1024;
    const uint32_t refill_off =
        (uint32_t)(min<int64_t>(s + 1, nst - 1) * kStageBytes + wv * kPiecesPerWave * 1024);
    // (the wave's subtile phase folded in: subtile u of the wave is u * PAIR + par)
    const uint8_t* sb = lds + slot * kStageBytes + par * kSub;
    const uint8_t* nb0 =
        nring + (s % kNormRing) * kStageNorm + norm_off(0, lane >> 4) + par * (kSubRows * 4);
#if SOD_I8_SEED
    if (s == 0) {
      // Seed pass: the chunk's first stage through the MFMAs once with no top-2 work, only a
      // running max of each lane's values per tile (the lane's 4 rows per subtile, one query).
      // The second largest of a query's 4 lane-group maxima comes from two distinct rows of
      // this chunk, so the query's final second best is >= it: a valid prefilter threshold
      // (and a valid shared bound) from the first subtile on.  The stage is then processed
      // normally, its rows below the seed skipped, instead of every tile of its 32 subtiles
      // taking the exact update (the dense phase).
      int sm[QT];
      [[maybe_unused]] int sb1[QT];
#pragma unroll
      for (int t = 0; t < QT; ++t) sm[t] = INT_MIN;
#pragma unroll 1
      for (int u = 0; u < (QT / PAIR <= 2 ? SOD_I8_SEEDSUB_QT2 : SOD_I8_SEEDSUB); u += PAIR) {
        const uint8_t* nb = sb + u * kSub + lane * 16;
        const i32x4 a0 = *reinterpret_cast<const i32x4*>(nb);
        const i32x4 a1 = *reinterpret_cast<const i32x4*>(nb + 1024);
        const i32x4 c = *reinterpret_cast<const i32x4*>(nb0 + norm_off(u, 0));
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          i32x4 acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq[t][0], c, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq[t][1], acc, 0, 0, 0);
          sm[t] = max(sm[t], max(max(acc[0], acc[1]), max(acc[2], acc[3])));
        }
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        int g1 = sm[t], g2 = INT_MIN;
        top2_xor32(g1, g2);
        top2_xor16(g1, g2);
        t2[t] = max(t2[t], g2);
#if SOD_I8_XCHUNK && SOD_I8_SEEDPUB
        // out to the chunks of the same queries now: their first threshold load (this
        // stage's share_load) then already sees the other chunks' seeds
        if (lane < 16 && t < ntile) {
          __hip_atomic_fetch_max(gw + 16 * t + lane, t2[t], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
          if constexpr (kSlots && SOD_I8_SEEDSLOT)
            __hip_atomic_fetch_max(gw + oslot * nq_pad + 16 * t + lane, g1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
#endif
        sb1[t] = g1;   // the chunk's best so far (h), for the seed load below (kSlots)
      }
#if SOD_I8_XCHUNK && SOD_I8_SEEDPUB && SOD_I8_SEEDLOAD
      // the chunks of a query block run their seed passes side by side: one round trip
      // now gives the stage's main pass the max of the seeds published so far.  The wait
      // also covers the next stage's prefetch (loads return in order), which costs more
      // than it saves when the DB stream dominates (many chunks of few queries: 500 x 1M,
      // 124 chunks, 0.078 vs 0.070 ms), so the launch enables it up to 64 chunks only, and
      // the one-image kernel (QT 2) does not carry the code (its mere presence cost 2-3 %)
      if (QT / PAIR >= 4 && seedload) {
        int gq[QT][kThrWords];
#pragma unroll
        for (int t = 0; t < QT; ++t)   // one load per query (lanes 0-15), then to its groups
#pragma unroll
          for (int r = 0; r < GW; ++r)
            gq[t][r] = lane < 16 && t < ntile
                           ? __hip_atomic_load(gw + r * nq_pad + 16 * t + lane,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : INT_MIN;
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          if constexpr (kSlots) {
            const bool odd = oslot == 2;   // selects, not an indexed register array
            const int own = max(odd ? gq[t][2] : gq[t][1], sb1[t]), other = odd ? gq[t][1] : gq[t][2];
            gq[t][0] = max(gq[t][0], min(own, other));
          }
          t2[t] = max(t2[t], __shfl(gq[t][0], lane & 15));
        }
      }
#endif
    }
#endif
    slot = slot + 1 == kRing ? 0 : slot + 1;
    i32x4 fa0[PF], fa1[PF], fc[PF];
    [[maybe_unused]] const uint32_t sbl = lds_addr(sb) + lane * 16, nbl = lds_addr(nb0);
    if constexpr (kAsm) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        fa0[j] = lds_read16(sbl, j * PAIR * kSub);
        fa1[j] = lds_read16(sbl, j * PAIR * kSub + 1024);
        fc[j] = lds_read16(nbl, norm_off(j * PAIR, 0));
      }
    } else {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      fa0[j] = *reinterpret_cast<const i32x4*>(sb + j * PAIR * kSub + lane * 16);
      fa1[j] = *reinterpret_cast<const i32x4*>(sb + j * PAIR * kSub + 1024 + lane * 16);
      fc[j] = *reinterpret_cast<const i32x4*>(nb0 + norm_off(j * PAIR, 0));
    }
    }
#pragma clang loop unroll(full)
    for (int ju = 0; ju < SUBS; ++ju) {
      const int u = ju * PAIR;   // the wave's subtile (plus par, folded into sb / nb0 / rowl)
      const int js = ju % PF;    // a constant after unrolling
      // (asm reads) this subtile's three reads done; the subtiles' ahead may be in flight
      if constexpr (kAsm) lds_wait3(fa0[js], fa1[js], fc[js], 3 * min(PF - 1, SUBS - 1 - ju));
      const i32x4 a0 = fa0[js], a1 = fa1[js], c = fc[js];   // c = floor(-||d'||^2 / 2)
      const uint8_t* p = nb0 + norm_off(u, 0) + kParOff;   // norm_off(u, g) = norm_off(u, 0) + 16 g
      i32x4 acc[QT];
#pragma unroll
      for (int t = 0; t < QT; ++t)
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq[t][0], c, 0, 0, 0);
      // piece u of the next stage (wave-uniform branch; u is a constant after unrolling)
      const bool piece_here = ju < kPiecesPerWave;
      if (piece_here)
        issue_piece(rs, refill + ju * 1024, refill_off + ju * 1024, lane);
      if (kAsm && ju + PF < SUBS) {   // the fragments PF subtiles ahead in flight
        fa0[js] = lds_read16(sbl, (u + PF * PAIR) * kSub);
        fa1[js] = lds_read16(sbl, (u + PF * PAIR) * kSub + 1024);
        fc[js] = lds_read16(nbl, norm_off(u + PF * PAIR, 0));
      }
      if (!kAsm && ju + PF < SUBS) {
        const uint8_t* nb = sb + (u + PF * PAIR) * kSub + lane * 16;
        fa0[js] = *reinterpret_cast<const i32x4*>(nb);
        fa1[js] = *reinterpret_cast<const i32x4*>(nb + 1024);
        fc[js] = *reinterpret_cast<const i32x4*>(nb0 + norm_off(u + PF * PAIR, 0));
      }
#pragma unroll
      for (int t = 0; t < QT; ++t)
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq[t][1], acc[t], 0, 0, 0);
      const int rowb = rowl + (int)((s * SPS + u) * kSubRows);
      {
        // the pending subtile's index in the chunk decides dense / final / prefilter
        const int64_t kp = s * SPS + u - PAIR;
        const int mode = SOD_I8_SEED ? 0 : (kp < kDense - 1 ? 1 : (kp == kDense - 1 ? 2 : 0));
        tile_update<QT, kAsm>(accp, pp, rowp, y1, y2, t2, id, mode, piece_here);
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) accp[t] = acc[t];
      pp = p;
      rowp = rowb;
#if SOD_I8_XCHUNK
      // shared thresholds, twice per stage: at subtile kShareLoad the wave DMAs the global
      // values of its queries into LDS; at kShareApply (they landed: vmcnt(0), the stage's
      // refill pieces went out before the load) it publishes its own t2 where above them and
      // raises t2 to them
      const bool xstage = kXEvery == 1 || s < kXDense || s % kXEvery == 0;   // wave-uniform
      // the wave's QT x 16 values of each word: QT*4 lanes x 16 B per word
      if (share_load(u) && xstage && lane < QT * 4) {
#pragma unroll
        for (int r = 0; r < GW; ++r)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rg, (lds_void*)(gl + r * QT * 64), 16,
              (uint32_t)((qw0 + r * nq_pad) * 4) + (uint32_t)lane * 16u, 0, 0,
              16 /* sc1: past this XCD's L2 */);
      }
      if (share_apply(u) && xstage) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int* gv = reinterpret_cast<const int*>(gl) + (lane & 15);
        // publishing is a device-scope atomic per query (a memory-side transaction each):
        // every stage while the thresholds still move fast, then every kPublishEvery-th
        const bool publish = s < kPublishDense || s % kPublishEvery == 0;
        int gq[QT];
        [[maybe_unused]] int go[QT], gx[QT];
#pragma unroll
        for (int t = 0; t < QT; ++t) {   // all reads, then one wait
          gq[t] = gv[16 * t];
          if constexpr (kSlots) {
            go[t] = gv[oslot * QT * 16 + 16 * t];
            gx[t] = gv[(3 - oslot) * QT * 16 + 16 * t];
          }
        }
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          if constexpr (kSlots) {
            // the query-wide best of this wave's rows (y units -> h)
            const int hb = max_xor3216(y1[t]) >> 1;
            if (publish && lane < 16 && t < ntile && hb > go[t])
              __hip_atomic_fetch_max(gw + oslot * nq_pad + 16 * t + lane, hb, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            // t2 goes out only where it beats what every chunk derives from the words itself
            // (a t2 raised by the slot bound would otherwise be re-published by all chunks at
            // every exchange: same-address atomics that the vmcnt(0) above then waits for)
            gq[t] = max(gq[t], min(max(go[t], hb), gx[t]));
          }
          if (publish && lane < 16 && t < ntile && t2[t] > gq[t])
            __hip_atomic_fetch_max(gw + 16 * t + lane, t2[t], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          t2[t] = max(t2[t], gq[t]);
        }
      }
#endif
    }
  }
  // LDS-DMA still in flight (the last stage's refill pieces re-read that stage, a shared-
  // threshold load) must land before the work-group's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tile_update<QT, kAsm>(accp, pp, rowp, y1, y2, t2, id,
                        !SOD_I8_SEED && nst * SPS <= kDense ? 1 : 0);

  if constexpr (PAIR == 2) {
    // the odd-phase wave hands its lanes' top-2 to the even-phase wave of the same queries
    // (the ring is free: every wave's DMA landed before the barrier, no wave reads it again)
    __builtin_amdgcn_s_barrier();
    int* const xl = reinterpret_cast<int*>(lds) + (qwave * QT) * 3 * 64 + lane;
    if (par == 1) {
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        xl[(3 * t) * 64] = y1[t];
        xl[(3 * t + 1) * 64] = id[t];
        xl[(3 * t + 2) * 64] = y2[t];
      }
    }
    __builtin_amdgcn_s_barrier();
    if (par == 1) return;
#pragma unroll
    for (int t = 0; t < QT; ++t)
      merge2i(y1[t], id[t], y2[t], xl[(3 * t) * 64], xl[(3 * t + 1) * 64], xl[(3 * t + 2) * 64]);
  }
#pragma unroll
  for (int t = 0; t < QT; ++t) {
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      const int o1 = __shfl_xor(y1[t], m), oi = __shfl_xor(id[t], m), o2 = __shfl_xor(y2[t], m);
      merge2i(y1[t], id[t], y2[t], o1, oi, o2);
    }
    const int qt = qt0 + t;
    if (lane < 16 && qt < nqt) {
      const int64_t q = (int64_t)qt * 16 + lane;
      const int n2 = qn[q];
      const int64_t o = (int64_t)sp * nq_pad + q;
      // padding rows only win when the shard has fewer than two real rows: keep them huge
      pd1[o] = y1[t] < -(1 << 29) ? 3.0e38f : (float)(n2 - y1[t]);
      pidx[o] = id[t];
      pd2[o] = y2[t] < -(1 << 29) ? 3.0e38f : (float)(n2 - y2[t]);
    }
  }
}


template <int QT, int PF, int PAIR>
#ifndef SOD_I8_MINB
#define SOD_I8_MINB 1      // work-groups per CU the register allocation must allow
#endif
#ifndef SOD_I8_QT2_WGS
#define SOD_I8_QT2_WGS 1   // work-groups per CU at 2 query tiles per wave (LDS permitting)
#endif
__global__ __launch_bounds__(NT16, SOD_I8_MINB) void match_i8_kernel(
    const uint8_t* __restrict__ dbpack, const int* __restrict__ dn, int64_t nsub,
    const uint8_t* __restrict__ qpack, const int* __restrict__ qn, int nqt, int64_t nq_pad,
    int split, int64_t sub_per_split, int row_offset, float* __restrict__ pd1,
    int* __restrict__ pidx, float* __restrict__ pd2, int nqb, int* __restrict__ gthr,
    int seedload) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRing * kStageBytes + kNormRing * kStageNorm +
                                                     SOD_I8_XCHUNK * NW16 * QT * 64 * gwords<QT / PAIR>()];
  // XCD-aware order: blocks b, b+8, ... share an XCD (and its L2); give each such group a
  // contiguous run of chunk-major units, so an XCD streams one or two DB chunks, in step,
  // instead of all of them (bijective for any grid size; cdna_hip_programming.md T1)
  const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = blockIdx.x % 8;
  const unsigned u = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + blockIdx.x / 8;
  match_unit<QT, PF, PAIR>(lds, (int)(u / nqb), (int)(u % nqb), dbpack, dn, nsub, qpack, qn, nqt, nq_pad,
             sub_per_split, row_offset, pd1, pidx, pd2, gthr, seedload);
}

// ---------------------------------------------------------------------------------------
// 32x32x32 variant (impl 2): lane l owns query l&31 and 16 rows (reg r -> row (r&3) +
// 8(r>>2) + 4(l>>5)) of each 32-row subtile.  An MFMA of this shape holds the SIMD's issue
// port for 8 of its 32 cycles (vs 8 of 16 for 16x16x64), and the prefilter reduces 16
// values per lane and tile (9 VALU per 1024 pairs instead of 12), so the instruction stream
// leaves room beside the matrix pipe.  Tile-major order: the 4 MFMAs (K = 4 x 32) of tile t
// are issued back to back (one accumulation chain) and tile t-1's prefilter runs beside
// them, so only two tile accumulators are alive (the last tile of a subtile is tested
// beside the next subtile's first tile).  DB stages of 512 rows in a 2-slot ring, norm words
// in a ring of their own (parity read on the slow path), as match_i8_kernel.
#ifndef SOD_I8W_NW
#define SOD_I8W_NW 8
#endif
namespace w {
constexpr int NW = SOD_I8W_NW;   // waves per work-group (8: one work-group per CU)
constexpr int NT = NW * 64;
constexpr int QT = 4;            // 32-query tiles per wave (128 queries)
constexpr int SPS = 16;          // 32-row subtiles per stage (512 rows)
constexpr int kSub = 4096;
constexpr int kStageBytes = SPS * kSub;          // 64 KiB
constexpr int kStageNorm = 2 * SPS * 32 * 4;     // c and p of 512 rows: 4 KiB
constexpr int kPiecesPerWave = kStageBytes / 1024 / NW;
constexpr int kRing = 2;
constexpr int kNormRows = SPS * 32 / NW;          // norm rows staged per wave
// offset (in a norm-ring entry) of c for the 4 consecutive rows starting at stage row r;
// parity at + 4 * kNormRows
__device__ __forceinline__ int norm_off(int r) {
  return (r / kNormRows) * (8 * kNormRows) + (r % kNormRows) * 4;
}
}  // namespace w

typedef __attribute__((ext_vector_type(16))) int i32x16;

__device__ __forceinline__ void issue_stage_w(const uint8_t* __restrict__ dbpack,
                                              const int* __restrict__ dn, int64_t npad, int64_t sub0,
                                              uint8_t* slot, uint8_t* norm_slot, int wave, int lane) {
  const uint8_t* src = dbpack + sub0 * w::kSub;
#pragma unroll
  for (int j = 0; j < w::kPiecesPerWave; ++j) {
    const int piece = wave * w::kPiecesPerWave + j;
    glds16(src + piece * 1024 + lane * 16, slot + piece * 1024);
  }
  issue_norms<w::NW, w::SPS * 32>(dn, npad, sub0 * 32, norm_slot, wave, lane);
}

// prefilter + exact update of ONE 32x32 tile: max of the lane's 16 values against the
// query's threshold, and on a hit the exact top-2 of the lane's rows (parity words from the
// norm ring) and the query-wide threshold over the two lane halves
// rowb is wave-uniform (the lane half's 4 h is added at the end), so the slow path's row
// numbers are scalar adds, not VALU
__device__ __forceinline__ void tile_update_w(const i32x16& acc, const uint8_t* pbase, int rowb,
                                              int& y1, int& y2, int& t2, int& id) {
  // two max3 chains of 7 values and one combine: 8 VALU, dependence depth 4
  const int ma = max(max(max(max(max(max(acc[0], acc[1]), acc[2]), acc[3]), acc[4]), acc[5]), acc[6]);
  const int mb = max(max(max(max(max(max(acc[7], acc[8]), acc[9]), acc[10]), acc[11]), acc[12]), acc[13]);
  const int m = max(max(ma, mb), max(acc[14], acc[15]));
  // interleave: MFMA, MFMA, 4 VALU, MFMA, 5 VALU, MFMA (the previous tile's MFMA result
  // is read two MFMAs after its last MFMA)
  __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
  __builtin_amdgcn_sched_group_barrier(0x2, 4, 0);
  __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x2, 5, 0);
  __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(m >= t2) != 0, 0)) {
    // scalar row base materialised inside the slow path (readfirstlane is convergent, so
    // the 16 row numbers are not hoisted into the hot block as vector adds)
    const int rs = __builtin_amdgcn_readfirstlane(rowb);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const i32x4 pv = *reinterpret_cast<const i32x4*>(pbase + w::norm_off(8 * g) + 4 * w::kNormRows);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int y = 2 * acc[4 * g + i] | pv[i];
        const bool gt = y > y1;
        y2 = imed3(y1, y, y2);
        id = gt ? rs + 8 * g + i : id;
        y1 = gt ? y : y1;
      }
    }
    int g1 = y1, g2 = y2;
    top2_xor32(g1, g2);
    t2 = g2 >> 1;
  }
}

template <int QT>   // 32-query tiles per wave (w::QT by default; option match_qt 1 / 2 / 4)
__global__ __launch_bounds__(w::NT) void match_i8w_kernel(
    const uint8_t* __restrict__ dbpack, const int* __restrict__ dn, int64_t nsub,
    const uint8_t* __restrict__ qpack, const int* __restrict__ qn, int nqt, int64_t nq_pad,
    int split, int64_t sub_per_split, int row_offset, float* __restrict__ pd1,
    int* __restrict__ pidx, float* __restrict__ pd2, int nqb) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[w::kRing * w::kStageBytes + kNormRing * w::kStageNorm];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware chunk-major order, as match_i8_kernel
  const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x8 = blockIdx.x % 8;
  const unsigned unit = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + blockIdx.x / 8;
  const int sp = (int)(unit / nqb);
  const int qb = (int)(unit % nqb);
  const int qt0 = (qb * w::NW + wave) * QT;
  const int64_t s_lo = (int64_t)sp * sub_per_split;
  const int64_t s_hi = min(nsub, s_lo + sub_per_split);
  const int64_t nst = (s_hi - s_lo) / w::SPS;
  const int h = lane >> 5;
  const int64_t npad = nsub * 32;
  uint8_t* const nring = lds + w::kRing * w::kStageBytes;

#pragma unroll
  for (int j = 0; j < w::kRing - 1; ++j)
    if (j < nst)
      issue_stage_w(dbpack, dn, npad, s_lo + j * w::SPS, lds + j * w::kStageBytes,
                    nring + j * w::kStageNorm, wave, lane);

  i32x4 bq[QT][4];
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int qt = qt0 + t;
      bq[t][k] = qt < nqt ? *reinterpret_cast<const i32x4*>(qpack + ((int64_t)qt * 4 + k) * 1024 + lane * 16)
                          : i32x4{0, 0, 0, 0};
    }
  int y1[QT], y2[QT], t2[QT], id[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    y1[t] = INT_MIN;
    y2[t] = INT_MIN;
    t2[t] = INT_MIN >> 1;
    id[t] = 0x7fffffff;
  }
  const int rowl = row_offset + (int)(s_lo * 32);   // + 4 h per lane half, added at the end
  // the last tile of the previous subtile, tested beside the next subtile's first tile
  i32x16 accp;
#pragma unroll
  for (int r = 0; r < 16; ++r) accp[r] = INT_MIN;
  const uint8_t* pp = nring;
  int rowp = 0;

  int slot = 0;
  for (int64_t s = 0; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this stage landed (2-slot ring)
    __builtin_amdgcn_s_barrier();
    if (s + w::kRing - 1 < nst) {
      const int ns = slot == 0 ? w::kRing - 1 : slot - 1;
      issue_stage_w(dbpack, dn, npad, s_lo + (s + w::kRing - 1) * w::SPS, lds + ns * w::kStageBytes,
                    nring + ((s + w::kRing - 1) % kNormRing) * w::kStageNorm, wave, lane);
    }
    const uint8_t* sb = lds + slot * w::kStageBytes;
    const uint8_t* nb = nring + (s % kNormRing) * w::kStageNorm + w::norm_off(4 * h);
    slot = slot + 1 == w::kRing ? 0 : slot + 1;
    i32x4 fa[4], fc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      fa[k] = *reinterpret_cast<const i32x4*>(sb + k * 1024 + lane * 16);
      fc[k] = *reinterpret_cast<const i32x4*>(nb + w::norm_off(8 * k));
    }
#pragma clang loop unroll(full)
    for (int u = 0; u < w::SPS; ++u) {
      i32x4 a[4];
      i32x16 c;   // c = floor(-||d'||^2 / 2) of the lane's 16 rows 8g + 4h + i
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = fa[k];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[4 * k + i] = fc[k][i];
      }
      const uint8_t* pu = nb + w::norm_off(32 * u);   // this subtile's norm words (lane half h)
      const int rowb = rowl + (int)((s * w::SPS + u) * 32);
      i32x16 accq;   // the previous tile of this subtile
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], bq[t][0], c, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[1], bq[t][1], acc, 0, 0, 0);
        if (t == 0 && u + 1 < w::SPS) {   // next subtile's fragments in flight
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            fa[k] = *reinterpret_cast<const i32x4*>(sb + (u + 1) * w::kSub + k * 1024 + lane * 16);
            fc[k] = *reinterpret_cast<const i32x4*>(nb + w::norm_off(32 * (u + 1) + 8 * k));
          }
        }
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[2], bq[t][2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[3], bq[t][3], acc, 0, 0, 0);
        if (t == 0)
          tile_update_w(accp, pp, rowp, y1[QT - 1], y2[QT - 1], t2[QT - 1], id[QT - 1]);
        else
          tile_update_w(accq, pu, rowb, y1[t - 1], y2[t - 1], t2[t - 1], id[t - 1]);
        accq = acc;
      }
      accp = accq;
      pp = pu;
      rowp = rowb;
    }
  }
  tile_update_w(accp, pp, rowp, y1[QT - 1], y2[QT - 1], t2[QT - 1], id[QT - 1]);

#pragma unroll
  for (int t = 0; t < QT; ++t) {
    if (y1[t] != INT_MIN) id[t] += 4 * h;   // the lane half's row offset
    const int o1 = __shfl_xor(y1[t], 32), oi = __shfl_xor(id[t], 32), o2 = __shfl_xor(y2[t], 32);
    merge2i(y1[t], id[t], y2[t], o1, oi, o2);
    const int qt = qt0 + t;
    if (lane < 32 && qt < nqt) {
      const int64_t q = (int64_t)qt * 32 + lane;
      const int n2 = qn[q];
      const int64_t o = (int64_t)sp * nq_pad + q;
      pd1[o] = y1[t] < -(1 << 29) ? 3.0e38f : (float)(n2 - y1[t]);
      pidx[o] = id[t];
      pd2[o] = y2[t] < -(1 << 29) ? 3.0e38f : (float)(n2 - y2[t]);
    }
  }
}

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Row-finding pass for the BFMatcher.knnMatch drop-in on the int8 layout (the counterpart
// of match.hip's match_kernel<true>): per query the LOWEST row other than excl[q] whose
// exact squared distance lies in [flo[q], fhi[q]] (the integers whose sqrtf is one float
// distance).  distance^2 = ||q'||^2 - y with y = 2 (q'.d' + c) + p exactly, so the test is
// y in [||q'||^2 - fhi, ||q'||^2 - flo] -- integer compares.  A wave keeps kFindQT query tiles
// in VGPRs and walks its subtiles of the work-group's DB chunk in increasing order (A
// fragments and the c / parity words straight from global: an auxiliary pass, not the hot
// loop); the lowest hit per lane is min-merged over the lane groups and atomicMin-merged over
// waves and chunks into found[q] (0x7f7f7f7f = none, preset by the launcher).
constexpr int kFindQT = 4;
constexpr int kFindWaves = 4;
__global__ __launch_bounds__(kFindWaves * 64) void find_rows_i8_kernel(
    const uint8_t* __restrict__ dbpack, const int* __restrict__ dn, int64_t nsub,
    const uint8_t* __restrict__ qpack, const int* __restrict__ qn, int nqt, int split,
    int64_t sub_per_split, int row_offset, const float* __restrict__ flo,
    const float* __restrict__ fhi, const int* __restrict__ excl, int* __restrict__ found) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sp = blockIdx.x % split, qb = blockIdx.x / split;
  const int qt0 = qb * kFindQT;
  const int64_t npad = nsub * kSubRows;
  i32x4 bq[kFindQT][2];
  int ylo[kFindQT], yhi[kFindQT], ex[kFindQT], id[kFindQT];
#pragma unroll
  for (int t = 0; t < kFindQT; ++t) {
    const int qt = qt0 + t;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      bq[t][k] = qt < nqt ? *reinterpret_cast<const i32x4*>(qpack + ((int64_t)qt * 2 + k) * 1024 + lane * 16)
                          : i32x4{0, 0, 0, 0};
    const int64_t q = (int64_t)qt * 16 + (lane & 15);
    ylo[t] = 1;   // empty
    yhi[t] = 0;
    ex[t] = -1;
    id[t] = 0x7fffffff;
    if (qt < nqt && flo[q] <= fhi[q]) {   // integers < 2^24: exact
      ylo[t] = qn[q] - (int)fhi[q];
      yhi[t] = qn[q] - (int)flo[q];
      ex[t] = excl[q];
    }
  }
  const int64_t s_lo = (int64_t)sp * sub_per_split;
  const int64_t s_hi = min(nsub, s_lo + sub_per_split);
  for (int64_t u = s_lo + wave; u < s_hi; u += kFindWaves) {
    const uint8_t* a = dbpack + u * kSub + lane * 16;
    const i32x4 a0 = *reinterpret_cast<const i32x4*>(a);
    const i32x4 a1 = *reinterpret_cast<const i32x4*>(a + 1024);
    const int64_t r0 = u * kSubRows + (lane >> 4) * 4;   // the lane's 4 rows
    const i32x4 c = *reinterpret_cast<const i32x4*>(dn + r0);
    const i32x4 p = *reinterpret_cast<const i32x4*>(dn + npad + r0);
    const int rowb = row_offset + (int)r0;
#pragma unroll
    for (int t = 0; t < kFindQT; ++t) {
      i32x4 acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq[t][0], c, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq[t][1], acc, 0, 0, 0);
#pragma unroll
      for (int r = 3; r >= 0; --r) {   // the lowest matching row of the four wins
        const int y = 2 * acc[r] + p[r];
        const bool in = y >= ylo[t] && y <= yhi[t] && rowb + r != ex[t];
        id[t] = (in && rowb + r < id[t]) ? rowb + r : id[t];
      }
    }
  }
#pragma unroll
  for (int t = 0; t < kFindQT; ++t) {
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) id[t] = min(id[t], __shfl_xor(id[t], m));
    const int qt = qt0 + t;
    if (lane < 16 && qt < nqt && id[t] != 0x7fffffff)
      atomicMin(&found[(int64_t)qt * 16 + lane], id[t]);
  }
}

}  // namespace

// per query the lowest row other than excl[q] whose exact squared distance lies in
// [flo[q], fhi[q]] over the int8-packed DB (16x16x64 layout; arrays [nq_pad] on the device);
// found[q] = 0x7f7f7f7f where there is none
int launch_find_rows_i8(sod_ctx* ctx, const float* flo, const float* fhi, const int32_t* excl,
                        int32_t* found) {
  if (ctx->impl != 1) return sod_fail(ctx, SOD_ESTATE, "find_rows_i8: int8 16x16x64 layout only");
  const int64_t nq_pad = (int64_t)ctx->nqt * kSubRows;
  const int64_t qblocks = cdiv(ctx->nqt, kFindQT);
  // about 8 work-groups per CU in total, chunks of whole subtiles
  int64_t split = std::max<int64_t>(1, 8LL * ctx->num_cus / qblocks);
  split = std::min<int64_t>(split, cdiv(ctx->nsub, kFindWaves));
  const int64_t sub_per_split = cdiv(ctx->nsub, split);
  split = cdiv(ctx->nsub, sub_per_split);
  SOD_HIP(ctx, hipMemsetAsync(found, 0x7f, (size_t)nq_pad * 4, ctx->stream));
  hipLaunchKernelGGL(find_rows_i8_kernel, dim3((unsigned)(qblocks * split)), dim3(kFindWaves * 64),
                     0, ctx->stream, ctx->dbpack.p, reinterpret_cast<const int*>(ctx->dn.p),
                     ctx->nsub, ctx->qpack.p, reinterpret_cast<const int*>(ctx->qn.p), ctx->nqt,
                     (int)split, sub_per_split, (int)ctx->row_offset, flo, fhi, excl, found);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_pack_i8(sod_ctx* ctx, const void* dsrc, int dtype, int64_t n, bool db) {
  const bool wide = ctx->impl == 2;
  const int rows = wide ? 32 : kSubRows;            // rows per subtile / queries per tile
  const int sub_bytes = wide ? w::kSub : kSub;
  // DB padded to whole stages of both layouts (kStageRows and the wide kernel's stage of
  // w::SPS 32-row subtiles: 512 rows -- equal to kStageRows at the default 32 subtiles)
  const int64_t spad = std::max<int64_t>(kStageRows, (int64_t)w::SPS * 32);
  const int64_t npad = db ? cdiv(n, spad) * spad : cdiv(n, rows) * rows;
  uint8_t* pack;
  int* norms;
  if (db) {
    ctx->nsub = npad / rows;
    SOD_TRY(sod_reserve(ctx, ctx->dbpack, (size_t)ctx->nsub * sub_bytes));
    SOD_TRY(sod_reserve(ctx, ctx->dn, (size_t)(2 * npad)));   // c and parity
    pack = ctx->dbpack.p;
    norms = reinterpret_cast<int*>(ctx->dn.p);
  } else {
    ctx->nqt = (int32_t)(npad / rows);
    SOD_TRY(sod_reserve(ctx, ctx->qpack, (size_t)ctx->nqt * sub_bytes));
    SOD_TRY(sod_reserve(ctx, ctx->qn, (size_t)npad));
    pack = ctx->qpack.p;
    norms = reinterpret_cast<int*>(ctx->qn.p);
  }
  const int64_t threads = npad * 8;
  const int bs = 256;
  const unsigned grid = (unsigned)cdiv(threads, bs);
  const int padnorm = db ? kPadNormI : 0;
  const int slot = db ? 1 : 2;
#define SOD_PACK(T, W)                                                                     \
  hipLaunchKernelGGL((pack_i8_kernel<T, W>), dim3(grid), dim3(bs), 0, ctx->stream,         \
                     (const T*)dsrc, n, npad, pack, norms, padnorm, ctx->flags.p, slot)
  if (dtype == SOD_DTYPE_U8) {
    if (wide) SOD_PACK(uint8_t, true); else SOD_PACK(uint8_t, false);
  } else {
    if (wide) SOD_PACK(float, true); else SOD_PACK(float, false);
  }
#undef SOD_PACK
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

// words per query of one shared-threshold slot (t2 + the two best-row words)
int64_t sod_thr_words(const sod_ctx*) { return kThrWords; }

// Query tiles per wave for the 16x16x64 kernel.  A work-group holds 8*QT tiles; the chip is
// filled by splitting the DB into chunks, and every chunk restarts its queries' top-2 (the
// dense early phase), so fewer queries per work-group buy longer chunks and no padding tiles
// for small query sets, at more LDS reads per MFMA.  Option match_qt overrides (experiments).
static int pick_qt(const sod_ctx* ctx, int32_t nqt) {
  {
    const int v = ctx->opt.match_qt;
    if (v == 2 || v == 4 || v == 8) return v;
  }
  // measured (C3-sized DB, one MI355X): 8 from ~16 work-groups of 1024 queries up (20k
  // queries: 8 is 3 % faster than 4), 4 below (10k x 100k: 11 % faster than 8; 2k x 1M: 12 %),
  // 2 for one query image (500 queries: 2 and 4 equal, both 38 % faster than 8)
  if (nqt >= 64 * 16) return 8;
  if (nqt > 32) return 4;
  return 2;
}

// waves per query slice (match_unit's PAIR); option match_pair overrides
static int pick_pair(const sod_ctx* ctx, int qt) {
  {
    const int v = ctx->opt.match_pair;
    if (v == 1 || (v == 2 && qt >= 4)) return v;
  }
  return 1;
}

// LDS prefetch distance (subtiles) per query tiles per wave; option match_pf overrides
static int pick_pf(const sod_ctx* ctx, int qt) {
  {
    const int v = ctx->opt.match_pf;
    if (v == 1 || v == 2) return v;
  }
  return 1;
}

int launch_match_i8(sod_ctx* ctx) {
  const bool wide = ctx->impl == 2;
  const int rows = wide ? 32 : kSubRows;
  const int sps = wide ? w::SPS : SPS;
  const int wqt = ctx->opt.match_qt == 1 || ctx->opt.match_qt == 2 ? ctx->opt.match_qt : w::QT;
  const int qt = wide ? wqt : pick_qt(ctx, ctx->nqt);
  const int pair = wide ? 1 : pick_pair(ctx, qt);
  const int qt_per_wg = wide ? w::NW * qt : NW16 / pair * qt;
  const int64_t nq_pad = (int64_t)ctx->nqt * rows;
  const int64_t qblocks = cdiv(ctx->nqt, qt_per_wg);
  const int64_t nstages = ctx->nsub / sps;
  // one round of work-groups (8 waves per CU): as few DB chunks as fill the chip (every chunk
  // restarts each query's running top-2, so more chunks mean more slow-path updates)
  // (work-groups per CU: as many as asked for and the LDS holds -- the ring kernel's 128 KiB
  // ring leaves room for one, whatever its wave count)
  const int64_t lds_wg = kRing * kStageBytes + kNormRing * kStageNorm +
                         (int64_t)SOD_I8_XCHUNK * NW16 * qt * 64 * kThrWords;   // (at most)
  const int64_t per_cu = wide ? ((w::NW == 4) ? 2 : 1)
                              : std::max<int64_t>(1, std::min<int64_t>(
                                    (NW16 == 4 ? 2 : 1) * (qt == 2 ? SOD_I8_QT2_WGS : 1),
                                    (160 * 1024) / lds_wg));
  const int64_t slots = per_cu * ctx->match_cus();   // in flight
  // (rounded down: one work-group more than the slots would run as a second round)
  int64_t split = std::max<int64_t>(1, slots / qblocks);
  split = std::min<int64_t>(split, nstages);
  int64_t st_per_split = cdiv(nstages, split);
  // a chunk is addressed through one buffer descriptor (32-bit byte offsets): < 1 GiB each
  const int64_t max_st = ((int64_t)1 << 30) / (wide ? w::kStageBytes : kStageBytes);
  if (st_per_split > max_st) st_per_split = max_st;
  split = cdiv(nstages, st_per_split);
  ctx->split = (int)split;
  SOD_TRY(sod_reserve(ctx, ctx->cd1, (size_t)nq_pad));
  SOD_TRY(sod_reserve(ctx, ctx->cd2, (size_t)nq_pad));
  SOD_TRY(sod_reserve(ctx, ctx->cidx, (size_t)nq_pad));
  hipStream_t ks;   // context stream, or the matcher's (sod_match_set_overlap)
  float *pd1, *pd2;
  int32_t* pidx;
  SOD_TRY(sod_match_stream_begin(ctx, split * nq_pad, &ks, &pd1, &pidx, &pd2));
  // shared thresholds, one array per partial-result slot: "nothing known" is bytes 0x80 (below
  // every reachable t2); the merge that releases a slot resets its array for the next launch,
  // a new slot layout (query count, kernel shape) resets BOTH slots here (stream_begin waited for both
  // merges) -- also the one an overlap-off context never uses, so switching overlap on later
  // (sod_match_set_overlap / sod_set_cu_reserve, which also clear gthr_n) never reads
  // uninitialised thresholds
  int32_t* gthr = nullptr;
  if (!wide) {
    const int64_t gslot = sod_thr_words(ctx) * nq_pad;   // words of one slot
    if (ctx->gthr.n < (size_t)(2 * gslot) || ctx->gthr_n != gslot) {
      if (ctx->gthr.n < (size_t)(2 * gslot)) {
        SOD_HIP(ctx, sod_stream_sync(ctx->mstream));
        SOD_HIP(ctx, sod_stream_sync(ctx->mstream2));
        SOD_HIP(ctx, sod_stream_sync(ctx->stream));
        SOD_TRY(sod_reserve(ctx, ctx->gthr, (size_t)(2 * gslot)));
      }
      // (a new layout: the other slot's matcher, possibly still running on the other matcher
      // stream, must not write bounds of the old layout into it)
      if (ctx->mtwo && !ctx->mk_main) SOD_HIP(ctx, sod_stream_sync(ctx->mstream_of(ctx->pslot ^ 1)));
      SOD_HIP(ctx, hipMemsetAsync(ctx->gthr.p, 0x80, (size_t)(2 * gslot) * 4, ks));
      ctx->gthr_n = gslot;
    }
    gthr = ctx->gthr.p + ctx->pslot * gslot;
  }
  const int seedload = split <= 64 ? 1 : 0;   // see match_unit (SOD_I8_SEEDLOAD)
  hipEvent_t eb, ee;
  SOD_TRY(sod_match_events(ctx, &eb, &ee));
  if (wide) {
#define SOD_LAUNCH_I8W(Q)                                                                     \
    hipExtLaunchKernelGGL(match_i8w_kernel<Q>, dim3((unsigned)(qblocks * split)), dim3(w::NT), 0, \
                          ks, eb, ee, 0, ctx->dbpack.p, reinterpret_cast<const int*>(ctx->dn.p),  \
                          ctx->nsub, ctx->qpack.p, reinterpret_cast<const int*>(ctx->qn.p),       \
                          ctx->nqt, nq_pad, (int)split, st_per_split * sps,                       \
                          (int)ctx->row_offset, pd1, pidx, pd2, (int)qblocks)
    if (qt == 1) SOD_LAUNCH_I8W(1); else if (qt == 2) SOD_LAUNCH_I8W(2); else SOD_LAUNCH_I8W(w::QT);
#undef SOD_LAUNCH_I8W
  }
  else {
#define SOD_LAUNCH_I8(Q, P, R)                                                                \
  hipExtLaunchKernelGGL((match_i8_kernel<Q, P, R>), dim3((unsigned)(qblocks * split)), dim3(NT16), 0, \
                        ks, eb, ee, 0, ctx->dbpack.p, reinterpret_cast<const int*>(ctx->dn.p),  \
                        ctx->nsub, ctx->qpack.p, reinterpret_cast<const int*>(ctx->qn.p),       \
                        ctx->nqt, nq_pad, (int)split, st_per_split * sps, (int)ctx->row_offset, \
                        pd1, pidx, pd2, (int)qblocks, gthr, seedload)
    const int pf = pick_pf(ctx, qt);
    if (pair == 2) {   // paired waves: 4 or 8 query tiles per wave, prefetch 1
      if (qt == 8) SOD_LAUNCH_I8(8, 1, 2); else SOD_LAUNCH_I8(4, 1, 2);
    } else if (qt == 8) {
      if (pf == 2) SOD_LAUNCH_I8(8, 2, 1); else SOD_LAUNCH_I8(8, 1, 1);
    } else if (qt == 4) {
      if (pf == 2) SOD_LAUNCH_I8(4, 2, 1); else SOD_LAUNCH_I8(4, 1, 1);
    } else {
      if (pf == 2) SOD_LAUNCH_I8(2, 2, 1); else SOD_LAUNCH_I8(2, 1, 1);
    }
#undef SOD_LAUNCH_I8
  }
  SOD_HIP(ctx, hipGetLastError());
  SOD_TRY(sod_match_stream_end(ctx, ee));
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, false));
  SOD_TRY(launch_merge(ctx, pd1, pidx, pd2, (int)split, nq_pad, gthr,
                       ctx->nranks <= 1 && !ctx->comm));   // no exchange follows: final
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, true));
  return sod_partials_merged(ctx);   // the slot is free again
}
