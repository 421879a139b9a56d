// match_s.hip -- the k=2 matcher for small query sets (one query image of ~500 keypoints up to
// a few thousand queries), the regime main.py runs: knnMatch of ONE image's descriptors
// against the whole DB (/root/reference/main.py:68-86).
//
// Same arithmetic as match_i8.hip (int8 of value - 128 on v_mfma_i32_16x16x64_i8, row norm
// folded into the accumulator init as c = floor(-||d'||^2 / 2), y = 2h + parity, the two
// largest y per query exact), different shape.  match_i8_kernel keeps 2-8 query tiles per
// wave in VGPRs and streams the DB through an LDS ring shared by 8 waves: at 2 tiles per wave
// (one query image) each 2 KiB DB fragment read from LDS feeds only 4 MFMAs and the LDS array,
// not the matrix pipe, sets the pace.  Here a wave holds a whole 512-query group -- 32 tiles x
// 2 k-steps = 64 B fragments, 256 registers, in the accumulator file (MFMA B operands may be
// AGPRs) -- and streams ITS OWN DB rows straight from global memory into VGPRs: every 2 KiB
// subtile feeds 64 MFMAs, every DB row is read once per query group (one query image: the DB
// once, compulsory traffic only), no LDS ring, one wave per SIMD.
//
// Prefilter over windows of kSN subtiles: per tile and lane a running max of the window's
// h values (2 v_max3 per subtile), then ONE compare against the query's threshold t2 per
// window -- 1.25 VALU per MFMA at kSN = 2 instead of 1.5.  A tile whose window passes is
// recomputed (its 2 kSN MFMAs) and takes the exact top-2 update: each lane keeps the exact
// top-2 of ITS rows (4 per subtile) for its query in LDS (lane-private slots, no atomics);
// the threshold is the query's second best over its four lane groups (permlane swaps).
// Rows of a lane are visited in increasing order, so the strict > keeps the lowest trainIdx.
//
// Thresholds: a wave first runs kSeedW windows with only the running max (no compare): the
// second largest of a query's four lane-group maxima comes from two distinct rows, so it is
// a valid threshold from the first exact window on.  The work-groups of a query group (one
// per DB range) share bounds without atomics: each keeps per query the top-2 (row value, id
// of the work-group whose row reaches it) of distinct ids it knows of -- its own best row and
// what it read -- and publishes that list to a slot of its own with plain stores; at
// exchange r it merges the slot of work-group (sp - 2^(r mod log2 n)) mod n into its list
// (a dissemination pattern: after log2 n rounds every list has seen every work-group).  The
// second entry is reached by two distinct rows, so no row below it is in the query's global
// top-2.  A stale slot is still a valid bound: loads are issued one exchange ahead of their
// use and nothing waits for them.  (Atomic max on one shared word per query -- round 5's
// first build -- serialised 256 work-groups' publications at the memory side: ~60 us.)
//
// Output: per work-group (4 waves = one DB range) the partial top-2 of every query of its
// group, merged over the waves and lane groups in LDS, into slot sp of pd1 / pidx / pd2 --
// the layout merge_kernel (match.hip) reduces.
#include <climits>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include <hip/hip_ext.h>

#include "sod_internal.h"

typedef __attribute__((ext_vector_type(4))) int i32x4;

namespace {

constexpr int kSQT = 32;          // query tiles per wave (a 512-query group)
constexpr int kSNW = 4;           // waves per work-group (one per SIMD)
#ifndef SOD_S_D
#define SOD_S_D 6                 // DB subtiles in flight per wave (register ring)
#endif
#ifndef SOD_S_N
#define SOD_S_N 2                 // subtiles per prefilter window
#endif
#ifndef SOD_S_SEEDW
#define SOD_S_SEEDW 1             // seed windows (running max only) before the exact pass
#endif
constexpr int kSD = SOD_S_D;
constexpr int kSN = SOD_S_N;
constexpr int kSeedW = SOD_S_SEEDW;
static_assert(kSD % kSN == 0 && kSeedW * kSN <= kSD, "ring holds whole windows and the seed");
constexpr int kSW = kSD / kSN;    // windows per loop body
#ifndef SOD_S_LAG
#define SOD_S_LAG 2               // tiles between a tile's MFMAs and its prefilter
#endif
constexpr int kLag = SOD_S_LAG;
#ifndef SOD_S_XCHG
#define SOD_S_XCHG 1              // thresholds shared between the waves of a query group
#endif
constexpr bool kXchg = SOD_S_XCHG;
#ifndef SOD_S_EARLYB
#define SOD_S_EARLYB 4            // loop bodies that exchange after every window
#endif
#ifndef SOD_S_PRELOAD
#define SOD_S_PRELOAD 1           // a hit window's subtiles copied, its refill issued first
#endif
constexpr bool kPreload = SOD_S_PRELOAD;
constexpr int kEarlyB = SOD_S_EARLYB;
constexpr int kSubB = 2048;       // bytes per 16-row subtile
constexpr int kRsrc3 = 0x00020000;
// accumulator init of a subtile beyond the wave's range: h < -2^30 <= every threshold, and
// no wrap (|q'.d'| <= 2^21)
constexpr int kMaskC = INT_MIN + (1 << 22);
// LDS boards per query group: lane j's 32 words at j * kGStride (a padded row: the 16 lanes'
// LDS reads of one tile word hit different banks)
constexpr int kGStride = kSQT + 4;
constexpr int kGroupWords = 16 * kGStride;
// a work-group's published top-2 (packed, below) of its query group: query (t, j) at words
// j * kLStride + 2t, 2t + 1; the same layout in LDS (the work-group's board) and in its
// global slot
constexpr int kLStride = 2 * kSQT + 4;
constexpr int kSlotWords = 16 * kLStride;

// a bound entry: a row value h (>= -2^22: any reachable h of a real row; kMaskC rows are
// clamped, they never become a bound) and the id of the work-group whose row reaches it --
// ordered by h, then id.  Two entries of different ids are reached by two distinct rows.
__device__ __forceinline__ int bpack(int h, int id) { return (max(h, -(1 << 22)) << 8) | id; }
// top-2 of distinct ids of two top-2 lists (each of distinct ids, a1 >= a2, b1 >= b2): the
// first is the larger first; the second the largest entry of another id (copies of one
// id -- a work-group's value seen at two times -- count once)
__device__ __forceinline__ void bmerge(int& a1, int& a2, int b1, int b2) {
  const int f = max(a1, b1), fid = f & 255;
  int s2 = (a1 & 255) != fid ? a1 : INT_MIN;
  s2 = max(s2, (a2 & 255) != fid ? a2 : INT_MIN);
  s2 = max(s2, (b1 & 255) != fid ? b1 : INT_MIN);
  s2 = max(s2, (b2 & 255) != fid ? b2 : INT_MIN);
  a1 = f;
  a2 = s2;
}

__device__ __forceinline__ int imed3(int a, int b, int c) {
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }

// top-2 values of {a, partner's a} for lane pairs (l, l^32) / (l, l^16) (match_i8.hip)
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

struct Sub {
  i32x4 a0, a1;   // DB fragments (k-steps 0, 1)
  i32x4 c;        // accumulator init: c of the lane's 4 rows (kMaskC beyond the range)
  i32x4 p;        // parity words of the lane's 4 rows
};

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1.  The loops that
// index register arrays (the DB ring, the query fragments, the thresholds) must be unrolled;
// #pragma unroll gives up on bodies as large as the slow path ("unrolled size too large"),
// and a register array indexed at run time lives in scratch memory.
template <class F, int... I>
__device__ __forceinline__ void sfor_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}

#ifdef SOD_S_COUNT
// diagnostic build only: [0] windows, [1] windows with a hit, [2] hit tiles
__device__ unsigned long long g_scounts[8];
#endif
#ifdef SOD_S_STAMP
// diagnostic build only: per wave (block * 4 + wave) s_memtime at [0] start, [1] query
// fragments loaded, seed: [2] scan, [3] pushes, [4] barrier, [5] apply, [6] load issued, [7]
// pull; body 0: [8 + 3w] window w scanned, [9 + 3w] its slow path done, [10 + 3w] its
// exchange done (w < 3); [16 + b] body b (1 <= b <= 8) starts; [25] end; s_memrealtime at
// start / end in [26] / [27]
__device__ unsigned long long g_sstamps[4096][28];
// hit tiles per wave and body: [0..7] bodies 0..7, [8] the later bodies together
__device__ unsigned g_shits[4096][9];
#define SSTAMP(i)                                                                 \
  do {                                                                            \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                   \
    if (lane == 0 && blockIdx.x * 4 + wave < 4096) g_sstamps[blockIdx.x * 4 + wave][(i)] = t_; \
  } while (0)
#else
#define SSTAMP(i) \
  do {            \
  } while (0)
#endif

template <int QT>
__global__ __launch_bounds__(kSNW * 64, 1) void match_s_kernel(
    const uint8_t* __restrict__ dbpack, const int* __restrict__ dn, int64_t nsub,
    const uint8_t* __restrict__ qpack, const int* __restrict__ qn, int nqt, int64_t nq_pad,
    int64_t sub_per_split, int row_offset, float* __restrict__ pd1, int* __restrict__ pidx,
    float* __restrict__ pd2, int nqb, int* __restrict__ gthr) {
  // gthr: [query group][DB range][kSlotWords] published top-2 lists
  static_assert(QT == 32, "a lane's 32 threshold words are 8 wide loads; 8 tiles per exchanging wave");
  // exact top-2 per (wave, tile, field, lane): 24 KiB per wave
  __shared__ int top2[kSNW * QT * 3 * 64];
  // threshold boards of the work-group (below)
  __shared__ __attribute__((aligned(16))) int t2b[kGroupWords], bb[kGroupWords];
  __shared__ __attribute__((aligned(16))) int tb[16 * kLStride];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // XCD-aware order (match_i8.hip): blocks b, b+8, ... share an XCD; each XCD gets a
  // contiguous run of range-major units, so the query groups of one DB range share its L2
  const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = blockIdx.x % 8;
  const unsigned u = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + blockIdx.x / 8;
  const int sp = (int)(u / nqb), qb = (int)(u % nqb);

  const int64_t s_lo = (int64_t)sp * sub_per_split;
  const int64_t s_hi = min(nsub, s_lo + sub_per_split);
  const int64_t npad = nsub * kSubRows;
  // this wave's subtiles: s_lo + wave + kSNW * i, i < nloc
  const int nloc = (int)max<int64_t>(0, (s_hi - s_lo - wave + kSNW - 1) / kSNW);
  const int qt0 = qb * QT;
  const int ntile = min(QT, nqt - qt0);
  SSTAMP(0);
#ifdef SOD_S_STAMP
  if (lane == 0 && blockIdx.x * 4 + wave < 4096)
    g_sstamps[blockIdx.x * 4 + wave][26] = __builtin_amdgcn_s_memrealtime();
#endif

  // buffers over the work-group's DB range (byte offsets < 2^31: sod_match_s_geometry)
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dbpack + s_lo * kSubB), (short)0, (int)((s_hi - s_lo) * kSubB), kRsrc3);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dn + s_lo * kSubRows), (short)0, (int)((s_hi - s_lo) * kSubRows * 4), kRsrc3);
  const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dn + npad + s_lo * kSubRows), (short)0, (int)((s_hi - s_lo) * kSubRows * 4), kRsrc3);

  auto load_sub = [&](Sub& d, int i) {
    const bool ok = i < nloc;   // wave-uniform
    const uint32_t so = ok ? (uint32_t)(wave + kSNW * i) : 0u;
    d.a0 = __builtin_amdgcn_raw_buffer_load_b128(rsa, (uint32_t)lane * 16u, so * kSubB, 0);
    d.a1 = __builtin_amdgcn_raw_buffer_load_b128(rsa, (uint32_t)lane * 16u + 1024u, so * kSubB, 0);
    const i32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rsc, (uint32_t)g * 16u, so * 64u, 0);
    d.p = __builtin_amdgcn_raw_buffer_load_b128(rsp, (uint32_t)g * 16u, so * 64u, 0);
    d.c = ok ? c : i32x4{kMaskC, kMaskC, kMaskC, kMaskC};
  };

  // the DB stream starts first (its HBM latency overlaps the query fragments' load)
  Sub ring[kSD];
  sfor<kSD>([&](auto J) { load_sub(ring[J], J); });

  // the query group, resident as MFMA B operands (the accumulator file: an MFMA reads its B
  // operand from there directly; the VGPRs keep the DB ring, the thresholds, the accumulators).
  // The 64 KiB of fragments are loaded once per work-group (each wave a quarter, through the
  // LDS the top-2 slots take later), not once per wave: 4x less L2 traffic at the start
  // (1 024 waves reading the same 64 KiB took ~8 k cycles)
  i32x4 bq[QT][2];
  {
    i32x4* stage = reinterpret_cast<i32x4*>(top2);   // [tile t][k][lane] = 64 KiB
    static_assert(sizeof(top2) >= QT * 2 * 64 * 16, "fragment staging fits the top-2 slots");
#pragma unroll
    for (int i = 0; i < 2 * QT / kSNW; ++i) {
      const int f = wave * (2 * QT / kSNW) + i;      // fragment (t, k) = (f / 2, f % 2)
      const int t = f >> 1;
      stage[f * 64 + lane] = *reinterpret_cast<const i32x4*>(
          qpack + ((int64_t)(t < ntile ? qt0 + t : qt0) * 2 + (f & 1)) * 1024 + lane * 16);
    }
    __syncthreads();
    sfor<QT>([&](auto T) {
#pragma unroll
      for (int k = 0; k < 2; ++k) bq[T][k] = stage[(2 * T + k) * 64 + lane];
    });
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
      for (int k = 0; k < 2; ++k) asm volatile("" : "+a"(bq[t][k]));
    __syncthreads();   // the staging area becomes the top-2 slots
  }
  SSTAMP(1);

  int* const slot = top2 + wave * (QT * 3 * 64) + lane;   // + (t * 3 + f) * 64
  for (int t = 0; t < QT; ++t) {
    slot[(t * 3 + 0) * 64] = INT_MIN;
    slot[(t * 3 + 1) * 64] = 0x7fffffff;
    slot[(t * 3 + 2) * 64] = INT_MIN;
  }
  int t2[QT];
  sfor<QT>([&](auto T) { t2[T] = INT_MIN >> 1; });

  // window W (ring slots W*kSN ..): the 2 kSN MFMAs per tile, software-pipelined kLag tiles
  // deep -- the running max and compare of tile t-kLag run beside tile t's MFMAs (MFMA, VALU,
  // MFMA, VALU, ...), far enough behind that no VALU waits for an MFMA result.  m[t] = the
  // lane's running max over the window; returns the OR of the tiles' ballots m >= t2 (one
  // SALU per tile; the slow path finds the tiles again from m).
  auto scan = [&](auto W, int (&m)[QT]) -> uint64_t {
    constexpr int w = W;
    uint64_t any = 0;
    i32x4 acc[kLag + 1][kSN];
    sfor<QT + kLag>([&](auto T) {
      constexpr int t = T;
      if constexpr (t < QT) {
#pragma unroll
        for (int j = 0; j < kSN; ++j)
          acc[t % (kLag + 1)][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
              ring[w * kSN + j].a0, bq[t][0], ring[w * kSN + j].c, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < kSN; ++j)
          acc[t % (kLag + 1)][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
              ring[w * kSN + j].a1, bq[t][1], acc[t % (kLag + 1)][j], 0, 0, 0);
      }
      if constexpr (t >= kLag) {
        constexpr int tp = t - kLag;
        const i32x4* a = acc[tp % (kLag + 1)];
        int mm = imax3(a[0][0], a[0][1], a[0][2]);
        mm = max(mm, a[0][3]);
#pragma unroll
        for (int j = 1; j < kSN; ++j) {
          mm = imax3(mm, a[j][0], a[j][1]);
          mm = imax3(mm, a[j][2], a[j][3]);
        }
        asm volatile("" : "+v"(mm));   // computed here, not sunk to a later use
        m[tp] = mm;
        any |= __builtin_amdgcn_ballot_w64(mm >= t2[tp]);
      }
      if constexpr (t >= kLag && t < QT) {
#pragma unroll
        for (int i = 0; i < 2 * kSN - 1; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);   // MFMA
          __builtin_amdgcn_sched_group_barrier(0x2, 1, 0);   // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 2 * kSN - 2, 0);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep each tile's block as laid out above
    });
    return any;
  };

  // ---- thresholds shared between waves and work-groups ----
  // LDS boards of the work-group (its 4 waves hold the same queries), layout [lane j]
  // [kGStride]: t2b = the best bound known per query (h), bb = the best row value (h) the
  // work-group has seen per query; tb = the work-group's top-2 list (layout [j][kLStride]).
  // Wave w exchanges tiles [8w, 8w+8), lane (g, j) the tiles 8w + 2g, 8w + 2g + 1 of query
  // j: one 16-byte word group of the list per lane
  const int nsplit = (int)(gridDim.x / nqb);
  const int nbits = nsplit > 1 ? 32 - __builtin_clz((unsigned)(nsplit - 1)) : 0;
  int* const gslot = gthr + (int64_t)qb * nsplit * kSlotWords;
  const uint32_t lo_off = (uint32_t)(j16 * kLStride + 2 * (wave * (QT / kSNW) + 2 * g)) * 4u;
  const __amdgpu_buffer_rsrc_t rsg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)gslot, (short)0, nsplit * kSlotWords * 4, kRsrc3);
  const int xt = wave * (QT / kSNW) + 2 * g;   // the lane's first exchanged tile
  i32x4 pe = i32x4{INT_MIN, INT_MIN, INT_MIN, INT_MIN};   // loaded partner entries
  int xr = 0;                                              // exchange rounds so far
  for (int i = tid; i < kGroupWords; i += kSNW * 64) {
    t2b[i] = INT_MIN >> 1;
    bb[i] = INT_MIN >> 1;
  }
  for (int i = tid; i < 16 * kLStride; i += kSNW * 64) tb[i] = INT_MIN;
  __syncthreads();
  // the partner slot of the next round, loaded (sc1: past this XCD's L2) for the round after
  auto exch_load = [&]() {
    if constexpr (kXchg) {
      if (nbits) {
        const int p = (sp - (1 << (xr % nbits)) + nsplit) % nsplit;
        pe = __builtin_amdgcn_raw_buffer_load_b128(rsg, lo_off, (uint32_t)p * kSlotWords * 4u,
                                                   16 /* sc1 */);
      }
      ++xr;
    }
  };
  // merge the own best rows and the loaded partner list into the work-group's list, publish
  // it (write-through stores: the other XCDs read it from memory) and raise the bounds
  auto exch_apply = [&]() {
    if constexpr (kXchg) {
      i32x4 l = *reinterpret_cast<const i32x4*>(tb + j16 * kLStride + 2 * xt);
      const int o0 = bb[j16 * kGStride + xt], o1 = bb[j16 * kGStride + xt + 1];
      int a1 = l[0], a2 = l[1], c1 = l[2], c2 = l[3];
      bmerge(a1, a2, bpack(o0, sp), INT_MIN);
      bmerge(c1, c2, bpack(o1, sp), INT_MIN);
      bmerge(a1, a2, pe[0], pe[1]);
      bmerge(c1, c2, pe[2], pe[3]);
      l = i32x4{a1, a2, c1, c2};
      *reinterpret_cast<i32x4*>(tb + j16 * kLStride + 2 * xt) = l;
      __builtin_amdgcn_raw_buffer_store_b128(l, rsg, lo_off, (uint32_t)sp * kSlotWords * 4u,
                                             17 /* sc0 sc1 */);
      __hip_atomic_fetch_max(&t2b[j16 * kGStride + xt], a2 >> 8, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_max(&t2b[j16 * kGStride + xt + 1], c2 >> 8, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };
  auto pull = [&]() {
    const int* tb2 = t2b + j16 * kGStride;
    sfor<QT / 4>([&](auto I) {
      const i32x4 v = *reinterpret_cast<const i32x4*>(tb2 + 4 * I);
#pragma unroll
      for (int k = 0; k < 4; ++k) t2[4 * I + k] = max(t2[4 * I + k], v[k]);
    });
  };
  // a tile's new bound (h units) and best row value (h) onto the boards
  auto push = [&](int t, int bound, int best) {
    if (lane < 16) {
      __hip_atomic_fetch_max(&t2b[j16 * kGStride + t], bound, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_max(&bb[j16 * kGStride + t], best, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };

  // seed: kSeedW windows of running maxima only; the second largest of a query's four
  // lane-group maxima is reached by two distinct rows, the largest by one
  {
    int sm[QT];
    sfor<QT>([&](auto T) { sm[T] = INT_MIN; });
    sfor<kSeedW>([&](auto W) {
      int m[QT];
      (void)scan(W, m);
      SSTAMP(2);
      sfor<QT>([&](auto T) { sm[T] = max(sm[T], m[T]); });
      if constexpr (W == 0 || W == kSeedW - 1) {
        sfor<QT>([&](auto T) {
          int g1 = sm[T], g2 = INT_MIN;
          top2_xor32(g1, g2);
          top2_xor16(g1, g2);
          t2[T] = max(t2[T], g2);
          push(T, t2[T], g1);
        });
        SSTAMP(3);
        __syncthreads();   // every wave's seeds are on the boards
        SSTAMP(4);
        exch_apply();   // the seeds' best rows go out at once
        SSTAMP(5);
        exch_load();
        SSTAMP(6);
        pull();
        SSTAMP(7);
      }
    });
  }

  const int rowl = row_offset + (int)(s_lo * kSubRows) + g * 4;
  const int nbody = (nloc + kSD - 1) / kSD;
  // one loop body = kSW windows; the first kEarlyB bodies (Early) exchange after every
  // window, while the bounds still move fast, the later ones once per body
  auto body = [&](auto Early, int b) {
    constexpr bool early = Early;
#ifdef SOD_S_STAMP
    if (b > 0 && b <= 8) SSTAMP(16 + b);
#endif
#ifdef SOD_S_STAMP
    unsigned hcnt = 0;
#endif
    sfor<kSW>([&](auto W) {
      constexpr int w = W;
      int m[QT];
      const uint64_t any = scan(W, m);
#ifdef SOD_S_STAMP
      if (b == 0 && w < 3) SSTAMP(8 + 3 * w);
#endif
#ifdef SOD_S_COUNT
      if (lane == 0) atomicAdd(&g_scounts[0], 1ull);
#endif
      // a window with a hit keeps a copy of its subtiles for the exact update and issues the
      // refill of its ring slots first: the update (~0.5-2 k cycles) then runs under the
      // loads' latency instead of delaying them (the ring's lead is only kSD subtiles)
      Sub keep[kSN];
      const bool hit = any != 0;
      if constexpr (kPreload) {
        if (__builtin_expect(hit, 0)) sfor<kSN>([&](auto J) { keep[J] = ring[w * kSN + J]; });
#pragma unroll
        for (int j = 0; j < kSN; ++j) load_sub(ring[w * kSN + j], (b + 1) * kSD + w * kSN + j);
      }
#ifdef SOD_S_NOSLOW
      if (b < 0)
#endif
      if (__builtin_expect(hit, 0)) {
#ifdef SOD_S_COUNT
        if (lane == 0) atomicAdd(&g_scounts[1], 1ull);
#endif
        const int i0 = b * kSD + w * kSN;   // local index of the window's first subtile
        sfor<QT>([&](auto T) {
          constexpr int t = T;
          int tt = t2[t];
          asm volatile("" : "+v"(tt));   // a fresh compare, not the scan's ballot kept alive
          if (__builtin_amdgcn_ballot_w64(m[t] >= tt) == 0) return;
#ifdef SOD_S_COUNT
          if (lane == 0) atomicAdd(&g_scounts[2], 1ull);
#endif
#ifdef SOD_S_STAMP
          ++hcnt;
#endif
          int y1 = slot[(t * 3 + 0) * 64], id = slot[(t * 3 + 1) * 64], y2 = slot[(t * 3 + 2) * 64];
#pragma unroll
          for (int j = 0; j < kSN; ++j) {
            if (i0 + j >= nloc) break;   // wave-uniform: beyond the range
            const Sub& d = kPreload ? keep[j] : ring[w * kSN + j];
            i32x4 acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(d.a0, bq[t][0], d.c, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(d.a1, bq[t][1], acc, 0, 0, 0);
            const int rowb = rowl + (wave + kSNW * (i0 + j)) * kSubRows;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int y = 2 * acc[r] | d.p[r];
              const bool gt = y > y1;
              y2 = imed3(y1, y, y2);
              id = gt ? rowb + r : id;
              y1 = gt ? y : y1;
            }
          }
          slot[(t * 3 + 0) * 64] = y1;
          slot[(t * 3 + 1) * 64] = id;
          slot[(t * 3 + 2) * 64] = y2;
          int g1 = y1, g2 = y2;
          top2_xor32(g1, g2);
          top2_xor16(g1, g2);
          t2[t] = max(t2[t], g2 >> 1);   // (equal over a query's four lanes)
          push(t, t2[t], g1 >> 1);
        });
      }
#ifdef SOD_S_STAMP
      if (b == 0 && w < 3) SSTAMP(9 + 3 * w);
#endif
      // the window's slots take the subtiles kSD ahead
      if constexpr (!kPreload) {
#pragma unroll
        for (int j = 0; j < kSN; ++j) load_sub(ring[w * kSN + j], (b + 1) * kSD + w * kSN + j);
      }
      // exchange (the list loaded one exchange ago; then the next load)
      if constexpr (early || w == kSW - 1) {
        exch_apply();
        exch_load();
        pull();
      }
#ifdef SOD_S_STAMP
      if (b == 0 && w < 3) SSTAMP(10 + 3 * w);
#endif
    });
#ifdef SOD_S_STAMP
    if (lane == 0 && blockIdx.x * 4 + wave < 4096) g_shits[blockIdx.x * 4 + wave][min(b, 8)] += hcnt;
#endif
  };
  int b = 0;
  for (; b < min(nbody, kEarlyB); ++b) body(std::true_type{}, b);
  for (; b < nbody; ++b) body(std::false_type{}, b);
  SSTAMP(25);
#ifdef SOD_S_STAMP
  if (lane == 0 && blockIdx.x * 4 + wave < 4096)
    g_sstamps[blockIdx.x * 4 + wave][27] = __builtin_amdgcn_s_memrealtime();
#endif
  __syncthreads();
  // merge the 4 waves x 4 lane groups of each query; 2 queries per thread
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ql = tid + h * (kSNW * 64);   // 0 .. 511
    const int t = ql >> 4, j = ql & 15;
    if (t >= ntile) continue;
    int y1 = INT_MIN, i1 = 0x7fffffff, y2 = INT_MIN;
#pragma unroll
    for (int wv = 0; wv < kSNW; ++wv)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int* sl = top2 + wv * (QT * 3 * 64) + (t * 3) * 64 + gg * 16 + j;
        const int o1 = sl[0], oi = sl[64], o2 = sl[128];
        if (o1 > y1 || (o1 == y1 && oi < i1)) {
          y2 = max(y1, o2);
          y1 = o1;
          i1 = oi;
        } else {
          y2 = max(y2, o1);
        }
      }
    const int64_t q = (int64_t)(qt0 + t) * 16 + j;
    const int n2 = qn[q];
    const int64_t o = (int64_t)sp * nq_pad + q;
    // padding rows only win when the shard has fewer than two real rows: keep them huge
    pd1[o] = y1 < -(1 << 29) ? 3.0e38f : (float)(n2 - y1);
    pidx[o] = i1;
    pd2[o] = y2 < -(1 << 29) ? 3.0e38f : (float)(n2 - y2);
  }
}

}  // namespace

#ifdef SOD_S_STAMP
extern "C" int sod_debug_sstamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sstamps), sizeof(g_sstamps)) == hipSuccess ? 0 : 1;
}
// per-wave hit tiles per body, summed over the launches since the last reset
extern "C" int sod_debug_shits(unsigned* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_shits), sizeof(g_shits)) != hipSuccess) return 1;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_shits)) != hipSuccess) return 1;
    if (hipMemset(p, 0, sizeof(g_shits)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
#ifdef SOD_S_COUNT
extern "C" int sod_debug_scounts(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_scounts), 64) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_scounts), z, 64) != hipSuccess) return 1;
  }
  return 0;
}
#endif

// the streamed kernel for one query image up to ~10k queries (measured: match_s vs match_i8
// per query count); sod_match_set_kernel forces either
constexpr bool kStreamedAuto = false;   // not yet faster than the ring kernel anywhere
bool sod_match_use_s(const sod_ctx* ctx) {
  if (ctx->impl != 1) return false;
  if (ctx->mkernel) return ctx->mkernel == 2;
  return kStreamedAuto && ctx->nqt >= 24 && ctx->nqt <= 640;
}

// words per query of one shared-threshold slot: match_i8's kThrWords, or for the streamed
// kernel its published lists (kSlotWords per query group and DB range)
int64_t sod_thr_words(const sod_ctx* ctx) {
  if (!sod_match_use_s(ctx)) return kThrWords;
  int64_t split, per;
  sod_match_s_geometry(ctx, &split, &per);
  const int64_t nq_pad = std::max<int64_t>(1, (int64_t)ctx->nqt * kSubRows);
  const int64_t sw = (int64_t)((ctx->nqt + kSQT - 1) / kSQT) * split * kSlotWords;
  return std::max<int64_t>(kThrWords, (sw + nq_pad - 1) / nq_pad);
}

// launch geometry: one work-group of 4 waves per CU, the query groups of one DB range side by
// side; ranges of whole subtiles
int launch_match_s_kernel(sod_ctx* ctx, hipStream_t ks, hipEvent_t eb, hipEvent_t ee,
                          float* pd1, int32_t* pidx, float* pd2, int32_t* gthr, int64_t split,
                          int64_t sub_per_split) {
  const int64_t nq_pad = (int64_t)ctx->nqt * kSubRows;
  const int64_t nqb = (ctx->nqt + kSQT - 1) / kSQT;
  if (split > 256)   // list entries carry the DB range in 8 bits (bpack)
    return sod_fail(ctx, SOD_EINVAL, "streamed matcher: more than 256 DB ranges");
  hipExtLaunchKernelGGL((match_s_kernel<kSQT>), dim3((unsigned)(nqb * split)), dim3(kSNW * 64), 0,
                        ks, eb, ee, 0, ctx->dbpack.p, reinterpret_cast<const int*>(ctx->dn.p),
                        ctx->nsub, ctx->qpack.p, reinterpret_cast<const int*>(ctx->qn.p), ctx->nqt,
                        nq_pad, sub_per_split, (int)ctx->row_offset, pd1, pidx, pd2, (int)nqb, gthr);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

// (split, sub_per_split) for ctx's shapes: as many DB ranges as fill the matcher's CUs with
// one work-group each, given the query groups
void sod_match_s_geometry(const sod_ctx* ctx, int64_t* split, int64_t* sub_per_split) {
  const int64_t nqb = (ctx->nqt + kSQT - 1) / kSQT;
  int64_t sp = std::max<int64_t>(1, ctx->match_cus() / nqb);
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, ctx->nsub / kSNW));
  int64_t per = (ctx->nsub + sp - 1) / sp;
  // byte offsets of a range through one buffer descriptor: < 1 GiB
  per = std::min<int64_t>(per, ((int64_t)1 << 30) / kSubB);
  *sub_per_split = per;
  *split = (ctx->nsub + per - 1) / per;
}
