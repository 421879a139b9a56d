// match.hip -- brute-force k=2 SIFT matcher for gfx950 (replaces cv2.BFMatcher().knnMatch,
// main.py:70-71) and the ratio test (main.py:81-86).
//
// Exactness.  SIFT descriptors are integers 0..255 (OpenCV saturate_cast<uchar>), exact in
// bf16, and -2*d is exact too.  The MFMA accumulates dn - 2 q.d with every partial sum an
// integer of magnitude < 2^24, so the f32 result is exact whatever order the hardware adds in;
// q.q is added once at the end (still < 2^24).  Squared distances are therefore exact
// integers and sqrtf (correctly rounded) reproduces OpenCV's float distance bit for bit.
//
// Layout.  D = A.B with A = DB rows (16-row subtiles), B = queries (16-query tiles),
// v_mfma_f32_16x16x32_bf16: lane l holds A[row l&15][k 8(l>>4)..+7] and B[k..][col l&15];
// the result register r of lane l is row (l>>4)*4+r, column l&15.  So a lane owns ONE query
// and walks DB rows in increasing order: the k=2 reduction is lane-local (no shuffles) and
// strict '<' keeps the lowest trainIdx on ties, as OpenCV's insertion does.  Subtiles are
// pre-packed in HBM in exactly the fragment order ([kstep][lane][16 B]), so the LDS image of
// a stage is a straight copy and every ds_read_b128 is a contiguous, conflict-free 1 KiB.
//
// ||d||^2 is folded into the accumulator init (C operand = the 4 row norms of the lane), so
// the MFMA output is already dn - 2 q.d: no epilogue add.  Epilogue per 16x16 tile: a 2-op min
// of the lane's 4 values against its running 2nd-best (wave-uniform branch); only when some
// lane can improve does the exact top-2 update run (rare after the first few thousand rows).
//
// Decomposition.  A workgroup = NW waves x QT query tiles (512 queries) kept in VGPRs for
// the whole launch; it streams one DB split through a 2-slot LDS ring filled by LDS-DMA
// (global_load_lds, the next stage in flight, vmcnt + raw s_barrier, one barrier per
// 128-row stage).  Per 16-row subtile a wave issues 32 MFMAs into 8 independent
// accumulators, then one compare pass and ONE wave-uniform branch.  Grid = query blocks x DB splits, sized to fill every CU twice;
// per-split partial top-2 are merged by merge_kernel (also used for the multi-GPU merge).
#include <hip/hip_ext.h>

#include "sod_internal.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#ifndef SOD_MATCH_PREFETCH
#define SOD_MATCH_PREFETCH 1   // read the next subtile's fragments during this one's MFMAs
#endif

namespace {

constexpr int QT = 8;    // 16-query tiles per wave
constexpr int NW = 4;    // waves per workgroup
constexpr int SPS = 8;   // 16-row subtiles per LDS stage (128 rows = 32 KiB)
constexpr int NT = NW * 64;
constexpr int kStageBytes = SPS * kSubBytes;
constexpr int kStageNorm = SPS * kSubRows * 4;
constexpr float kInit = 3.0e38f;


// ---------------------------------------------------------------------------------------
// pack: rows -> MFMA-fragment order, bf16 (x scale), plus exact squared norms.
// One thread per (row, 8-dim chunk c).  Fragment: subtile r/16, kstep c/4,
// lane (r%16) + 16*(c%4), 16 bytes.
template <typename TIn>
__global__ void pack_rows_kernel(const TIn* __restrict__ src, int64_t n, int64_t npad,
                                 float scale, uint8_t* __restrict__ pack,
                                 float* __restrict__ norms, float padnorm,
                                 uint32_t* __restrict__ flags, int max_slot) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t >> 4;
  const int c = (int)(t & 15);
  if (row >= npad) return;  // npad*16 threads is a multiple of 64: whole waves exit
  float v[8];
  uint32_t bad = 0;
  if (row < n) {
    if constexpr (sizeof(TIn) == 1) {
      const uint2 raw = *reinterpret_cast<const uint2*>(src + row * kDim + c * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (float)((raw.x >> (8 * j)) & 0xFF);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 + j] = (float)((raw.y >> (8 * j)) & 0xFF);
    } else {
      const float4 a = *reinterpret_cast<const float4*>(src + row * kDim + c * 8);
      const float4 b = *reinterpret_cast<const float4*>(src + row * kDim + c * 8 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // this file is compiled with -fno-honor-nans: reject NaN/Inf on the bit pattern
        const bool finite = (__float_as_uint(v[j]) & 0x7f800000u) != 0x7f800000u;
        const bool ok = finite && (v[j] >= 0.f) && (v[j] <= 255.f) && (v[j] == truncf(v[j]));
        bad |= ok ? 0u : 1u;
        if (!ok) v[j] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  float ss = 0.f;
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss += v[j] * v[j];  // integers, < 2^24: exact in any order
    o[j] = (__bf16)(v[j] * scale);
  }
  // the 16 chunks of one row are 16 consecutive lanes
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) ss += __shfl_xor(ss, m, 16);
  const int64_t sub = row >> 4;
  const int rr = (int)(row & 15);
  const int64_t off = sub * kSubBytes + (c >> 2) * 1024 + (rr + 16 * (c & 3)) * 16;
  *reinterpret_cast<bf16x8*>(pack + off) = o;
  if (c == 0) {
    norms[row] = (row < n) ? ss : padnorm;
    if (row < n) atomicMax(&flags[max_slot], __float_as_uint(ss));
  }
  if (bad) atomicAdd(&flags[0], 1u);
}

// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void merge2(float& v1, int& i1, float& v2, float o1, int oi, float o2) {
  // lexicographic (distance, trainIdx) on the best, plain min on the second
  if (o1 < v1 || (o1 == v1 && oi < i1)) {
    v2 = fminf(v1, o2);
    v1 = o1;
    i1 = oi;
  } else {
    v2 = fminf(v2, o1);
  }
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, uint8_t* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_base, 16, 0, 0);
}

// LDS-DMA ring: stage s lives in buffer s % 2.  The loads of stage s+1 are issued right
// after the barrier that opens stage s (which guarantees every wave finished reading stage
// s-1 from that buffer) and have the whole stage's MFMA work to land.
constexpr int kRing = 2;
constexpr int kStageSlot = kStageBytes + kStageNorm;   // 33280 B, a multiple of 16
constexpr int kPiecesPerWave = kStageBytes / 1024 / NW;
constexpr int kNormLanes = kStageNorm / 16 / NW;        // 16-B norm pieces per wave
static_assert(kStageBytes / 1024 % NW == 0, "fragment pieces split evenly over waves");
static_assert(kStageNorm % (16 * NW) == 0 && kNormLanes <= 64, "norm pieces split over waves");

__device__ __forceinline__ void issue_stage(const uint8_t* __restrict__ dbpack,
                                            const float* __restrict__ dn, int64_t sub0,
                                            uint8_t* slot, int wave, int lane) {
  const uint8_t* src = dbpack + sub0 * kSubBytes;
#pragma unroll
  for (int j = 0; j < kPiecesPerWave; ++j) {
    const int piece = wave * kPiecesPerWave + j;
    glds16(src + piece * 1024 + lane * 16, slot + piece * 1024);
  }
  const float* nsrc = dn + sub0 * kSubRows + wave * (kNormLanes * 4) + lane * 4;
  if (lane < kNormLanes) glds16(nsrc, slot + kStageBytes + wave * (kNormLanes * 16));
}

struct Frag {
  bf16x8 a0, a1, a2, a3;
  f32x4 cn;
};

__device__ __forceinline__ Frag read_frag(const uint8_t* sb, int u, int lane) {
  const uint8_t* base = sb + u * kSubBytes + lane * 16;
  Frag f;
  f.a0 = *reinterpret_cast<const bf16x8*>(base);
  f.a1 = *reinterpret_cast<const bf16x8*>(base + 1024);
  f.a2 = *reinterpret_cast<const bf16x8*>(base + 2048);
  f.a3 = *reinterpret_cast<const bf16x8*>(base + 3072);
  f.cn = *reinterpret_cast<const f32x4*>(sb + kStageBytes + u * 64 + (lane >> 4) * 16);
  return f;
}

// kFind = false: the k=2 search.  kFind = true: a row-finding pass for the BFMatcher.knnMatch
// drop-in -- the same pass over the DB, looking per query for the LOWEST row other than
// excl[q] whose exact squared distance lies in [flo[q], fhi[q]] (the integers whose sqrtf is
// one float distance; a single value when every distance is < 2048).  OpenCV's strict-'<'
// insertion keeps the lowest trainIdx among equal float distances, so that row is its
// trainIdx.  Rows are found per lane in increasing order, then min-merged over the lanes
// and (atomicMin) over the DB splits into found[q].
template <bool kFind>
__global__ __launch_bounds__(NT, 2) void match_kernel(
    const uint8_t* __restrict__ dbpack, const float* __restrict__ dn, int64_t nsub,
    const uint8_t* __restrict__ qpack, const float* __restrict__ qn, int nqt, int64_t nq_pad,
    int split, int64_t sub_per_split, int row_offset, float* __restrict__ pd1,
    int* __restrict__ pidx, float* __restrict__ pd2, const float* __restrict__ flo,
    const float* __restrict__ fhi, const int* __restrict__ excl, int* __restrict__ found) {
  // ONE __shared__ array (a second one can make hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRing * kStageSlot];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int sp = blockIdx.x % split;
  const int qb = blockIdx.x / split;
  const int qt0 = (qb * NW + wave) * QT;

  const int64_t s_lo = (int64_t)sp * sub_per_split;
  const int64_t s_hi = min(nsub, s_lo + sub_per_split);
  const int64_t nst = (s_hi - s_lo) / SPS;  // nsub and sub_per_split are multiples of SPS

  if (nst > 0) issue_stage(dbpack, dn, s_lo, lds, wave, lane);

  // queries: B fragments stay in registers for the whole launch
  bf16x8 bq[QT][4];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int qt = qt0 + t;
      if (qt < nqt)
        bq[t][k] = *reinterpret_cast<const bf16x8*>(qpack + ((int64_t)qt * 4 + k) * 1024 + lane * 16);
      else
        bq[t][k] = bf16x8{};
    }
  }
  float v1[QT], v2[QT];
  int id[QT];
  float vh[kFind ? QT : 1];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    v1[t] = kInit;
    v2[t] = kInit;
    id[t] = 0x7fffffff;
    if constexpr (kFind) {   // [v2, vh] = the target interval in dn - 2 q.d units, v1 = excl
      const int qt = qt0 + t;
      const int64_t q = (int64_t)qt * 16 + (lane & 15);
      vh[t] = -kInit;
      if (qt < nqt && flo[q] <= fhi[q]) {   // an empty interval: nothing to find
        v2[t] = flo[q] - qn[q];             // integers < 2^24: exact
        vh[t] = fhi[q] - qn[q];
        v1[t] = __int_as_float(excl[q]);
      }
    }
  }

  for (int64_t s = 0; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's part of stage s landed
    __builtin_amdgcn_s_barrier();                       // every wave's; stage s-1 fully read
    uint8_t* nxt = lds + ((s + 1) & 1) * kStageSlot;
    if (s + 1 < nst) issue_stage(dbpack, dn, s_lo + (s + 1) * SPS, nxt, wave, lane);
    const uint8_t* sb = lds + (s & 1) * kStageSlot;
#if SOD_MATCH_PREFETCH
    Frag f = read_frag(sb, 0, lane);
#endif
#pragma unroll
    for (int u = 0; u < SPS; ++u) {
#if SOD_MATCH_PREFETCH
      const Frag c = f;
#else
      const Frag c = read_frag(sb, u, lane);
#endif
      f32x4 acc[QT];
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c.a0, bq[t][0], c.cn, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c.a1, bq[t][1], acc[t], 0, 0, 0);
      // next subtile's fragments in flight once a0/a1/cn are dead (keeps VGPRs < 256)
#if SOD_MATCH_PREFETCH
      if (u + 1 < SPS) f = read_frag(sb, u + 1, lane);
#endif
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c.a2, bq[t][2], acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c.a3, bq[t][3], acc[t], 0, 0, 0);
      if constexpr (kFind) {
        bool any = false;
#pragma unroll
        for (int t = 0; t < QT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) any |= (acc[t][r] >= v2[t]) & (acc[t][r] <= vh[t]);
        if (__any(any)) {
          const int rowb = row_offset + (int)((s_lo + s * SPS + u) * kSubRows) + (lane >> 4) * 4;
#pragma unroll
          for (int t = 0; t < QT; ++t) {
#pragma unroll
            for (int r = 3; r >= 0; --r) {   // the lowest matching row of the four wins
              const bool in = (acc[t][r] >= v2[t]) && (acc[t][r] <= vh[t]) &&
                              (rowb + r != __float_as_int(v1[t]));
              id[t] = (in && rowb + r < id[t]) ? rowb + r : id[t];
            }
          }
        }
        continue;
      }
      // prefilter: can any of this lane's 4 x QT candidates beat its running 2nd best?
      bool hit[QT];
      bool any = false;
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        const float m = fminf(fminf(acc[t][0], acc[t][1]), acc[t][2]);
        hit[t] = (m < v2[t]) | (acc[t][3] < v2[t]);
        any |= hit[t];
      }
      if (__any(any)) {
        const int rowb = row_offset + (int)((s_lo + s * SPS + u) * kSubRows) + (lane >> 4) * 4;
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          if (__any(hit[t])) {       // exact top-2 update, only for tiles that can change
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float x = acc[t][r];
              const bool lt = x < v1[t];
              v2[t] = __builtin_amdgcn_fmed3f(v1[t], v2[t], x);
              id[t] = lt ? rowb + r : id[t];
              v1[t] = lt ? x : v1[t];
            }
          }
        }
      }
    }
  }

  if constexpr (kFind) {
#pragma unroll
    for (int t = 0; t < QT; ++t) {
#pragma unroll
      for (int m = 16; m <= 32; m <<= 1) id[t] = min(id[t], __shfl_xor(id[t], m));
      const int qt = qt0 + t;
      if (lane < 16 && qt < nqt && id[t] != 0x7fffffff)
        atomicMin(&found[(int64_t)qt * 16 + lane], id[t]);
    }
    return;
  }
  // merge the 4 row groups of each query (lanes l, l^16, l^32, l^48)
#pragma unroll
  for (int t = 0; t < QT; ++t) {
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      const float o1 = __shfl_xor(v1[t], m);
      const int oi = __shfl_xor(id[t], m);
      const float o2 = __shfl_xor(v2[t], m);
      merge2(v1[t], id[t], v2[t], o1, oi, o2);
    }
    const int qt = qt0 + t;
    if (lane < 16 && qt < nqt) {
      const int64_t q = (int64_t)qt * 16 + lane;
      const float n2 = qn[q];
      const int64_t o = (int64_t)sp * nq_pad + q;
      pd1[o] = v1[t] + n2;
      pidx[o] = id[t];
      pd2[o] = v2[t] + n2;
    }
  }
}

// Correctly rounded sqrt of an exact integer-valued float n >= 0 (OpenCV: std::sqrt on
// the float sum).  The hardware estimate is within an ulp; it is then corrected with the
// exact midpoint test: a midpoint m of two adjacent floats has <= 25 significant bits, so
// m*m is exact in f64 and compares exactly with n (ties -> even).
__device__ __forceinline__ float sqrt_rn_exact(float n) {
#pragma clang fp contract(off)
  float s = sqrtf(n);
  const double dn = (double)n;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const float up = __uint_as_float(__float_as_uint(s) + 1u);   // s >= 0, finite
    const double mh = 0.5 * ((double)s + (double)up);
    const double h2 = mh * mh;
    if (h2 < dn || (h2 == dn && (__float_as_uint(up) & 1u) == 0u)) {
      s = up;
      continue;
    }
    const float lo = s > 0.0f ? __uint_as_float(__float_as_uint(s) - 1u) : s;
    const double ml = 0.5 * ((double)s + (double)lo);
    const double l2 = ml * ml;
    if (lo != s && (l2 > dn || (l2 == dn && (__float_as_uint(lo) & 1u) == 0u))) {
      s = lo;
      continue;
    }
    break;
  }
  return s;
}

__global__ void ratio_kernel(const float* __restrict__ cd1, const int* __restrict__ cidx,
                             const float* __restrict__ cd2, int64_t nq, double ratio,
                             float* __restrict__ d1, float* __restrict__ d2,
                             int* __restrict__ idx1, uint8_t* __restrict__ good) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const float a = sqrt_rn_exact(cd1[q]);   // OpenCV: std::sqrt(float) of the exact sum
  const float b = sqrt_rn_exact(cd2[q]);
  d1[q] = a;
  d2[q] = b;
  idx1[q] = cidx[q];
  good[q] = ((double)a < ratio * (double)b) ? 1 : 0;   // main.py:82, Python floats
}

// per query: the partial top-2 of every DB chunk (or rank) merged; when this is the final
// merge of a pipeline call (one rank, or the global merge after the all-gather) and ratio >=
// 0, the ratio test of ratio_kernel is applied in the same pass (one launch fewer).
// A work-group covers 64 queries (one per lane) with kMergeW waves, wave w merging parts
// w, w + W, ... (their loads issued 8 at a time, independent of the merges), then the W
// partial results through LDS: the top-2 merge of disjoint row sets is associative and
// commutative (lexicographic (d^2, trainIdx) on the best, plain min on the second), so any
// grouping gives the sequential result bit for bit -- and hundreds of DB chunks (one query
// image over a large DB) cost a few dependent loads per lane instead of one per chunk.
constexpr int kMergeW = 16;
__global__ __launch_bounds__(64 * kMergeW) void merge_kernel(
    const float* __restrict__ d1, const int* __restrict__ idx, const float* __restrict__ d2,
    int nparts, int64_t stride, int64_t nq, float* __restrict__ od1, int* __restrict__ oidx,
    float* __restrict__ od2, int* __restrict__ reset, int reset_words, double ratio, int64_t nq_real,
    float* __restrict__ rd1, float* __restrict__ rd2, int* __restrict__ ridx,
    uint8_t* __restrict__ rgood) {
  __shared__ float s1[kMergeW][64], s2[kMergeW][64];
  __shared__ int si[kMergeW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = min((int)(blockDim.x >> 6), nparts);
  const int64_t q = (int64_t)blockIdx.x * 64 + lane;
  float v1 = 3.0e38f, v2 = 3.0e38f;
  int i1 = 0x7fffffff;
  if (q < nq && w < nw) {
    v1 = d1[(int64_t)w * stride + q];   // the wave's first part as is (as the sequential merge)
    i1 = idx[(int64_t)w * stride + q];
    v2 = d2[(int64_t)w * stride + q];
    int p = w + nw;
    for (; p + 7 * nw < nparts; p += 8 * nw) {   // 8 parts' loads in flight
      float a1[8], a2[8];
      int ai[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t o = (int64_t)(p + k * nw) * stride + q;
        a1[k] = d1[o];
        ai[k] = idx[o];
        a2[k] = d2[o];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) merge2(v1, i1, v2, a1[k], ai[k], a2[k]);
    }
    for (; p < nparts; p += nw) {
      const int64_t o = (int64_t)p * stride + q;
      merge2(v1, i1, v2, d1[o], idx[o], d2[o]);
    }
  }
  if (nw > 1) {
    s1[w][lane] = v1;
    si[w][lane] = i1;
    s2[w][lane] = v2;
    __syncthreads();
    if (w != 0) return;
    for (int k = 1; k < nw; ++k) merge2(v1, i1, v2, s1[k][lane], si[k][lane], s2[k][lane]);
  } else if (w != 0) {
    return;
  }
  if (q >= nq) return;
  // the matcher's shared thresholds of this partial-result slot: "nothing known" again for
  // the next launch that takes the slot (it waits for this merge)
  if (reset)
    for (int r = 0; r < reset_words; ++r) reset[(int64_t)r * nq + q] = (int)0x80808080;
  od1[q] = v1;
  oidx[q] = i1;
  od2[q] = v2;
  if (ratio >= 0.0 && q < nq_real) {
    const float a = sqrt_rn_exact(v1), b = sqrt_rn_exact(v2);
    rd1[q] = a;
    rd2[q] = b;
    ridx[q] = i1;
    rgood[q] = ((double)a < ratio * (double)b) ? 1 : 0;   // main.py:82, Python floats
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------
static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

int launch_pack_db(sod_ctx* ctx, const void* dsrc, int dtype, int64_t n) {
  const int64_t npad = ceil_div(n, SPS * kSubRows) * SPS * kSubRows;
  ctx->nsub = npad / kSubRows;
  SOD_TRY(sod_reserve(ctx, ctx->dbpack, (size_t)ctx->nsub * kSubBytes));
  SOD_TRY(sod_reserve(ctx, ctx->dn, (size_t)npad));
  const int64_t threads = npad * 16;
  const int bs = 256;
  const int64_t grid = ceil_div(threads, bs);
  if (dtype == SOD_DTYPE_U8)
    hipLaunchKernelGGL(pack_rows_kernel<uint8_t>, dim3((unsigned)grid), dim3(bs), 0, ctx->stream,
                       (const uint8_t*)dsrc, n, npad, -2.0f, ctx->dbpack.p, ctx->dn.p, kPadNorm,
                       ctx->flags.p, 1);
  else
    hipLaunchKernelGGL(pack_rows_kernel<float>, dim3((unsigned)grid), dim3(bs), 0, ctx->stream,
                       (const float*)dsrc, n, npad, -2.0f, ctx->dbpack.p, ctx->dn.p, kPadNorm,
                       ctx->flags.p, 1);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_pack_queries(sod_ctx* ctx, const void* dsrc, int dtype, int32_t nq) {
  const int64_t npad = ceil_div(nq, kSubRows) * kSubRows;
  ctx->nqt = (int32_t)(npad / kSubRows);
  SOD_TRY(sod_reserve(ctx, ctx->qpack, (size_t)ctx->nqt * kSubBytes));
  SOD_TRY(sod_reserve(ctx, ctx->qn, (size_t)npad));
  const int64_t threads = npad * 16;
  const int bs = 256;
  const int64_t grid = ceil_div(threads, bs);
  if (dtype == SOD_DTYPE_U8)
    hipLaunchKernelGGL(pack_rows_kernel<uint8_t>, dim3((unsigned)grid), dim3(bs), 0, ctx->stream,
                       (const uint8_t*)dsrc, (int64_t)nq, npad, 1.0f, ctx->qpack.p, ctx->qn.p, 0.0f,
                       ctx->flags.p, 2);
  else
    hipLaunchKernelGGL(pack_rows_kernel<float>, dim3((unsigned)grid), dim3(bs), 0, ctx->stream,
                       (const float*)dsrc, (int64_t)nq, npad, 1.0f, ctx->qpack.p, ctx->qn.p, 0.0f,
                       ctx->flags.p, 2);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_match(sod_ctx* ctx) {
  const int64_t nq_pad = (int64_t)ctx->nqt * kSubRows;
  const int qtiles_per_wg = NW * QT;
  const int64_t qblocks = ceil_div(ctx->nqt, qtiles_per_wg);
  const int64_t nstages = ctx->nsub / SPS;
  // fill every CU twice (2 workgroups of 4 waves per CU); each split >= 1 stage
  int64_t target = 2LL * ctx->match_cus();
  // (rounded down: one work-group more than the slots would run as a second round)
  int64_t split = std::max<int64_t>(1, target / qblocks);
  split = std::min<int64_t>(split, nstages);
  const int64_t st_per_split = ceil_div(nstages, split);
  split = ceil_div(nstages, st_per_split);
  ctx->split = (int)split;
  SOD_TRY(sod_reserve(ctx, ctx->cd1, (size_t)nq_pad));
  SOD_TRY(sod_reserve(ctx, ctx->cd2, (size_t)nq_pad));
  SOD_TRY(sod_reserve(ctx, ctx->cidx, (size_t)nq_pad));
  const int64_t grid = qblocks * split;
  hipStream_t ks;   // context stream, or the matcher's (sod_match_set_overlap)
  float *pd1, *pd2;
  int32_t* pidx;
  SOD_TRY(sod_match_stream_begin(ctx, split * nq_pad, &ks, &pd1, &pidx, &pd2));
  SOD_TRY(sod_match_mark(ctx, ks, 0));
  hipLaunchKernelGGL(match_kernel<false>, dim3((unsigned)grid), dim3(NT), 0, ks,
                     ctx->dbpack.p, ctx->dn.p, ctx->nsub, ctx->qpack.p, ctx->qn.p, ctx->nqt,
                     nq_pad, (int)split, st_per_split * SPS, (int)ctx->row_offset, pd1, pidx, pd2,
                     nullptr, nullptr, nullptr, nullptr);
  SOD_HIP(ctx, hipGetLastError());
  SOD_TRY(sod_match_mark(ctx, ks, 1));
  SOD_TRY(sod_match_stream_end(ctx));
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, false));
  SOD_TRY(launch_merge(ctx, pd1, pidx, pd2, (int)split, nq_pad, nullptr,
                       ctx->nranks <= 1 && !ctx->comm));
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, true));
  return sod_partials_merged(ctx);   // the slot is free again
}

// per query the lowest row other than excl[q] whose exact squared distance lies in
// [flo[q], fhi[q]] (kFind pass over the bf16-packed DB; all four arrays on the device,
// [nq_pad]); found[q] = 0x7f7f7f7f where there is none
int launch_find_rows(sod_ctx* ctx, const float* flo, const float* fhi, const int32_t* excl,
                     int32_t* found) {
  const int64_t nq_pad = (int64_t)ctx->nqt * kSubRows;
  const int64_t qblocks = ceil_div(ctx->nqt, NW * QT);
  const int64_t nstages = ctx->nsub / SPS;
  int64_t split = std::max<int64_t>(1, 2LL * ctx->match_cus() / qblocks);
  split = std::min<int64_t>(split, nstages);
  const int64_t st_per_split = ceil_div(nstages, split);
  split = ceil_div(nstages, st_per_split);
  SOD_HIP(ctx, hipMemsetAsync(found, 0x7f, (size_t)nq_pad * 4, ctx->stream));
  hipLaunchKernelGGL(match_kernel<true>, dim3((unsigned)(qblocks * split)), dim3(NT), 0,
                     ctx->stream, ctx->dbpack.p, ctx->dn.p, ctx->nsub, ctx->qpack.p, ctx->qn.p,
                     ctx->nqt, nq_pad, (int)split, st_per_split * SPS, (int)ctx->row_offset,
                     nullptr, nullptr, nullptr, flo, fhi, excl, found);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_merge(sod_ctx* ctx, const float* d1, const int32_t* idx, const float* d2, int nparts,
                 int64_t stride, int32_t* reset, bool final_merge) {
  const int64_t nq_pad = sod_nq_pad(ctx);
  // sod_pipeline_enqueue announces its ratio: the final merge applies it as well
  const bool fuse = final_merge && ctx->fuse_ratio >= 0.0;
  if (fuse) {
    SOD_TRY(sod_reserve(ctx, ctx->d1, (size_t)ctx->nq));
    SOD_TRY(sod_reserve(ctx, ctx->d2, (size_t)ctx->nq));
    SOD_TRY(sod_reserve(ctx, ctx->idx1, (size_t)ctx->nq));
    SOD_TRY(sod_reserve(ctx, ctx->good, (size_t)ctx->nq));
  }
  // waves per 64 queries: one per part up to kMergeW (a few parts: one wave, no LDS step)
  const int wv = std::max(1, std::min(kMergeW, nparts));
  hipLaunchKernelGGL(merge_kernel, dim3((unsigned)ceil_div(nq_pad, 64)), dim3(64 * wv), 0,
                     ctx->stream, d1, idx, d2, nparts, stride, nq_pad, ctx->cd1.p, ctx->cidx.p,
                     ctx->cd2.p, reset, (int)sod_thr_words(ctx), fuse ? ctx->fuse_ratio : -1.0,
                     (int64_t)ctx->nq, ctx->d1.p,
                     ctx->d2.p, ctx->idx1.p, ctx->good.p);
  ctx->ratio_fused_valid = fuse;
  if (fuse) ctx->ratio_fused = ctx->fuse_ratio;
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_ratio(sod_ctx* ctx, double ratio) {
  SOD_TRY(sod_reserve(ctx, ctx->d1, (size_t)ctx->nq));
  SOD_TRY(sod_reserve(ctx, ctx->d2, (size_t)ctx->nq));
  SOD_TRY(sod_reserve(ctx, ctx->idx1, (size_t)ctx->nq));
  SOD_TRY(sod_reserve(ctx, ctx->good, (size_t)ctx->nq));
  const int bs = 256;
  hipLaunchKernelGGL(ratio_kernel, dim3((unsigned)ceil_div(ctx->nq, bs)), dim3(bs), 0, ctx->stream,
                     ctx->cd1.p, ctx->cidx.p, ctx->cd2.p, (int64_t)ctx->nq, ratio, ctx->d1.p,
                     ctx->d2.p, ctx->idx1.p, ctx->good.p);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}
