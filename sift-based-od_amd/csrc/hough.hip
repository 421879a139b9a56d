// hough.hip -- generalized-Hough pose voting, valid-bin selection, PoseBin means and the
// per-bin affine verification, for gfx950.
//
// Compiled with -ffp-contract=off: every f64 expression below is evaluated exactly as the
// reference's Python floats are (one rounding per operation, no FMA), so bin indices are
// bit-exact.  Reference: HoughTransformHelperFunctions.py:4-72, main.py:89-157,
// PoseBin.py:6-51, AffineParameters.py:89-160, SiftHelperFunctions.py:25-40.
//
// Data flow (all device resident, one stream, no host round trip):
//   pose_kernel      per query q with a good match: pose (x,y,alpha,s) f64, base bin
//                    (ix,iy,it,is) packed in a u32, 16-bit mask of the in-range votes
//   hist_kernel      LDS-privatised histogram over a slab of bins: counts + first-touch
//                    ordinal (q*16 + slot = dict insertion order), flushed with integer
//                    atomics (deterministic)
//   select_kernel    votes that are the first touch of a bin with >= thr votes, compacted
//                    in ordinal order = dict insertion order of main.py:126 (one pass,
//                    decoupled look-back)
//   member_fill      wave-aggregated slot reservation: per vote slot, one atomic per distinct
//                    bin among a wave's lanes reserves a run in the bin's member list
//   member_order     query order per bin: <= 256 members sorted in one wave's registers,
//                    larger bins through an LDS bitmap of their query range
//   members_kernel   fallback for ranges beyond the bitmap (nq > 512 Ki): one wave scans
//   means_kernel     PoseBin running means, sequential per bin (PoseBin.py:19-43), its
//                    members' inputs gathered a batch ahead
//   affine_kernel    one wave per bin: decoupled 3x3 normal equations, pinv by Jacobi,
//                    outlier rejection, fixed point (AffineParameters.py:89-160)
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <utility>

#include <hip/hip_ext.h>

#include "glibc_trig.h"
#include "sod_internal.h"

namespace {

constexpr double kPi = 3.141592653589793;        // Py_MATH_PI
constexpr double kDeg2Rad = kPi / 180.0;         // math.radians factor (CPython degToRad)
constexpr double kTwoPi = 2 * kPi;

struct Bins {
  int x, y, t, s;
};

__device__ __forceinline__ int unpack_octave(int packed) {  // SiftHelperFunctions.py:31-35
  int o = packed & 0xFF;
  return o >= 128 ? o - 256 : o;
}

// Python int() of a float that is then clamped to [0, b-1] after a -1 (HTHF:49-58).
__host__ __device__ __forceinline__ int xy_index(double v, int b) {
  long long i;
  if (!(v == v)) i = 0;                 // NaN: unreachable for finite inputs
  else if (v > 1e9) i = 1000000000LL;
  else if (v < -1e9) i = -1000000000LL;
  else i = (long long)v;                // truncation toward zero == Python int()
  i = i - 1;
  if (i < 0) i = 0;
  if (i > b - 1) i = b - 1;
  return (int)i;
}

// calculate_bin_index (HTHF:39-72) of a pose (x, y, alpha, scale_factor = 2^k)
__device__ __forceinline__ void bin_index(double x, double y, double a, int k, int H, int W,
                                          Bins b, const int* __restrict__ lut, int idx[4]) {
  idx[0] = xy_index((x * b.x) / W, b.x);
  idx[1] = xy_index((y * b.y) / H, b.y);
  idx[2] = (int)fmod((a * b.t) / kTwoPi, (double)b.t);
  idx[3] = lut[k + kSigmaLutHalf];
}

// estimate_object_pose (HTHF:4-37) + calculate_bin_index (HTHF:39-72); t = the translation
// (tx, ty) the rotation acts on, for the boundary guard below
// the pose's terms before the rotation (HTHF:20-30): scale exponent k, s = 2^k, the
// translation (tx, ty) the rotation acts on, the angle a in [0, 2 pi)
__device__ __forceinline__ void pose_terms(float mx, float my, float ma, int mo, float qa, int qo,
                                           double cx, double cy, int& k, double& s, double& tx,
                                           double& ty, double& a) {
  k = unpack_octave(qo) - unpack_octave(mo);  // m_scale / q_scale = 2^(oQ-oM), exact
  s = ldexp(1.0, k);
  tx = (cx - (double)mx) * s;
  ty = (cy - (double)my) * s;
  a = ((double)qa - (double)ma) * kDeg2Rad;
  a = fmod(a + kTwoPi, kTwoPi);   // argument > 0, so Python % == C fmod
}

__device__ __forceinline__ void pose_bins(float mx, float my, float ma, int mo, float qx, float qy,
                                          float qa, int qo, double cx, double cy, int H, int W,
                                          Bins b, const int* __restrict__ lut, double pose[4],
                                          int idx[4], double t[2]) {
  int k;
  double s, tx, ty, a;
  pose_terms(mx, my, ma, mo, qa, qo, cx, cy, k, s, tx, ty, a);
  // glibc's cos / sin bit for bit (glibc_trig.h): math.cos / math.sin of HTHF:31-32
  const double ca = gtrig::cos(a), sa = gtrig::sin(a);
  const double x = (ca * tx - sa * ty) + (double)qx;
  const double y = (sa * tx + ca * ty) + (double)qy;
  pose[0] = x;
  pose[1] = y;
  pose[2] = a;
  pose[3] = s;
  t[0] = tx;
  t[1] = ty;
  bin_index(x, y, a, k, H, W, b, lut, idx);
}

// ---- boundary guard (SURVEY 7 "Hough parity") -------------------------------------------
// Round 5: the device's cos / sin are glibc's x86_64 FMA variant bit for bit (glibc_trig.h),
// so every pose is the reference's and the guard is armed only when the host's libm is a
// different variant (sod_trig_exact() == 0: a CPU without FMA / AVX2), whose last bits the
// reference there follows; the launchers then pass the record buffer, else nullptr.
// Every step of the pose is one correctly rounded IEEE operation, the same on both sides,
// except cos/sin: the device's and glibc's (math.cos / math.sin of the reference,
// HTHF:31-32) may round differently by an ulp or two.  The x / y bin indices are then still
// exact unless v = (x*b)/W lies within that error of an integer where int(v)-1 clamped to
// [0, b-1] (HTHF:49-58) steps -- 2..b.  Such matches are listed (guard records) and done
// again on the host with glibc (guard_resolve in api.hip), so bin counts are exact by
// construction.  Error bound: with trig off by <= 4 ulp, |dx| <= 2e-15 (|tx|+|ty|+|qx|+|x|);
// the tolerance below is 50x that in units of v.  theta and sigma use no transcendental
// (theta: exact fmod; sigma: the LUT).
constexpr int kGuardRec = 8;    // doubles per record: q, tx, ty, alpha, qx, qy, H, W

__device__ __forceinline__ bool near_edge(double v, int b, double mag) {
  const double n = rint(v);
  if (!(n >= 2.0 && n <= (double)b)) return false;   // NaN / inf / clamped: no step
  return fabs(v - n) <= 1e-13 * (mag + fabs(v) + 1.0);
}

__device__ __forceinline__ bool guard_flag(const double p[4], const double t[2], double qx,
                                           double qy, int H, int W, Bins b) {
  const double ax = fabs(t[0]) + fabs(t[1]);
  return near_edge((p[0] * b.x) / W, b.x, (ax + fabs(qx) + fabs(p[0])) * b.x / W) ||
         near_edge((p[1] * b.y) / H, b.y, (ax + fabs(qy) + fabs(p[1])) * b.y / H);
}

__device__ __forceinline__ void guard_push(double* __restrict__ rec, uint32_t* __restrict__ n,
                                           int64_t q, const double p[4], const double t[2],
                                           double qx, double qy, int H, int W) {
  const uint32_t i = atomicAdd(n, 1u);   // capacity = queries: every query fits
  double* r = rec + (int64_t)kGuardRec * i;
  r[0] = (double)q;
  r[1] = t[0];
  r[2] = t[1];
  r[3] = p[2];
  r[4] = qx;
  r[5] = qy;
  r[6] = (double)H;
  r[7] = (double)W;
}

// scale_factor -> k with s == 2^k exactly (estimate_object_pose only produces powers of 2);
// any other scale takes the generic path of HTHF:67 (log2 via libm-equivalent ocml log).
__device__ __forceinline__ int sigma_from_scale(double s, Bins b, const int* lut, bool* generic) {
  int e;
  const double m = frexp(s, &e);          // s = m * 2^e, m in [0.5, 1)
  if (m == 0.5 && e - 1 >= -kSigmaLutHalf && e - 1 <= kSigmaLutHalf) {
    *generic = false;
    return e - 1;
  }
  *generic = true;
  return 0;
}

// main.py:105-110: 16 votes (w, x, y, z in {0,1}, lexicographic), kept when every index is
// < bins (no theta wrap)
__device__ __forceinline__ uint32_t vote_mask(const int ix[4], Bins b) {
  uint32_t mask = 0;
#pragma unroll
  for (int slot = 0; slot < 16; ++slot) {
    const int w = (slot >> 3) & 1, x = (slot >> 2) & 1, y = (slot >> 1) & 1, z = slot & 1;
    if (ix[0] + w < b.x && ix[1] + x < b.y && ix[2] + y < b.t && ix[3] + z < b.s)
      mask |= 1u << slot;
  }
  return mask;
}

__device__ __forceinline__ uint32_t lin_bin(int ix, int iy, int it, int is, Bins b) {
  return (uint32_t)(((ix * b.y + iy) * b.t + it) * b.s + is);
}

__global__ void pose_kernel(int64_t nq, const uint8_t* __restrict__ good,
                            const int* __restrict__ idx1, const float* __restrict__ qx,
                            const float* __restrict__ qy, const float* __restrict__ qa,
                            const int* __restrict__ qo, const float* __restrict__ mx,
                            const float* __restrict__ my, const float* __restrict__ ma,
                            const int* __restrict__ mo, const int* __restrict__ mimg,
                            const double* __restrict__ cent, int H, int W,
                            const int* __restrict__ qimg, const int* __restrict__ qshape, Bins b,
                            const int* __restrict__ lut, int64_t own_lo, int64_t own_hi,
                            double* __restrict__ pose, uint32_t* __restrict__ basekey,
                            uint32_t* __restrict__ vmask, int64_t nbins,
                            uint32_t* __restrict__ counts, uint32_t* __restrict__ first,
                            const int* __restrict__ isize, int2* __restrict__ msize,
                            double* __restrict__ grec, uint32_t* __restrict__ gstat) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the histogram the next kernel fills starts empty: count 0, first touch "none" (folded
  // in here instead of two memset launches on the tail's critical path)
  for (int64_t b2 = q; b2 < nbins; b2 += (int64_t)gridDim.x * blockDim.x) {
    counts[b2] = 0u;
    first[b2] = 0xFFFFFFFFu;
  }
  if (q >= nq) return;
  if (qimg) {   // batch of query images: this query's image shape (main.py:102)
    H = qshape[2 * qimg[q]];
    W = qshape[2 * qimg[q] + 1];
  }
  if (!good[q]) {
    vmask[q] = 0;
    return;
  }
  const int m = idx1[q];
  const int im = mimg[m];
  double p[4], t[2];
  int ix[4];
  const float fqx = qx[q], fqy = qy[q];
  pose_bins(mx[m], my[m], ma[m], mo[m], fqx, fqy, qa[q], qo[q], cent[2 * im], cent[2 * im + 1],
            H, W, b, lut, p, ix, t);
  if (grec && guard_flag(p, t, fqx, fqy, H, W, b)) guard_push(grec, gstat, q, p, t, fqx, fqy, H, W);
  pose[4 * q + 0] = p[0];
  pose[4 * q + 1] = p[1];
  pose[4 * q + 2] = p[2];
  pose[4 * q + 3] = p[3];
  msize[q] = make_int2(isize[2 * im], isize[2 * im + 1]);   // PoseBin img_size input
  basekey[q] = (uint32_t)ix[0] | ((uint32_t)ix[1] << 8) | ((uint32_t)ix[2] << 16) |
               ((uint32_t)ix[3] << 24);
  const bool own = (m >= own_lo) && (m < own_hi);
  vmask[q] = vote_mask(ix, b) | (own ? 0x10000u : 0u);
}

// guard fix-up (api.hip guard_resolve): the host's (glibc) x, y and base key for the listed
// queries; their vote masks follow the new keys and keep the shard bit
__global__ void guard_patch_kernel(int n, const int32_t* __restrict__ pq,
                                   const uint32_t* __restrict__ pkey, const double* __restrict__ pxy,
                                   Bins b, uint32_t* __restrict__ basekey,
                                   uint32_t* __restrict__ vmask, double* __restrict__ pose) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t q = pq[i];
  const uint32_t key = pkey[i];
  const int ix[4] = {(int)(key & 0xFF), (int)((key >> 8) & 0xFF), (int)((key >> 16) & 0xFF),
                     (int)(key >> 24)};
  basekey[q] = key;
  vmask[q] = vote_mask(ix, b) | (vmask[q] & 0x10000u);
  pose[4 * q + 0] = pxy[2 * i];
  pose[4 * q + 1] = pxy[2 * i + 1];
}

// the re-done histogram holds every rank's votes (the all-reduce is not repeated): every
// voting query counts here
__global__ void own_all_kernel(int64_t nq, uint32_t* __restrict__ vmask) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
       q += (int64_t)gridDim.x * blockDim.x)
    if (vmask[q] & 0xFFFFu) vmask[q] |= 0x10000u;
}

__global__ void pose_batch_kernel(int64_t n, const float* __restrict__ mx,
                                  const float* __restrict__ my, const float* __restrict__ ma,
                                  const int* __restrict__ mo, const float* __restrict__ qx,
                                  const float* __restrict__ qy, const float* __restrict__ qa,
                                  const int* __restrict__ qo, const double* __restrict__ cx,
                                  const double* __restrict__ cy, int H, int W, Bins b,
                                  const int* __restrict__ lut, double* __restrict__ pose,
                                  int* __restrict__ idx, double* __restrict__ grec,
                                  uint32_t* __restrict__ gstat) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double p[4], t[2];
  int ix[4];
  pose_bins(mx[i], my[i], ma[i], mo[i], qx[i], qy[i], qa[i], qo[i], cx[i], cy[i], H, W, b, lut, p,
            ix, t);
  if (grec && guard_flag(p, t, qx[i], qy[i], H, W, b)) guard_push(grec, gstat, i, p, t, qx[i], qy[i], H, W);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pose[4 * i + j] = p[j];
    idx[4 * i + j] = ix[j];
  }
}

__global__ void bin_index_batch_kernel(int64_t n, const double* __restrict__ pose, int H, int W,
                                       Bins b, const int* __restrict__ lut, int* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* p = pose + 4 * i;
  bool generic;
  const int k = sigma_from_scale(p[3], b, lut, &generic);
  int ix[4];
  bin_index(p[0], p[1], p[2], k, H, W, b, lut, ix);
  if (generic) {  // HTHF:67 for a scale that is not a power of two
    const double v = (log(p[3]) / log(2.0)) / 6.5 * (double)b.s;
    long long i3 = !(v == v) ? 0 : (v > 1e9 ? 1000000000LL : (v < -1e9 ? -1000000000LL : (long long)v));
    ix[3] = (int)(i3 < 0 ? 0 : (i3 > b.s - 1 ? b.s - 1 : i3));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) idx[4 * i + j] = ix[j];
}

// ---------------------------------------------------------------------------------------
// LDS-privatised histogram.  blockIdx.x = bin slab, blockIdx.y = query chunk.  A query's 16
// votes lie in a window of lin_bin(1,1,1,1) bins above its base bin, so a work-group first
// lists the voting queries of its chunk whose window meets its slab (an LDS list, one atomic
// per wave) and then votes only those: ~1/slabs of the chunk instead of every query, which
// cuts the issued LDS atomics (each executed for a wave's in-slab lanes only) by that factor.
constexpr int kSlab = 8192;     // bins per workgroup
constexpr int kChunk = 8192;    // queries per workgroup
constexpr int kHistThreads = 1024;

__global__ __launch_bounds__(kHistThreads) void hist_kernel(
    int64_t nq, const uint32_t* __restrict__ basekey, const uint32_t* __restrict__ vmask, Bins b,
    int64_t nbins, const int* __restrict__ qimg, int64_t nbins1, const int* __restrict__ rng,
    uint32_t* __restrict__ gcount, uint32_t* __restrict__ gfirst, uint32_t* __restrict__ gstat) {
  // the guard records pose_kernel listed: their count moves to the slot the host reads, and
  // the append counter starts the next launch at 0 (stream order: pose_kernel is done)
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    gstat[1] = gstat[0];
    gstat[0] = 0u;
  }
  // 64 KiB: two work-groups per CU
  __shared__ uint32_t cnt2[kSlab / 2];     // two u16 counts per word (<= kChunk votes per bin)
  __shared__ uint32_t fst[kSlab];
  __shared__ unsigned short lst[kChunk];   // chunk-relative queries voting into the slab
  __shared__ uint32_t nlst;
  // batch of query images: a chunk only visits the slabs of its images' bin ranges
  const int64_t slab = rng ? (int64_t)rng[2 * blockIdx.y] + blockIdx.x : blockIdx.x;
  if (rng && slab > rng[2 * blockIdx.y + 1]) return;
  const uint32_t slab0 = (uint32_t)(slab * kSlab);
  for (int i = threadIdx.x; i < kSlab; i += kHistThreads) {
    if (i < kSlab / 2) cnt2[i] = 0;
    fst[i] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) nlst = 0;
  __syncthreads();
  const int64_t q0 = (int64_t)blockIdx.y * kChunk;
  const int64_t q1 = min(nq, q0 + kChunk);
  const int64_t span = (int64_t)lin_bin(1, 1, 1, 1, b);
  const int lane = threadIdx.x & 63;
  // all of a thread's queries are loaded before any is listed: one memory latency per
  // work-group instead of one per query (the kernel is latency-bound on a CU split's few
  // reserved CUs)
  // (unconditional loads from clamped indices: a load under a branch gets a vmcnt(0) at the
  // branch's join, i.e. one round trip per load)
  constexpr int kPer = kChunk / kHistThreads;
  uint32_t mv[kPer], kv[kPer], bv[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t q = q0 + threadIdx.x + (int64_t)u * kHistThreads;
    const int64_t qc = q < q1 ? q : q0;
    mv[u] = vmask[qc];
    kv[u] = basekey[qc];
    bv[u] = qimg ? (uint32_t)qimg[qc] : 0u;
    if (q >= q1) mv[u] = 0u;
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) bv[u] = (mv[u] & 0x10000u) ? bv[u] * (uint32_t)nbins1 : 0u;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    bool hit = false;
    // no vote, or the match's DB row is not in this shard: not listed
    if ((mv[u] & 0xFFFFu) && (mv[u] & 0x10000u)) {
      const uint32_t key = kv[u];
      const int64_t lo = (int64_t)bv[u] +
                         lin_bin(key & 0xFF, (key >> 8) & 0xFF, (key >> 16) & 0xFF, key >> 24, b) -
                         (int64_t)slab0;
      hit = lo < kSlab && lo + span >= 0;
    }
    const uint64_t bal = __ballot(hit);
    if (bal) {
      const int leader = __ffsll((unsigned long long)bal) - 1;
      uint32_t pos = 0;
      if (lane == leader) pos = atomicAdd(&nlst, (uint32_t)__popcll(bal));
      pos = __shfl(pos, leader);
      if (hit)
        lst[pos + __popcll(bal & ((1ull << lane) - 1ull))] =
            (unsigned short)(threadIdx.x + u * kHistThreads);
    }
  }
  __syncthreads();
  const uint32_t n = nlst;
  for (uint32_t i = threadIdx.x; i < n; i += kHistThreads) {
    const int64_t q = q0 + lst[i];
    const uint32_t m = vmask[q];
    const uint32_t key = basekey[q];
    const int ix = key & 0xFF, iy = (key >> 8) & 0xFF, it = (key >> 16) & 0xFF, is = key >> 24;
    const uint32_t base = qimg ? (uint32_t)(qimg[q] * nbins1) : 0u;
#pragma unroll
    for (int slot = 0; slot < 16; ++slot) {
      if (!((m >> slot) & 1u)) continue;
      const uint32_t lb = base + lin_bin(ix + ((slot >> 3) & 1), iy + ((slot >> 2) & 1),
                                         it + ((slot >> 1) & 1), is + (slot & 1), b) - slab0;
      if (lb < (uint32_t)kSlab) {
        atomicAdd(&cnt2[lb >> 1], 1u << ((lb & 1u) * 16u));
        atomicMin(&fst[lb], (uint32_t)(q * 16 + slot));
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kSlab; i += kHistThreads) {
    const uint32_t c = (cnt2[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
    if (c && slab0 + i < nbins) {
      atomicAdd(&gcount[slab0 + i], c);
      atomicMin(&gfirst[slab0 + i], fst[i]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Ordered compaction of "first touch of a bin with >= thr votes" over ordinals q*16+slot.
constexpr int kSelThreads = 256;   // one thread per query, 256 queries per block

__device__ __forceinline__ uint32_t first_touch_slots(int64_t q, const uint32_t* basekey,
                                                      const uint32_t* vmask,
                                                      const uint32_t* gcount,
                                                      const uint32_t* gfirst, Bins b,
                                                      uint32_t qbase, uint32_t thr,
                                                      uint32_t bins_out[16]) {
  const uint32_t m = vmask[q] & 0xFFFFu;
  uint32_t n = 0;
  if (!m) return 0;
  const uint32_t key = basekey[q];
  const int ix = key & 0xFF, iy = (key >> 8) & 0xFF, it = (key >> 16) & 0xFF, is = key >> 24;
  // all of the query's count / first-touch loads in flight at once, then the compaction
  // (a load per slot inside the compacting loop was one dependent round trip per vote)
  uint32_t lbs[16], c[16], f[16];
#pragma unroll
  for (int slot = 0; slot < 16; ++slot) {
    lbs[slot] = qbase + lin_bin(ix + ((slot >> 3) & 1), iy + ((slot >> 2) & 1),
                                it + ((slot >> 1) & 1), is + (slot & 1), b);
    // unconditional loads (slots out of range read bin qbase, a valid address): a load under
    // a branch gets a vmcnt(0) wait at the branch's join, one round trip per slot again
    const bool in = (m >> slot) & 1u;
    const uint32_t a = in ? lbs[slot] : qbase;
    c[slot] = gcount[a];
    f[slot] = gfirst[a];
    if (!in) c[slot] = 0u;
  }
#pragma unroll
  for (int slot = 0; slot < 16; ++slot)
    if (c[slot] >= thr && f[slot] == (uint32_t)(q * 16 + slot)) bins_out[n++] = lbs[slot];
  return n;
}

// 256-thread exclusive scan (sum, or max with identity 0): wave prefix via shuffles, then
// the preceding waves' totals; sh holds 4 entries.  Ends with a barrier (sh reusable).
template <bool kMax>
__device__ __forceinline__ uint32_t block_scan256(uint32_t v, uint32_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x = kMax ? max(x, y) : x + y;
  }
  const uint32_t ex = __shfl_up(x, 1);   // exclusive within the wave
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < w; ++i) off = kMax ? max(off, sh[i]) : off + sh[i];
  __syncthreads();
  const uint32_t inw = lane ? ex : 0u;
  return kMax ? max(off, inw) : off + inw;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  // kSelThreads-wide exclusive scan (4 waves): wave prefix via shuffles, then wave offsets
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int i = 0; i < kSelThreads / 64; ++i) {
    if (i < w) off += sh[i];
    tot += sh[i];
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

// One pass, decoupled look-back (no count / scan / write kernel chain): a block counts its
// queries' first-touch slots, publishes its aggregate, and its thread 0 walks back over the
// preceding blocks' published words until one carries an inclusive prefix.  A status word is
// (epoch * 4 + flag) << 32 | value, flag 1 = aggregate, 2 = inclusive prefix; a word of an
// older call (other epoch) reads as "not yet published", so the array needs no reset.
// A block's position in the scan is a ticket drawn from a device counter when it starts
// (HIP does not promise dispatch in blockIdx order, and the stream may be CU-masked beside
// a full-chip matcher): every block waited on has already started, so it is resident or
// done.  The counter is never reset: the host passes the number of tickets drawn by earlier
// launches (stream order: they have all drawn theirs).
__global__ __launch_bounds__(kSelThreads) void select_kernel(
    int64_t nq, const uint32_t* __restrict__ basekey, const uint32_t* __restrict__ vmask,
    const uint32_t* __restrict__ gcount, const uint32_t* __restrict__ gfirst, Bins b,
    const int* __restrict__ qimg, int64_t nbins1, uint32_t thr, uint64_t* __restrict__ status,
    uint32_t epoch, unsigned long long* __restrict__ ticket, unsigned long long ticket_base,
    uint32_t* __restrict__ out, uint32_t* __restrict__ vidx, uint32_t* __restrict__ total) {
  __shared__ uint32_t sh[kSelThreads / 64];
  __shared__ uint32_t excl_s;
  __shared__ int blk_s;
  if (threadIdx.x == 0) blk_s = (int)(atomicAdd(ticket, 1ULL) - ticket_base);
  __syncthreads();
  const int blk = blk_s;
  const int64_t q = (int64_t)blk * kSelThreads + threadIdx.x;
  uint32_t tmp[16];
  const uint32_t qb = (qimg && q < nq) ? (uint32_t)(qimg[q] * nbins1) : 0u;
  const uint32_t n = q < nq ? first_touch_slots(q, basekey, vmask, gcount, gfirst, b, qb, thr, tmp) : 0;
  uint32_t tot;
  const uint32_t loc = block_excl_scan(n, sh, &tot);
  if (threadIdx.x < 64) {   // the look-back, by the first wave: 64 predecessors per round
    const int lane = threadIdx.x;
    const uint32_t e4 = epoch << 2;
    uint32_t ex = 0;
    if (blk > 0) {
      if (lane == 0)
        __hip_atomic_store(&status[blk], ((uint64_t)(e4 | 1u) << 32) | tot, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
      // lane l reads block hi - l; "before block 0" reads as an inclusive prefix of 0.  A
      // round ends at the nearest inclusive prefix in its window (lowest such lane) once every
      // word up to it is published, and adds the values up to it; a window with no inclusive
      // prefix adds all 64 aggregates and moves 64 blocks back.  (One round trip per 64
      // predecessors: a block-by-block walk was 47 us of C3's one-image tail.)
      for (int hi = blk - 1;;) {
        const int j = hi - lane;
        uint64_t st = (uint64_t)(e4 | 2u) << 32;
        if (j >= 0) st = __hip_atomic_load(&status[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t h = (uint32_t)(st >> 32);
        const uint32_t flag = (h & ~3u) == e4 ? (h & 3u) : 0u;
        const uint64_t incl = __ballot(flag == 2u), unpub = __ballot(flag == 0u);
        const int stop = incl ? __builtin_ctzll(incl) : 63;
        const uint64_t need = stop == 63 ? ~0ull : ((2ull << stop) - 1ull);
        if (unpub & need) {   // a word the round needs is not published yet
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint32_t v = lane <= stop ? (uint32_t)st : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
        ex += v;
        if (incl) break;
        hi -= 64;
      }
    }
    if (lane == 0) {
      __hip_atomic_store(&status[blk], ((uint64_t)(e4 | 2u) << 32) | (ex + tot), __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
      if (blk == (int)gridDim.x - 1) *total = ex + tot;
      excl_s = ex;
    }
  }
  __syncthreads();
  const uint32_t pos = excl_s + loc;
  for (uint32_t i = 0; i < n; ++i) {
    out[pos + i] = tmp[i];
    if (vidx) vidx[tmp[i]] = pos + i;   // bin -> valid index (reset after the member sort)
  }
}

// member offsets: voff[i] = sum_{j<i} count[vbin[j]], voff[V] = total (single workgroup)
__global__ __launch_bounds__(1024) void member_offsets_kernel(const uint32_t* __restrict__ vbin,
                                                              const uint32_t* __restrict__ gcount,
                                                              uint32_t* __restrict__ scal,
                                                              int64_t* __restrict__ voff,
                                                              uint32_t* __restrict__ cursor) {
  __shared__ uint32_t sh[16];
  __shared__ int64_t carry_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = scal[0];
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const uint32_t v = i < n ? gcount[vbin[i]] : 0;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < w) off += sh[k];
      tot += sh[k];
    }
    const int64_t c = carry_s;
    if (i < n) {
      voff[i] = c + off + x - v;
      cursor[i] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) carry_s = c + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    voff[n] = carry_s;
    scal[1] = (uint32_t)carry_s;
  }
}

// members, step 1 (valid-bin count known to fit LDS): a work-group takes 256 consecutive
// queries.  Their votes first reserve LDS slots per valid bin (local rank = the LDS atomic's
// return), then ONE global atomicAdd per (work-group, bin it touched) reserves the run in
// the bin's member list -- those atomics are independent, so a wave has them all in flight
// at once instead of one returning atomic per distinct bin after another (the chain that
// made the per-wave aggregation latency-bound on the few reserved CUs).  Runs land in
// arbitrary order; member_order_*_kernel sort each bin into query order afterwards.
// With V beyond the LDS table every wave aggregates its own votes instead: per vote slot,
// the lanes voting for the same bin take ONE atomicAdd (leader = lowest lane) and place
// their queries in lane order inside the reserved run.
constexpr int kFillMaxV = 12288;   // 48 KiB of u32 per work-group
constexpr int kFillBatch = 8;      // global atomics a thread keeps in flight

__device__ __forceinline__ void fill_wave_aggregated(
    int64_t q, bool in, uint32_t m, uint32_t k, uint32_t base, Bins b,
    const uint32_t* __restrict__ vidx, const int64_t* __restrict__ voff,
    uint32_t* __restrict__ cursor, int32_t* __restrict__ members) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  if (__ballot(in && m != 0) == 0) return;
  const int ix = k & 0xFF, iy = (k >> 8) & 0xFF, it = (k >> 16) & 0xFF, is = k >> 24;
  for (int slot = 0; slot < 16; ++slot) {
    uint32_t v = 0xFFFFFFFFu;
    if (in && ((m >> slot) & 1u))
      v = vidx[base + lin_bin(ix + ((slot >> 3) & 1), iy + ((slot >> 2) & 1),
                              it + ((slot >> 1) & 1), is + (slot & 1), b)];
    uint64_t pend = __ballot(v != 0xFFFFFFFFu);
    while (pend) {
      const int leader = __ffsll((unsigned long long)pend) - 1;
      const uint32_t vv = __shfl(v, leader);
      const uint64_t same = __ballot(v == vv);
      uint32_t r = 0;
      if (lane == leader) r = atomicAdd(&cursor[vv], (uint32_t)__popcll(same));
      r = __shfl(r, leader);
      if (v == vv) members[voff[vv] + r + __popcll(same & below)] = (int32_t)q;
      pend &= ~same;
    }
  }
}

__global__ __launch_bounds__(256) void member_fill_lds_kernel(
    int64_t nq, const uint32_t* __restrict__ scal, const uint32_t* __restrict__ basekey,
    const uint32_t* __restrict__ vmask, Bins b, const int* __restrict__ qimg, int64_t nbins1,
    const uint32_t* __restrict__ vidx, const int64_t* __restrict__ voff,
    uint32_t* __restrict__ cursor, int32_t* __restrict__ members) {
  __shared__ uint32_t cnt[kFillMaxV];
  const int64_t V = scal[0];
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool in = q < nq;
  uint32_t m = 0, k = 0, base = 0;
  if (in) {
    m = vmask[q] & 0xFFFFu;
    k = basekey[q];
    base = qimg ? (uint32_t)(qimg[q] * nbins1) : 0u;
  }
  if (V > kFillMaxV) {   // uniform over the grid
    fill_wave_aggregated(q, in, m, k, base, b, vidx, voff, cursor, members);
    return;
  }
  for (int64_t i = threadIdx.x; i < V; i += 256) cnt[i] = 0;
  __syncthreads();
  const int ix = k & 0xFF, iy = (k >> 8) & 0xFF, it = (k >> 16) & 0xFF, is = k >> 24;
  uint32_t v[16], r[16];
  // independent loads, one wait: unconditional (a slot without a vote reads entry 0; its
  // key may be stale -- basekey is written for good matches only) -- a load under a branch
  // waits at the branch's join
#pragma unroll
  for (int slot = 0; slot < 16; ++slot) {
    const bool vin = (m >> slot) & 1u;
    v[slot] = vidx[vin ? base + lin_bin(ix + ((slot >> 3) & 1), iy + ((slot >> 2) & 1),
                                        it + ((slot >> 1) & 1), is + (slot & 1), b)
                       : 0u];
    if (!vin) v[slot] = 0xFFFFFFFFu;
  }
#pragma unroll
  for (int slot = 0; slot < 16; ++slot)
    r[slot] = v[slot] != 0xFFFFFFFFu ? atomicAdd(&cnt[v[slot]], 1u) : 0u;
  __syncthreads();
  // the work-group's run of every bin it touched: kFillBatch returning atomics in flight
  for (int64_t i0 = threadIdx.x; i0 < V; i0 += 256 * kFillBatch) {
    uint32_t c[kFillBatch], o[kFillBatch];
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j) {
      const int64_t i = i0 + 256 * j;
      c[j] = i < V ? cnt[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j)
      o[j] = c[j] ? atomicAdd(&cursor[i0 + 256 * j], c[j]) : 0u;
#pragma unroll
    for (int j = 0; j < kFillBatch; ++j)
      if (c[j]) cnt[i0 + 256 * j] = o[j];
  }
  __syncthreads();
#pragma unroll
  for (int slot = 0; slot < 16; ++slot)
    if (v[slot] != 0xFFFFFFFFu) members[voff[v[slot]] + cnt[v[slot]] + r[slot]] = (int32_t)q;
}

// Small bins (the great majority: a few to a few dozen members) take a wave of their own:
// each query votes a bin at most once, so query order is ascending order, and up to
// kWaveCap members sort in registers (bitonic, kWaveE per lane, cross-lane stages by
// shuffles) -- no LDS, no barriers, so the kernel stays fast on the few CUs a reserved
// tail gets (sod_set_cu_reserve).  Also resets the bin -> valid index map of EVERY valid
// bin; member_order_kernel then takes the bins above kWaveCap.
constexpr int kWaveE = 4;
constexpr int kWaveCap = 64 * kWaveE;

template <int J>
__device__ __forceinline__ void wave_sort_reg(uint32_t (&a)[kWaveE], int lane, int k) {
#pragma unroll
  for (int r = 0; r < kWaveE; ++r) {
    if (r & J) continue;
    const bool asc = ((lane * kWaveE + r) & k) == 0;
    const uint32_t x = a[r], y = a[r | J];
    const bool sw = asc ? (x > y) : (x < y);
    a[r] = sw ? y : x;
    a[r | J] = sw ? x : y;
  }
}

__global__ __launch_bounds__(256) void member_order_small_kernel(
    const uint32_t* __restrict__ scal, const uint32_t* __restrict__ vbin,
    const int64_t* __restrict__ voff, uint32_t* __restrict__ vidx,
    int32_t* __restrict__ members) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t V = scal[0];
  for (int64_t v = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); v < V;
       v += nwaves) {
    const int64_t a0 = voff[v];
    const int n = (int)(voff[v + 1] - a0);
    if (lane == 0) vidx[vbin[v]] = 0xFFFFFFFFu;
    if (n <= 1 || n > kWaveCap) continue;                     // uniform over the wave
    uint32_t a[kWaveE];
#pragma unroll
    for (int r = 0; r < kWaveE; ++r) {
      const int i = lane * kWaveE + r;
      a[r] = i < n ? (uint32_t)members[a0 + i] : 0xFFFFFFFFu;
    }
    int p = kWaveE;
    while (p < n) p <<= 1;
    for (int k = 2; k <= p; k <<= 1) {
      for (int j = k >> 1; j >= kWaveE; j >>= 1) {            // partner in lane ^ (j / E)
#pragma unroll
        for (int r = 0; r < kWaveE; ++r) {
          const uint32_t o = __shfl_xor(a[r], j / kWaveE);
          const int i = lane * kWaveE + r;
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          a[r] = keep_min ? min(a[r], o) : max(a[r], o);
        }
      }
      if (k >= 4) wave_sort_reg<2>(a, lane, k);
      wave_sort_reg<1>(a, lane, k);
    }
#pragma unroll
    for (int r = 0; r < kWaveE; ++r) {
      const int i = lane * kWaveE + r;
      if (i < n) members[a0 + i] = (int32_t)a[r];
    }
  }
}

// Bins above kWaveCap members: one work-group per bin marks its members in an LDS bitmap
// over the bin's query range [min, max] and writes them back in bit order (= query
// order): a popcount scan over the words gives every word its output offset.  Ranges
// beyond kBitWords*32 queries (only when nq > kBitQ) are rebuilt by members_kernel.
constexpr int kOrderT = 256;
constexpr int kBitWords = 16384;                // 64 KiB of LDS: query ranges up to 512 Ki
constexpr int64_t kBitQ = (int64_t)kBitWords * 32;

__device__ __forceinline__ uint32_t block_reduce_min256(uint32_t x, uint32_t* sh) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x = min(x, (uint32_t)__shfl_xor(x, d));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
  __syncthreads();
  return min(min(sh[0], sh[1]), min(sh[2], sh[3]));
}

__global__ __launch_bounds__(kOrderT) void member_order_kernel(const uint32_t* __restrict__ scal,
                                                               const int64_t* __restrict__ voff,
                                                               int64_t nq,
                                                               int32_t* __restrict__ members) {
  __shared__ uint32_t bits[kBitWords];
  __shared__ uint32_t red[2][4];
  __shared__ uint32_t part[4];
  if (nq > kBitQ) return;                                     // members_kernel rebuilds them
  const int64_t V = scal[0];
  for (int64_t v = blockIdx.x; v < V; v += gridDim.x) {
    const int64_t a = voff[v];
    const int64_t n = voff[v + 1] - a;
    if (n <= kWaveCap) continue;                              // uniform over the group
    uint32_t lo = 0xFFFFFFFFu, hi_neg = 0xFFFFFFFFu;
    for (int64_t i = threadIdx.x; i < n; i += kOrderT) {
      const uint32_t q = (uint32_t)members[a + i];
      lo = min(lo, q);
      hi_neg = min(hi_neg, ~q);
    }
    lo = block_reduce_min256(lo, red[0]);
    const uint32_t hi = ~block_reduce_min256(hi_neg, red[1]);
    const int words = (int)((hi - lo) / 32 + 1);
    for (int w = threadIdx.x; w < words; w += kOrderT) bits[w] = 0u;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < n; i += kOrderT) {
      const uint32_t d = (uint32_t)members[a + i] - lo;
      atomicOr(&bits[d >> 5], 1u << (d & 31));
    }
    __syncthreads();
    // contiguous words per thread, exclusive scan of their popcounts, then write in order
    const int per = (words + kOrderT - 1) / kOrderT;
    const int w0 = threadIdx.x * per, w1 = min(words, w0 + per);
    uint32_t cnt = 0;
    for (int w = w0; w < w1; ++w) cnt += __popc(bits[w]);
    uint32_t off = block_scan256<false>(cnt, part);
    for (int w = w0; w < w1; ++w) {
      uint32_t x = bits[w];
      while (x) {
        const int bit = __ffs(x) - 1;
        members[a + off++] = (int32_t)(lo + (uint32_t)w * 32u + (uint32_t)bit);
        x &= x - 1u;
      }
    }
    __syncthreads();
  }
}

// one wave per valid bin: members = matches voting for it, in query order.  Each pass
// covers 256 queries (4 loads per lane in flight) from the bin's first touch until all
// of its votes are found.
__global__ __launch_bounds__(256) void members_kernel(
    int64_t nq, const uint32_t* __restrict__ scal, const uint32_t* __restrict__ vbin,
    const int64_t* __restrict__ voff, const uint32_t* __restrict__ gcount,
    const uint32_t* __restrict__ gfirst, const uint32_t* __restrict__ basekey,
    const uint32_t* __restrict__ vmask, Bins b, const int* __restrict__ qimg, int64_t nbins1,
    int32_t* __restrict__ members) {
  constexpr int U = 4;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t V = scal[0];
  for (int64_t v = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); v < V; v += nwaves) {
    const uint32_t lb = vbin[v];
    const int img = qimg ? (int)(lb / nbins1) : 0;
    const uint32_t ll = qimg ? (uint32_t)(lb % nbins1) : lb;   // bin within its image
    const int bs_ = ll % b.s, bt_ = (ll / b.s) % b.t, by_ = (ll / (b.s * b.t)) % b.y,
              bx_ = ll / (b.s * b.t * b.y);
    const uint32_t need = gcount[lb];
    if (need <= (uint32_t)kWaveCap || nq <= kBitQ) continue;   // fill + order kernels
    const int64_t off = voff[v];
    uint32_t got = 0;
    for (int64_t q0 = gfirst[lb] >> 4; got < need && q0 < nq; q0 += 64 * U) {
      uint32_t m[U], key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + u * 64 + lane;
        m[u] = (q < nq && (!qimg || qimg[q] == img)) ? (vmask[q] & 0xFFFFu) : 0u;
        key[u] = q < nq ? basekey[q] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        bool mem = false;
        if (m[u]) {
          const int dx = bx_ - (int)(key[u] & 0xFF), dy = by_ - (int)((key[u] >> 8) & 0xFF),
                    dt = bt_ - (int)((key[u] >> 16) & 0xFF), ds = bs_ - (int)(key[u] >> 24);
          if ((unsigned)dx <= 1u && (unsigned)dy <= 1u && (unsigned)dt <= 1u && (unsigned)ds <= 1u)
            mem = (m[u] >> (dx * 8 + dy * 4 + dt * 2 + ds)) & 1u;
        }
        const uint64_t bal = __ballot(mem);
        if (mem) {
          const uint32_t pos = __popcll(bal & ((1ull << lane) - 1ull));
          members[off + got + pos] = (int32_t)(q0 + u * 64 + lane);
        }
        got += __popcll(bal);
      }
    }
  }
}

// Small query windows (<= kSmallQ): select + member offsets + ordered member lists in ONE
// work-group, one launch instead of five (select, offsets, fill, two orderings).  On the
// few reserved CUs a one-image tail is a chain of dependent launches of a few microseconds
// each whatever their work; here the phases are separated by work-group barriers.
//   1. the window's queries are copied to LDS while the valid bins are compacted in
//      first-touch order (first_touch_slots, as select_kernel; a running carry replaces the
//      look-back: the work-group walks the queries in order)
//   2. voff = exclusive scan of the bins' vote counts (as member_offsets_kernel)
//   3. one wave per bin scans the queries in LDS from the bin's first touch until it has
//      found all its votes, in query order by construction (the test of members_kernel)
// Same outputs as the multi-kernel path: vbin, scal[0] = V, voff, scal[1], members.
constexpr int kSmallT = 1024;
constexpr int kSmallQ = 2048;
constexpr int kSmallV = 2048;   // valid bins whose (bin, count, first touch, offset) stay in LDS

__global__ __launch_bounds__(kSmallT) void select_small_kernel(
    int64_t nq, const uint32_t* __restrict__ basekey, const uint32_t* __restrict__ vmask,
    const uint32_t* __restrict__ gcount, const uint32_t* __restrict__ gfirst, Bins b,
    const int* __restrict__ qimg, int64_t nbins1, uint32_t thr, uint32_t* __restrict__ vbin,
    uint32_t* __restrict__ scal, int64_t* __restrict__ voff, int32_t* __restrict__ members) {
  __shared__ uint32_t skey[kSmallQ], smask[kSmallQ];
  __shared__ int simg[kSmallQ];
  __shared__ uint32_t sh[kSmallT / 64];
  __shared__ uint32_t vb_lb[kSmallV], vb_need[kSmallV], vb_first[kSmallV], vb_off[kSmallV];
  __shared__ uint32_t carry_s;
  __shared__ int64_t carry64_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int kW = kSmallT / 64;
  if (tid == 0) {
    carry_s = 0;
    carry64_s = 0;
  }
  __syncthreads();
  // 1. valid bins in first-touch order
  for (int64_t q0 = 0; q0 < nq; q0 += kSmallT) {
    const int64_t q = q0 + tid;
    uint32_t tmp[16];
    uint32_t n = 0;
    if (q < nq) {
      const int im = qimg ? qimg[q] : 0;
      n = first_touch_slots(q, basekey, vmask, gcount, gfirst, b, (uint32_t)(im * nbins1), thr, tmp);
      skey[q] = basekey[q];
      smask[q] = vmask[q] & 0xFFFFu;
      simg[q] = im;
    }
    uint32_t x = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t off = carry_s, tot = 0;
    for (int i = 0; i < kW; ++i) {
      if (i < w) off += sh[i];
      tot += sh[i];
    }
    const uint32_t pos = off + x - n;
    for (uint32_t i = 0; i < n; ++i) {
      vbin[pos + i] = tmp[i];
      if (pos + i < kSmallV) vb_lb[pos + i] = tmp[i];
    }
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  const int64_t V = carry_s;
  // 2. member offsets
  const bool in_lds = V <= kSmallV;
  for (int64_t v0 = 0; v0 < V; v0 += kSmallT) {
    const int64_t v = v0 + tid;
    uint32_t c = 0u;
    if (v < V) {
      const uint32_t lb = in_lds ? vb_lb[v] : vbin[v];
      c = gcount[lb];
      if (in_lds) {
        vb_need[v] = c;
        vb_first[v] = gfirst[lb];
      }
    }
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < kW; ++i) {
      if (i < w) off += sh[i];
      tot += sh[i];
    }
    const int64_t base = carry64_s;
    if (v < V) {
      voff[v] = base + off + x - c;
      if (in_lds) vb_off[v] = (uint32_t)(base + off + x - c);   // < 16 * kSmallQ
    }
    __syncthreads();
    if (tid == 0) carry64_s = base + tot;
    __syncthreads();
  }
  if (tid == 0) {
    scal[0] = (uint32_t)V;
    scal[1] = (uint32_t)carry64_s;
    voff[V] = carry64_s;
  }
  __syncthreads();   // voff (global) written above is read by other waves below
  // 3. members in query order, one wave per bin
  for (int64_t v = w; v < V; v += kW) {
    const uint32_t lb = in_lds ? vb_lb[v] : vbin[v];
    const int img = qimg ? (int)(lb / nbins1) : 0;
    const uint32_t ll = qimg ? (uint32_t)(lb % nbins1) : lb;   // bin within its image
    const int bs_ = ll % b.s, bt_ = (ll / b.s) % b.t, by_ = (ll / (b.s * b.t)) % b.y,
              bx_ = ll / (b.s * b.t * b.y);
    const uint32_t need = in_lds ? vb_need[v] : gcount[lb];
    const int64_t off = in_lds ? (int64_t)vb_off[v] : voff[v];
    uint32_t got = 0;
    const int qn = (int)nq;
    for (int q0 = (int)((in_lds ? vb_first[v] : gfirst[lb]) >> 4); got < need && q0 < qn; q0 += 64) {
      // branch-free test (a lane past the window reads the last query and is masked off):
      // nested conditions cost an exec-mask branch and an LDS wait each
      const int q = q0 + lane;
      const int qq = min(q, qn - 1);
      const uint32_t m = smask[qq], key = skey[qq];
      const int qimg_q = simg[qq];
      const uint32_t dx = (uint32_t)(bx_ - (int)(key & 0xFF)), dy = (uint32_t)(by_ - (int)((key >> 8) & 0xFF)),
                     dt = (uint32_t)(bt_ - (int)((key >> 16) & 0xFF)), ds = (uint32_t)(bs_ - (int)(key >> 24));
      const bool win = (dx | dy | dt | ds) <= 1u;
      const bool mem = (q < qn) & (qimg_q == img) & win & (((m >> ((dx * 8 + dy * 4 + dt * 2 + ds) & 15u)) & 1u) != 0u);
      const uint64_t bal = __ballot(mem);
      if (mem) members[off + got + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)q;
      got += __popcll(bal);
    }
  }
}

// ---------------------------------------------------------------------------------------
// One query image of <= kFusedQ queries in ONE work-group: pose + votes + valid bins + member
// lists + the affine gather -- pose_kernel, hist_kernel, select_small_kernel and
// affine_gather_kernel in one launch (main.py's own regime, one image of ~500 keypoints: those
// four launches took ~37 us of a ~0.2 ms step, rocprofv3 r04 lat1).  Same outputs, bit for bit.
//
// No dense bin table.  Query q votes the 2x2x2x2 box above its base bin K(q), each vote kept
// when every index is < bins -- a property of the bin, not of the query (vote_mask).  So the
// votes of bin B come from the queries whose base key is B - e, e in {0,1}^4, and
//   count(B) = sum_e n(B - e),   first(B) = min_e 16 q0(B - e) + slot(e)
// (slot(e) = 8 e0 + 4 e1 + 2 e2 + e3; first = main.py:113-119's dict insertion ordinal, as
// hist_kernel computes it), with n(K) / q0(K) = the number / the lowest index of the voting
// queries whose base key is K: an LDS hash over at most kFusedQ distinct base keys, instead of
// 98 304 bins (C3) that do not fit LDS.  A voting query then finds, for each of its votes, the
// bin's count and first touch from 16 lookups; a vote that is its bin's first touch of a bin
// with >= thr votes emits the bin (valid bins in first-touch order); members in query order as
// select_small_kernel finds them (one wave per bin from its first touch), and the member's
// model / query points for affine_kernel from LDS.
constexpr int kFusedT = 1024;
constexpr int kFusedQ = 1024;                   // one query per thread
constexpr int kFusedHash = 2048;                // >= 2 slots per distinct base key
constexpr uint32_t kNoKey = 0xFFFFFFFFu;        // indices are <= 254: never a base key

__device__ __forceinline__ uint32_t key_hash(uint32_t k) {
  return (k * 0x9E3779B1u) >> (32 - 11);        // log2(kFusedHash) = 11
}

// count and first-touch ordinal of vote slot sl of a query with base key `key`: bin B = key +
// e(sl); its voters are the queries with base key B - e for the e in {0,1}^4 that keep every
// index >= 0, each contributing n(B - e) votes, the first at ordinal 16 q0(B - e) + slot(e)
__device__ __forceinline__ void bin_votes(uint32_t key, uint32_t sl, const uint32_t* hk,
                                          const uint32_t* hn, const uint32_t* hq,
                                          uint32_t* cnt_out, uint32_t* fst_out) {
  const int bx = (int)(key & 0xFF) + (int)((sl >> 3) & 1), by = (int)((key >> 8) & 0xFF) + (int)((sl >> 2) & 1),
            bt = (int)((key >> 16) & 0xFF) + (int)((sl >> 1) & 1), bs = (int)(key >> 24) + (int)(sl & 1);
  uint32_t h[16], k2[16], kv[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {   // every first probe in flight at once
    const int kx = bx - ((e >> 3) & 1), ky = by - ((e >> 2) & 1), kt = bt - ((e >> 1) & 1),
              ks = bs - (e & 1);
    k2[e] = (kx | ky | kt | ks) < 0 ? kNoKey
                                     : (uint32_t)kx | ((uint32_t)ky << 8) | ((uint32_t)kt << 16) |
                                           ((uint32_t)ks << 24);
    h[e] = key_hash(k2[e]);
    kv[e] = hk[h[e]];
  }
  // nearly every probe ends at its first slot (a hit or an empty slot: <= 50 % load); the
  // values of all 16 first slots are read together, and only a collision walks on
  uint32_t nv_[16], qv_[16];
  bool coll = false;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    nv_[e] = hn[h[e]];
    qv_[e] = hq[h[e]];
    coll |= k2[e] != kNoKey && kv[e] != k2[e] && kv[e] != kNoKey;
  }
  uint32_t cnt = 0u, fst = 0xFFFFFFFFu;
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if (k2[e] != kNoKey && kv[e] == k2[e]) {
      cnt += nv_[e];
      fst = min(fst, qv_[e] * 16u + (uint32_t)e);
    }
  if (__builtin_expect(coll, 0)) {
#pragma unroll 1
    for (int e = 0; e < 16; ++e) {
      if (k2[e] == kNoKey || kv[e] == k2[e] || kv[e] == kNoKey) continue;
      uint32_t hh = h[e], kk = kv[e];
      while (kk != k2[e] && kk != kNoKey) {   // linear probe past the collision
        hh = (hh + 1) & (kFusedHash - 1);
        kk = hk[hh];
      }
      if (kk == k2[e]) {
        cnt += hn[hh];
        fst = min(fst, hq[hh] * 16u + (uint32_t)e);
      }
    }
  }
  *cnt_out = cnt;
  *fst_out = fst;
}

__global__ __launch_bounds__(kFusedT) void hough_small_kernel(
    int64_t nq, const uint8_t* __restrict__ good, const int* __restrict__ idx1,
    const float* __restrict__ qx, const float* __restrict__ qy, const float* __restrict__ qa,
    const int* __restrict__ qo, const float* __restrict__ mx, const float* __restrict__ my,
    const float* __restrict__ ma, const int* __restrict__ mo, const int* __restrict__ mimg,
    const double* __restrict__ cent, const int* __restrict__ isize, int H, int W, Bins b,
    const int* __restrict__ lut, uint32_t thr, double* __restrict__ pose,
    uint32_t* __restrict__ basekey, uint32_t* __restrict__ vmask, int2* __restrict__ msize,
    double* __restrict__ grec, uint32_t* __restrict__ gstat, uint32_t* __restrict__ vbin,
    uint32_t* __restrict__ vcnt, uint32_t* __restrict__ vfirst, uint32_t* __restrict__ scal,
    int64_t* __restrict__ voff, int32_t* __restrict__ members, float* __restrict__ amx,
    float* __restrict__ amy, float* __restrict__ aqx, float* __restrict__ aqy,
    int32_t* __restrict__ aisig) {
  __shared__ uint32_t skey[kFusedQ], smask[kFusedQ];
  __shared__ float smx[kFusedQ], smy[kFusedQ], sqx[kFusedQ], sqy[kFusedQ];
  __shared__ uint32_t hk[kFusedHash], hn[kFusedHash], hq[kFusedHash];
  __shared__ uint32_t vb_lb[kSmallV], vb_need[kSmallV], vb_first[kSmallV], vb_off[kSmallV];
  __shared__ uint16_t vlist[kFusedQ];   // voting queries in order
  __shared__ uint32_t vfm[kFusedQ];     // their valid-first-touch slot masks
  __shared__ uint32_t vbase[kFusedQ];   // valid index of their first valid-first slot
  __shared__ uint16_t vfc[kFusedQ * 16];   // vote count of each valid-first vote
  __shared__ uint32_t sh[kFusedT / 64];
  __shared__ uint32_t carry_s;
  __shared__ int64_t carry64_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int kW = kFusedT / 64;
  for (int i = tid; i < kFusedHash; i += kFusedT) {
    hk[i] = kNoKey;
    hn[i] = 0u;
    hq[i] = 0xFFFFFFFFu;
  }
  if (tid == 0) {
    carry_s = 0;
    carry64_s = 0;
  }
  __syncthreads();
  // 1. pose + base key + vote mask per query (pose_kernel); the voting queries' base keys
  //    into the hash (count, lowest query)
  for (int64_t q = tid; q < nq; q += kFusedT) {
    uint32_t key = 0u, mask = 0u;
    float fmx = 0.f, fmy = 0.f;
    const bool g = good[q] != 0;
    const float fqx = qx[q], fqy = qy[q];
    if (g) {
      const int m = idx1[q];
      const int im = mimg[m];
      double p[4], t[2];
      int ix[4];
      fmx = mx[m];
      fmy = my[m];
      pose_bins(fmx, fmy, ma[m], mo[m], fqx, fqy, qa[q], qo[q], cent[2 * im], cent[2 * im + 1],
                H, W, b, lut, p, ix, t);
      if (grec && guard_flag(p, t, fqx, fqy, H, W, b)) guard_push(grec, gstat, q, p, t, fqx, fqy, H, W);
      pose[4 * q + 0] = p[0];
      pose[4 * q + 1] = p[1];
      pose[4 * q + 2] = p[2];
      pose[4 * q + 3] = p[3];
      msize[q] = make_int2(isize[2 * im], isize[2 * im + 1]);
      key = (uint32_t)ix[0] | ((uint32_t)ix[1] << 8) | ((uint32_t)ix[2] << 16) |
            ((uint32_t)ix[3] << 24);
      mask = vote_mask(ix, b);   // one rank: every match's DB row is this shard's
      basekey[q] = key;
    }
    vmask[q] = mask ? (mask | 0x10000u) : 0u;
    skey[q] = key;
    smask[q] = mask;
    smx[q] = fmx;
    smy[q] = fmy;
    sqx[q] = fqx;
    sqy[q] = fqy;
    if (mask) {
      for (uint32_t h = key_hash(key);; h = (h + 1) & (kFusedHash - 1)) {
        const uint32_t old = atomicCAS(&hk[h], kNoKey, key);
        if (old == kNoKey || old == key) {
          atomicAdd(&hn[h], 1u);
          atomicMin(&hq[h], (uint32_t)q);
          break;
        }
      }
    }
  }
  __syncthreads();
  // the voting queries, in query order (the votes' ordinals follow it)
  for (int64_t q0 = 0; q0 < nq; q0 += kFusedT) {
    const int64_t q = q0 + tid;
    const bool vote = q < nq && smask[q] != 0u;
    const uint64_t bal = __ballot(vote);
    if (lane == 0) sh[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t off = carry_s, tot = 0;
    for (int i = 0; i < kW; ++i) {
      if (i < w) off += sh[i];
      tot += sh[i];
    }
    if (vote) {
      const uint32_t pos = off + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
      vlist[pos] = (uint16_t)q;
      vfm[pos] = 0u;
    }
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  const uint32_t nv = carry_s;
  __syncthreads();
  if (tid == 0) carry_s = 0;
  // 2. one thread per vote (voting query i, slot s): its bin's count and first touch from 16
  //    hash lookups; the first touch of a bin with >= thr votes sets bit s of vfm[i]
  for (uint32_t it = tid; it < nv * 16u; it += kFusedT) {
    const uint32_t i = it >> 4, sl = it & 15u;
    const uint32_t q = vlist[i];
    const uint32_t m = smask[q];
    if (!((m >> sl) & 1u)) continue;
    const uint32_t key = skey[q];
    uint32_t cnt, fst;
    bin_votes(key, sl, hk, hn, hq, &cnt, &fst);
    if (cnt >= thr && fst == q * 16u + sl) {
      atomicOr(&vfm[i], 1u << sl);
      vfc[it] = (uint16_t)cnt;   // <= voting queries <= kFusedQ
    }
  }
  __syncthreads();
  // valid bins in first-touch order (voting query, then slot): the first valid index of each
  // voting query = the scan of the masks' popcounts (nv <= kFusedT: one round) ...
  {
    const uint32_t i = tid;
    const uint32_t fm = i < nv ? vfm[i] : 0u;
    const uint32_t n = (uint32_t)__popc(fm);
    uint32_t x = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int k = 0; k < kW; ++k) {
      if (k < w) off += sh[k];
      tot += sh[k];
    }
    if (i < nv) vbase[i] = off + x - n;
    if (tid == 0) carry_s = tot;
  }
  __syncthreads();
  // ... and every valid-first vote writes its bin there, one thread per vote
  for (uint32_t it = tid; it < nv * 16u; it += kFusedT) {
    const uint32_t i = it >> 4, sl = it & 15u;
    const uint32_t fm = vfm[i];
    if (!((fm >> sl) & 1u)) continue;
    const uint32_t v = vbase[i] + (uint32_t)__popc(fm & ((1u << sl) - 1u));
    const uint32_t key = skey[vlist[i]];
    const uint32_t lb = lin_bin((int)(key & 0xFF) + (int)((sl >> 3) & 1),
                                (int)((key >> 8) & 0xFF) + (int)((sl >> 2) & 1),
                                (int)((key >> 16) & 0xFF) + (int)((sl >> 1) & 1),
                                (int)(key >> 24) + (int)(sl & 1), b);
    const uint32_t cnt = vfc[it];
    vbin[v] = lb;
    aisig[v] = (int32_t)(lb % (uint32_t)b.s);   // affine_gather_kernel's i_sigma
    if (v < (uint32_t)kSmallV) {
      vb_lb[v] = lb;
      vb_need[v] = cnt;
      vb_first[v] = i;   // the bin's first voting query (its index in vlist)
    } else {
      vcnt[v] = cnt;
      vfirst[v] = i;
    }
  }
  __syncthreads();
  const int64_t V = carry_s;
  // 3. member offsets (exclusive scan of the counts, in valid order)
  for (int64_t v0 = 0; v0 < V; v0 += kFusedT) {
    const int64_t v = v0 + tid;
    uint32_t c = 0u;
    if (v < V)
      c = v < kSmallV ? vb_need[v]
                      : __hip_atomic_load(&vcnt[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < kW; ++i) {
      if (i < w) off += sh[i];
      tot += sh[i];
    }
    const int64_t base = carry64_s;
    if (v < V) {
      voff[v] = base + off + x - c;
      if (v < kSmallV) vb_off[v] = (uint32_t)(base + off + x - c);   // < 16 * kFusedQ
    }
    __syncthreads();
    if (tid == 0) carry64_s = base + tot;
    __syncthreads();
  }
  if (tid == 0) {
    scal[0] = (uint32_t)V;
    scal[1] = (uint32_t)carry64_s;
    voff[V] = carry64_s;
  }
  __syncthreads();   // voff (global) past the LDS copy is read by other waves below
  // 4. members in query order, one wave per bin from its first voting query, with the affine
  //    inputs of each member
  for (int64_t v = w; v < V; v += kW) {
    const bool lds_v = v < kSmallV;
    const uint32_t lb = lds_v ? vb_lb[v] : __hip_atomic_load(&vbin[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t need = lds_v ? vb_need[v] : __hip_atomic_load(&vcnt[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t off = lds_v ? (int64_t)vb_off[v]
                              : __hip_atomic_load(&voff[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int jf = (int)(lds_v ? vb_first[v]
                               : __hip_atomic_load(&vfirst[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const int bs_ = lb % b.s, bt_ = (lb / b.s) % b.t, by_ = (lb / (b.s * b.t)) % b.y,
              bx_ = lb / (b.s * b.t * b.y);
    uint32_t got = 0;
    const int jn = (int)nv;
    // over the voting queries only (in query order), from the bin's first one
    for (int j0 = jf; got < need && j0 < jn; j0 += 64) {
      const int j = j0 + lane;
      const int q = vlist[min(j, jn - 1)];
      const uint32_t mm = smask[q], key = skey[q];
      const uint32_t dx = (uint32_t)(bx_ - (int)(key & 0xFF)), dy = (uint32_t)(by_ - (int)((key >> 8) & 0xFF)),
                     dt = (uint32_t)(bt_ - (int)((key >> 16) & 0xFF)), ds = (uint32_t)(bs_ - (int)(key >> 24));
      const bool win = (dx | dy | dt | ds) <= 1u;
      const bool mem = (j < jn) & win & (((mm >> ((dx * 8 + dy * 4 + dt * 2 + ds) & 15u)) & 1u) != 0u);
      const uint64_t bal = __ballot(mem);
      if (mem) {
        const int64_t jj = off + got + __popcll(bal & ((1ull << lane) - 1ull));
        members[jj] = (int32_t)q;
        amx[jj] = smx[q];
        amy[jj] = smy[q];
        aqx[jj] = sqx[q];
        aqy[jj] = sqy[q];
      }
      got += __popcll(bal);
    }
  }
  // 5. the guard records listed above: their count to the slot the host reads, and the append
  //    counter back to 0 for the next launch (hist_kernel's handover)
  __syncthreads();
  if (tid == 0) {
    const uint32_t g = __hip_atomic_load(&gstat[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gstat[1] = g;
    gstat[0] = 0u;
  }
}

// (tx, ty, alpha, qx, qy) of the poses of the members of listed valid bins, for the host's
// glibc redo of the PoseBin x / y means (sod_exact_xy_means); one work-group per bin:
// record roff[b] + t is member t of valid bin vb[b] (vote order)
__global__ void pose_rec_bins_kernel(int nb, const int32_t* __restrict__ vb,
                                     const int64_t* __restrict__ roff,
                                     const int64_t* __restrict__ voff,
                                     const int32_t* __restrict__ members,
                                     const int* __restrict__ idx1, const float* __restrict__ qx,
                                     const float* __restrict__ qy, const float* __restrict__ qa,
                                     const int* __restrict__ qo, const float* __restrict__ mx,
                                     const float* __restrict__ my, const float* __restrict__ ma,
                                     const int* __restrict__ mo, const int* __restrict__ mimg,
                                     const double* __restrict__ cent, double* __restrict__ rec) {
  const int b = blockIdx.x;
  if (b >= nb) return;
  const int64_t a = voff[vb[b]], cnt = voff[vb[b] + 1] - a, r0 = roff[b];
  for (int64_t t = threadIdx.x; t < cnt; t += blockDim.x) {
    const int q = members[a + t], m = idx1[q], im = mimg[m];
    int k;
    double s, tx, ty, al;
    pose_terms(mx[m], my[m], ma[m], mo[m], qa[q], qo[q], cent[2 * im], cent[2 * im + 1], k, s, tx,
               ty, al);
    double* r = rec + 5 * (r0 + t);
    r[0] = tx;
    r[1] = ty;
    r[2] = al;
    r[3] = (double)qx[q];
    r[4] = (double)qy[q];
  }
}

// PoseBin running means in vote order (PoseBin.py:19-43).  The recurrence
//   v' = (v*n + new) / (n+1)
// rounds at every step, so each bin's chain is inherently sequential; but the six
// quantities (x, y, alpha, s, w, h) are independent chains and their inputs can be fetched in
// parallel first.  One wave per valid bin; lanes 0-5 run the six chains in lockstep (same n,
// same 1/(n+1)).  All 64 lanes gather the next 64 members' inputs (member -> query -> pose,
// model keypoint -> model image -> size) into LDS while the chains run on the current batch,
// so a chain step is 4 dependent f64 ops and never a memory wait.  Division r / d (d = n + 1)
// is r times the double-double reciprocal hi + lo (hi = RN(1/d), lo = RN(1 - hi*d) * hi, both
// off the chain): RN(r*hi + RN(r*lo)), one FMA after one multiply.  Its error, ~2^-104 of r/d,
// is far below the distance from r/d to a rounding midpoint (>= 2^-53/d of r/d when r/d is
// not a double; never 0: a midpoint would need 54 significant bits in r), so it equals the
// correctly rounded r / d (also checked against r / d on 3e8 random cases).  Round 3's form,
// RN(r*hi) corrected by an FMA residual (Markstein), was 5 dependent ops.
constexpr int kGatherK = 4;   // members per thread per round in affine_gather_kernel

__global__ void recip_table_kernel(int64_t M, double* __restrict__ rtab) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M;
       i += (int64_t)gridDim.x * blockDim.x)
    rtab[i] = 1.0 / (double)(i + 1);
}

constexpr int kMeansU = 4;                  // members per lane per fetch: 256 per batch
constexpr int kMeansB = 64 * kMeansU;

// one wave: the bins v0, v0 + stride, ... (xs: the wave's LDS batch buffer)
__device__ __forceinline__ void means_wave(int64_t v0, int64_t stride, double (*xs)[kMeansB],
                                           const uint32_t* __restrict__ scal,
                                           const int64_t* __restrict__ voff,
                                           const int32_t* __restrict__ members,
                                           const double* __restrict__ pose,
                                           const int2* __restrict__ msize,
                                           const double* __restrict__ rtab,
                                           double* __restrict__ means) {
  const int lane = threadIdx.x & 63;
  const int k = lane < 6 ? lane : 0;
  const int64_t V = scal[0];
  for (int64_t v = v0; v < V; v += stride) {
    const int64_t a = voff[v], e = voff[v + 1];
    // batch b covers members a+256b ... ; n of member j is j - a (the first one sets the mean)
    double nx[kMeansU][7];
    auto fetch = [&](int64_t j0) {   // two dependent levels: member -> (pose, model size)
      int q[kMeansU];
#pragma unroll
      for (int u = 0; u < kMeansU; ++u) {
        const int64_t j = j0 + u * 64 + lane;
        q[u] = j < e ? members[j] : -1;
      }
#pragma unroll
      for (int u = 0; u < kMeansU; ++u) {
        const int64_t j = j0 + u * 64 + lane;
        const bool in = q[u] >= 0;
        const double* p = pose + 4 * (int64_t)(in ? q[u] : 0);
        const int2 wh = msize[in ? q[u] : 0];
#pragma unroll
        for (int c = 0; c < 4; ++c) nx[u][c] = in ? p[c] : 0.0;
        nx[u][4] = in ? (double)wh.x : 0.0;
        nx[u][5] = in ? (double)wh.y : 0.0;
        nx[u][6] = in ? rtab[j - a] : 0.0;   // 1 / (n + 1)
      }
    };
    double m = 0.0;
    fetch(a);
    for (int64_t j0 = a; j0 < e; j0 += kMeansB) {
#pragma unroll
      for (int u = 0; u < kMeansU; ++u)
#pragma unroll
        for (int c = 0; c < 7; ++c) xs[c][u * 64 + lane] = nx[u][c];
      __builtin_amdgcn_wave_barrier();
      if (j0 + kMeansB < e) fetch(j0 + kMeansB);   // in flight during the chains below
      const int cnt = (int)min<int64_t>(kMeansB, e - j0);
      if (lane < 6) {
        const double n0 = (double)(j0 - a);
        int i = 0;
        if (j0 == a) {              // first vote: mean = pose / model size
          m = xs[k][0];
          i = 1;
        }
        // 16 steps per block, the block's LDS operands in registers before its chain and the
        // next block's loads issued before it: the chain never waits on LDS (reading each
        // step's operands one step ahead put an LDS round trip on the chain every two steps,
        // ~2.5x the chain's own dependent f64 latency)
        double xv[16], iv[16];
        if (i + 16 <= cnt) {
#pragma unroll
          for (int t = 0; t < 16; ++t) {
            xv[t] = xs[k][i + t];
            iv[t] = xs[6][i + t];
          }
        }
        for (; i + 16 <= cnt; i += 16) {
          double xn[16], in_[16];
          const bool more = i + 32 <= cnt;
#pragma unroll
          for (int t = 0; t < 16; ++t) {   // (clamped: a read past the batch is never used)
            const int jn = more ? i + 16 + t : i + t;
            xn[t] = xs[k][jn];
            in_[t] = xs[6][jn];
          }
#pragma unroll
          for (int t = 0; t < 16; ++t) {
            const double n = n0 + (i + t), d = n + 1.0, inv = iv[t];
            const double lo = __builtin_fma(-inv, d, 1.0) * inv;   // off the chain
            const double r = m * n + xv[t];   // -ffp-contract=off: 2 roundings
            m = __builtin_fma(r, inv, r * lo);
          }
#pragma unroll
          for (int t = 0; t < 16; ++t) {
            xv[t] = xn[t];
            iv[t] = in_[t];
          }
        }
        for (; i < cnt; ++i) {
          const double n = n0 + i, d = n + 1.0, inv = xs[6][i];
          const double lo = __builtin_fma(-inv, d, 1.0) * inv;
          const double r = m * n + xs[k][i];
          m = __builtin_fma(r, inv, r * lo);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (lane < 6) means[6 * v + k] = m;
  }
}

__global__ __launch_bounds__(64) void means_kernel(const uint32_t* __restrict__ scal,
                                                   const int64_t* __restrict__ voff,
                                                   const int32_t* __restrict__ members,
                                                   const double* __restrict__ pose,
                                                   const int2* __restrict__ msize,
                                                   const double* __restrict__ rtab,
                                                   double* __restrict__ means) {
  // one buffer: the wave stores a batch, runs its chains, and only then stores the next
  __shared__ double xs[7][kMeansB];   // [quantity 0-5, 1/(n+1)][member]
  means_wave(blockIdx.x, gridDim.x, xs, scal, voff, members, pose, msize, rtab, means);
}

// ---------------------------------------------------------------------------------------
// affine verification
__global__ void affine_gather_kernel(const uint32_t* __restrict__ scal,
                                     const int32_t* __restrict__ members,
                                     const int* __restrict__ idx1, const float* __restrict__ mx,
                                     const float* __restrict__ my, const float* __restrict__ qx,
                                     const float* __restrict__ qy, const uint32_t* __restrict__ vbin,
                                     Bins b, int64_t nbins1, const int* __restrict__ qshape,
                                     float* __restrict__ amx, float* __restrict__ amy,
                                     float* __restrict__ aqx, float* __restrict__ aqy,
                                     int32_t* __restrict__ aisig, int32_t* __restrict__ bwh) {
  const int64_t M = scal[1], V = scal[0];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // kGatherK members per thread per round, each gather level issued for all of them
  for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x * kGatherK + threadIdx.x; e0 < M;
       e0 += stride * kGatherK) {
    int q[kGatherK], m[kGatherK];
#pragma unroll
    for (int i = 0; i < kGatherK; ++i) {
      const int64_t e = e0 + (int64_t)i * blockDim.x;
      q[i] = e < M ? members[e] : 0;
    }
#pragma unroll
    for (int i = 0; i < kGatherK; ++i) m[i] = idx1[q[i]];
#pragma unroll
    for (int i = 0; i < kGatherK; ++i) {
      const int64_t e = e0 + (int64_t)i * blockDim.x;
      if (e >= M) break;
      amx[e] = mx[m[i]];
      amy[e] = my[m[i]];
      aqx[e] = qx[q[i]];
      aqy[e] = qy[q[i]];
    }
  }
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += stride) {
    aisig[v] = (int32_t)(vbin[v] % b.s);   // nbins1 is a multiple of b.s
    if (qshape) {   // batch of query images: the bin's image (w, h) = image_query_size
      const int img = (int)(vbin[v] / nbins1);
      bwh[2 * v] = qshape[2 * img + 1];
      bwh[2 * v + 1] = qshape[2 * img];
    }
  }
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

// pinv of a symmetric 3x3 (numpy.linalg.pinv default rcond 1e-15 relative to the largest
// singular value; for a symmetric matrix the singular values are |eigenvalues|).
__device__ void pinv3_sym(const double g[3][3], double p[3][3]) {
  double a[3][3], v[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      a[i][j] = g[i][j];
      v[i][j] = (i == j) ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 32; ++sweep) {
    const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    const double dia = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
    if (off <= 1e-36 * dia || off == 0.0) break;
    for (int pq = 0; pq < 3; ++pq) {
      const int p_ = pq == 2 ? 1 : 0, q_ = pq == 0 ? 1 : 2;
      const double apq = a[p_][q_];
      if (apq == 0.0) continue;
      const double theta = (a[q_][q_] - a[p_][p_]) / (2.0 * apq);
      const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
      for (int k = 0; k < 3; ++k) {  // A <- A J (columns p, q)
        const double akp = a[k][p_], akq = a[k][q_];
        a[k][p_] = c * akp - s * akq;
        a[k][q_] = s * akp + c * akq;
      }
      for (int k = 0; k < 3; ++k) {  // A <- J^T A (rows p, q)
        const double apk = a[p_][k], aqk = a[q_][k];
        a[p_][k] = c * apk - s * aqk;
        a[q_][k] = s * apk + c * aqk;
      }
      for (int k = 0; k < 3; ++k) {
        const double vkp = v[k][p_], vkq = v[k][q_];
        v[k][p_] = c * vkp - s * vkq;
        v[k][q_] = s * vkp + c * vkq;
      }
    }
  }
  const double l[3] = {a[0][0], a[1][1], a[2][2]};
  const double lmax = fmax(fabs(l[0]), fmax(fabs(l[1]), fabs(l[2])));
  const double cut = 1e-15 * lmax;
  double inv[3];
  for (int i = 0; i < 3; ++i) inv[i] = (fabs(l[i]) > cut) ? 1.0 / l[i] : 0.0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      p[i][j] = v[i][0] * inv[0] * v[j][0] + v[i][1] * inv[1] * v[j][1] + v[i][2] * inv[2] * v[j][2];
}

// sum over the kG lanes of a lane group (xor butterfly inside the group)
template <int kG>
__device__ __forceinline__ double group_sum(double x) {
#pragma unroll
  for (int m = kG / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}
template <int kG>
__device__ __forceinline__ int group_sum_i(int x) {
#pragma unroll
  for (int m = kG / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

// One lane group of kAffG lanes per bin, 64 / kAffG bins per wave: a bin's work is a serial
// chain (member sums -> 3x3 Jacobi pinv -> residual test, repeated), so several bins in one
// wave run their chains in the same instructions -- the few reserved CUs of a chip split
// (sod_set_cu_reserve) hold 64 / kAffG times as many chains in flight.
constexpr int kAffG = 64;   // 16 measured slower at C3: the large bins' member loops lengthen
constexpr int kAffU = 8;    // members per lane per round of loads

// lane groups of G lanes: group g0 of ngroups takes the bins g0, g0 + ngroups, ...
template <int G>
__device__ __forceinline__ void affine_groups(
    int64_t g0, int64_t ngroups, int64_t nb_host, const uint32_t* __restrict__ nb_dev,
    const int64_t* __restrict__ off, const float* __restrict__ mx, const float* __restrict__ my,
    const float* __restrict__ qx, const float* __restrict__ qy, const int32_t* __restrict__ isig,
    int qw, int qh, const int32_t* __restrict__ bwh, double xf, double yf, int thr, int max_iter,
    const double* __restrict__ params_in, uint8_t* __restrict__ surv,
    int32_t* __restrict__ votes, double* __restrict__ params, uint8_t* __restrict__ alive,
    int mxfma) {
  const int lane = threadIdx.x & (G - 1);                 // lane within the bin's group
  const int64_t NB = nb_dev ? (int64_t)nb_dev[0] : nb_host;
  // every group of the wave runs the loop the same number of times (shuffles need the
  // whole wave): groups past the last bin idle with an empty member range
  const int64_t wave_first = g0 - (threadIdx.x & 63) / G;
  for (int64_t vb = wave_first; vb < NB; vb += ngroups) {
    const int64_t v = vb + (threadIdx.x & 63) / G;
    const bool live = v < NB;
    const int64_t a = live ? off[v] : 0, e = live ? off[v + 1] : 0;
    for (int64_t j = a + lane; j < e; j += G) alive[j] = 1;
    // AffineParameters.py:120-121: tolerance scales with the scale-bin INDEX pose[3]
    const int64_t bw = !live ? 0 : bwh ? bwh[2 * v] : qw;
    const int64_t bh = !live ? 0 : bwh ? bwh[2 * v + 1] : qh;
    const int32_t sig = live ? isig[v] : 0;
    const double xref = (double)(bw * sig) / xf;
    const double yref = (double)(bh * sig) / yf;
    int64_t n = e - a;
    double prm[6] = {0, 0, 0, 0, 0, 0};
    bool ok = false;
    const int rounds = max_iter < 1 ? 1 : max_iter;   // max_iter 0: solve once, remove nothing
    for (int it = 0; it < rounds; ++it) {
      double s[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      // kAffU members of the lane per round, all loads in flight before the sums (a load
      // under the alive test was one dependent round trip per member: a C3 bin of ~2 700
      // members took ~42 of them per pass); same order of additions as one at a time
      for (int64_t j0 = a + lane; j0 < e; j0 += (int64_t)G * kAffU) {
        float fx[kAffU], fy[kAffU], fu[kAffU], fw[kAffU];
        uint8_t al[kAffU];
#pragma unroll
        for (int t = 0; t < kAffU; ++t) {
          const int64_t j = j0 + (int64_t)t * G;
          const int64_t jc = j < e ? j : j0;   // clamped: an unused, valid address
          al[t] = j < e ? alive[jc] : 0;
          fx[t] = mx[jc];
          fy[t] = my[jc];
          fu[t] = qx[jc];
          fw[t] = qy[jc];
        }
#pragma unroll
        for (int t = 0; t < kAffU; ++t) {
          if (!al[t]) continue;
          const double x = fx[t], y = fy[t], u = fu[t], w = fw[t];
          s[0] += x * x; s[1] += x * y; s[2] += x; s[3] += y * y; s[4] += y; s[5] += 1.0;
          s[6] += x * u; s[7] += y * u; s[8] += u; s[9] += x * w; s[10] += y * w; s[11] += w;
        }
      }
#pragma unroll
      for (int k = 0; k < 12; ++k) s[k] = group_sum<G>(s[k]);
      if (params_in) {  // remove_outliers with the caller's posebin.affine_parameters
#pragma unroll
        for (int k = 0; k < 6; ++k) prm[k] = live ? params_in[6 * v + k] : 0.0;
      } else if (n > 0) {  // AffineParameters.py:105: no-op for an empty bin
        const double g[3][3] = {{s[0], s[1], s[2]}, {s[1], s[3], s[4]}, {s[2], s[4], s[5]}};
        double p[3][3];
        pinv3_sym(g, p);
        // x = [m1 m2 m3 m4 tx ty]: (m1,m2,tx) from the u rows, (m3,m4,ty) from the v rows
        prm[0] = p[0][0] * s[6] + p[0][1] * s[7] + p[0][2] * s[8];
        prm[1] = p[1][0] * s[6] + p[1][1] * s[7] + p[1][2] * s[8];
        prm[4] = p[2][0] * s[6] + p[2][1] * s[7] + p[2][2] * s[8];
        prm[2] = p[0][0] * s[9] + p[0][1] * s[10] + p[0][2] * s[11];
        prm[3] = p[1][0] * s[9] + p[1][1] * s[10] + p[1][2] * s[11];
        prm[5] = p[2][0] * s[9] + p[2][1] * s[10] + p[2][2] * s[11];
      }
      if (max_iter < 1) {
        ok = true;
        break;
      }
      // remove_outliers, AffineParameters.py:134-159
      int dropped = 0;
      for (int64_t j0 = a + lane; j0 < e; j0 += (int64_t)G * kAffU) {
        float fx[kAffU], fy[kAffU], fu[kAffU], fw[kAffU];
        uint8_t al[kAffU];
#pragma unroll
        for (int t = 0; t < kAffU; ++t) {
          const int64_t j = j0 + (int64_t)t * G;
          const int64_t jc = j < e ? j : j0;
          al[t] = j < e ? alive[jc] : 0;
          fx[t] = mx[jc];
          fy[t] = my[jc];
          fu[t] = qx[jc];
          fw[t] = qy[jc];
        }
#pragma unroll
        for (int t = 0; t < kAffU; ++t) {
          if (!al[t]) continue;
          const double x = fx[t], y = fy[t];
          // np.matmul(M, X) + T (AffineParameters.py:145-146) rounded as this host's numpy
          // does (option affine_fma, set by the Python layer from a probe of np.matmul):
          // 1 = fma(m1, x, m2 y) (OpenBLAS dgemv on an FMA CPU), 2 = fma(m2, y, m1 x),
          // 0 = m1 x + m2 y
          const double up = (mxfma == 1   ? fma(prm[0], x, prm[1] * y)
                             : mxfma == 2 ? fma(prm[1], y, prm[0] * x)
                                          : prm[0] * x + prm[1] * y) + prm[4];
          const double vp = (mxfma == 1   ? fma(prm[2], x, prm[3] * y)
                             : mxfma == 2 ? fma(prm[3], y, prm[2] * x)
                                          : prm[2] * x + prm[3] * y) + prm[5];
          if (fabs(up - (double)fu[t]) > xref || fabs(vp - (double)fw[t]) > yref) {
            alive[j0 + (int64_t)t * G] = 0;
            ++dropped;
          }
        }
      }
      dropped = group_sum_i<G>(dropped);
      n -= dropped;
      if (n < thr) {  // main.py:152
        ok = false;
        break;
      }
      ok = true;
      if (dropped == 0) break;  // main.py:151 fixed point
    }
    if (lane == 0 && live) {
      surv[v] = ok ? 1 : 0;
      votes[v] = (int32_t)n;
      for (int k = 0; k < 6; ++k) params[6 * v + k] = prm[k];
    }
  }
}

__global__ __launch_bounds__(256) void affine_kernel(
    int64_t nb_host, const uint32_t* __restrict__ nb_dev, const int64_t* __restrict__ off,
    const float* __restrict__ mx, const float* __restrict__ my, const float* __restrict__ qx,
    const float* __restrict__ qy, const int32_t* __restrict__ isig, int qw, int qh,
    const int32_t* __restrict__ bwh, double xf, double yf, int thr, int max_iter,
    const double* __restrict__ params_in,
    uint8_t* __restrict__ surv, int32_t* __restrict__ votes, double* __restrict__ params,
    uint8_t* __restrict__ alive, int mxfma) {
  constexpr int G = kAffG;
  affine_groups<G>((int64_t)blockIdx.x * (blockDim.x / G) + threadIdx.x / G,
                   (int64_t)gridDim.x * (blockDim.x / G), nb_host, nb_dev, off, mx, my, qx, qy,
                   isig, qw, qh, bwh, xf, yf, thr, max_iter, params_in, surv, votes, params, alive,
                   mxfma);
}

// The PoseBin means (blocks 0..nM-1) beside the affine verification (blocks nM..), one wave
// per bin each -- independent stages, so one launch on the context stream instead of two
// serial ones there or a fork to the side stream and back (the fused one-image path, and the
// staged path when the context has nothing to overlap).  The means go first: their serial
// chains are the longer stage, and blocks are dispatched in index order.
__global__ __launch_bounds__(64) void means_affine_kernel(
    int nM, const uint32_t* __restrict__ scal, const int64_t* __restrict__ voff,
    const int32_t* __restrict__ members, const double* __restrict__ pose,
    const int2* __restrict__ msize, const double* __restrict__ rtab, double* __restrict__ means,
    const float* __restrict__ mx, const float* __restrict__ my, const float* __restrict__ qx,
    const float* __restrict__ qy, const int32_t* __restrict__ isig, int qw, int qh, double xf,
    double yf, int thr, uint8_t* __restrict__ surv, int32_t* __restrict__ votes,
    double* __restrict__ params, uint8_t* __restrict__ alive, int mxfma) {
  __shared__ double xs[7][kMeansB];
  if ((int)blockIdx.x < nM)
    means_wave(blockIdx.x, nM, xs, scal, voff, members, pose, msize, rtab, means);
  else
    affine_groups<64>(blockIdx.x - nM, gridDim.x - nM, 0, scal, voff, mx, my, qx, qy, isig, qw, qh,
                      nullptr, xf, yf, thr, 1 << 30, nullptr, surv, votes, params, alive, mxfma);
}

}  // namespace

// ---------------------------------------------------------------------------------------
static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
static Bins ctx_bins(const sod_ctx* c) { return Bins{c->bins[0], c->bins[1], c->bins[2], c->bins[3]}; }
// image of each query when a batch of query images is declared (nullptr: one image)
static const int* qimg_p(const sod_ctx* c) { return c->n_qimg ? c->qimg.p : nullptr; }

int sod_build_sigma_lut(sod_ctx* ctx, int32_t bs) {
  // HTHF:66-70 evaluated with the same libm calls CPython's math.log(x, 2) makes:
  // log(x) / log(2.0), then / (2*(n_oct-1)+0.5) * bins, int() truncation, clamp.
  int32_t lut[kSigmaLutSize];
  for (int k = -kSigmaLutHalf; k <= kSigmaLutHalf; ++k) {
    const double s = ldexp(1.0, k);
    const double lg = log(s) / log(2.0);
    const double v = lg / 6.5 * (double)bs;
    long long i = (long long)v;
    if (i < 0) i = 0;
    if (i > bs - 1) i = bs - 1;
    lut[k + kSigmaLutHalf] = (int32_t)i;
  }
  SOD_TRY(sod_reserve(ctx, ctx->sig_lut, kSigmaLutSize));
  SOD_HIP(ctx, hipMemcpyAsync(ctx->sig_lut.p, lut, sizeof(lut), hipMemcpyHostToDevice, ctx->stream));
  // the host array dies with this frame: make the copy complete before returning
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  return SOD_OK;
}

int launch_pose_batch(sod_ctx* ctx, int64_t n, const float* mx, const float* my, const float* ma,
                      const int32_t* mo, const float* qx, const float* qy, const float* qa,
                      const int32_t* qo, const double* cx, const double* cy, double* pose,
                      int32_t* idx, double* grec, uint32_t* gstat) {
  const int bs = 256;
  hipLaunchKernelGGL(pose_batch_kernel, dim3((unsigned)cdiv(n, bs)), dim3(bs), 0, ctx->stream, n,
                     mx, my, ma, mo, qx, qy, qa, qo, cx, cy, ctx->qh, ctx->qw, ctx_bins(ctx),
                     ctx->sig_lut.p, pose, idx, ctx->trig_exact ? nullptr : grec, gstat);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

// Does the host's libm compute sin / cos as glibc_trig.h does (x86_64 glibc, FMA variant)?
// 20 000 angles in [0, 2 pi) plus branch edges, called through volatile pointers (a compiler
// may fold sin(x), cos(x) into sincos(), whose last bits differ).  The non-FMA variants
// differ from the FMA one in ~0.07 % of angles, so a different libm shows ~14 differences.
bool sod_host_trig_matches_device() {
  static int cached = -1;
  if (cached >= 0) return cached == 1;
  double (*volatile hs)(double) = ::sin;
  double (*volatile hc)(double) = ::cos;
  uint64_t st = 0x9E3779B97F4A7C15ull;
  bool ok = true;
  for (int i = 0; i < 20000 && ok; ++i) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    double x = (double)(st >> 11) * 0x1p-53 * 6.283185307179586;
    if (i < 8) x = (const double[]){0.126, 0.855468749, 0.85546875, 2.4262652397, 2.42626524,
                                    3.141592653589793, 1.5707963267948966, 6.28318530717958}[i];
    ok = gtrig::ubits(hs(x)) == gtrig::ubits(gtrig::sin(x)) &&
         gtrig::ubits(hc(x)) == gtrig::ubits(gtrig::cos(x));
  }
  cached = ok ? 1 : 0;
  return ok;
}

// the device's glibc sin / cos of n angles (test hook: sod_glibc_sincos)
namespace {
__global__ void glibc_sincos_kernel(int64_t n, const double* __restrict__ x, double* __restrict__ s,
                                    double* __restrict__ c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  s[i] = gtrig::sin(x[i]);
  c[i] = gtrig::cos(x[i]);
}
}  // namespace

int launch_glibc_sincos(sod_ctx* ctx, int64_t n, const double* x, double* s, double* c) {
  hipLaunchKernelGGL(glibc_sincos_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, ctx->stream,
                     n, x, s, c);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_bin_index_batch(sod_ctx* ctx, int64_t n, const double* pose, int32_t* idx) {
  const int bs = 256;
  hipLaunchKernelGGL(bin_index_batch_kernel, dim3((unsigned)cdiv(n, bs)), dim3(bs), 0, ctx->stream,
                     n, pose, ctx->qh, ctx->qw, ctx_bins(ctx), ctx->sig_lut.p, idx);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

// the next parity of a double-buffered set: usable once the means that read it are done
// (no wait when the stream already waited for that launch or a later one, or it is done)
static int next_parity(sod_ctx* ctx, int& par, hipEvent_t (&ev)[2], uint64_t (&id)[2]) {
  par ^= 1;
  if (id[par] == 0 || id[par] <= ctx->means_waited) return SOD_OK;
  const hipError_t q = hipEventQuery(ev[par]);
  if (q != hipSuccess) {
    if (q != hipErrorNotReady) SOD_HIP(ctx, q);
    (void)hipGetLastError();   // hipErrorNotReady is an answer, not an error
    SOD_HIP(ctx, hipStreamWaitEvent(ctx->stream, ev[par], 0));
  }
  ctx->means_waited = id[par];
  return SOD_OK;
}

static int mark_read(sod_ctx* ctx, hipStream_t s, int par, hipEvent_t (&ev)[2], uint64_t (&id)[2]) {
  if (!ev[par]) SOD_HIP(ctx, hipEventCreateWithFlags(&ev[par], hipEventDisableTiming));
  SOD_HIP(ctx, hipEventRecord(ev[par], s));
  id[par] = ctx->means_id;
  return SOD_OK;
}

// hist_kernel over the current window: one work-group per (bin slab, query chunk)
static int launch_hist(sod_ctx* ctx) {
  const int64_t nq = sod_win_n(ctx);
  const int64_t nchunk = cdiv(nq, kChunk);
  dim3 grid((unsigned)cdiv(ctx->nbins, kSlab), (unsigned)nchunk);
  const int* rng = nullptr;
  if (ctx->n_qimg) {
    // a chunk of queries spans a few consecutive images: only their bin slabs
    std::vector<int32_t> r((size_t)nchunk * 2);
    int64_t span = 1;
    for (int64_t c = 0; c < nchunk; ++c) {
      const int64_t qa = c * kChunk, qb = std::min(nq, qa + kChunk) - 1;
      auto img_of = [&](int64_t q) {
        return (int64_t)(std::upper_bound(ctx->qoff_h.begin(), ctx->qoff_h.end(), (int32_t)q) -
                         ctx->qoff_h.begin()) - 1;
      };
      r[2 * c] = (int32_t)((img_of(qa) * ctx->nbins1) / kSlab);
      r[2 * c + 1] = (int32_t)(((img_of(qb) + 1) * ctx->nbins1 - 1) / kSlab);
      span = std::max<int64_t>(span, r[2 * c + 1] - r[2 * c] + 1);
    }
    SOD_TRY(sod_reserve(ctx, ctx->hist_rng, r.size()));
    SOD_HIP(ctx, hipMemcpyAsync(ctx->hist_rng.p, r.data(), r.size() * 4, hipMemcpyHostToDevice,
                                ctx->stream));
    SOD_HIP(ctx, sod_stream_sync(ctx->stream));   // r is a host temporary
    grid.x = (unsigned)span;
    rng = ctx->hist_rng.p;
  }
  hipLaunchKernelGGL(hist_kernel, grid, dim3(kHistThreads), 0, ctx->stream, nq, ctx->basekey.p,
                     ctx->vmask.p, ctx_bins(ctx), ctx->nbins, qimg_p(ctx), ctx->nbins1, rng,
                     ctx->counts.p, ctx->first.p, ctx->gstat.p);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

static int guard_reserve(sod_ctx* ctx, int64_t n) {
  SOD_TRY(sod_reserve(ctx, ctx->grec, (size_t)n * kGuardRec));
  if (!ctx->gstat.p) {   // append counter + handed-over count: zero before the first launch
    SOD_TRY(sod_reserve(ctx, ctx->gstat, 2));
    SOD_HIP(ctx, hipMemsetAsync(ctx->gstat.p, 0, 8, ctx->stream));
  }
  return SOD_OK;
}

int launch_hough(sod_ctx* ctx, int64_t own_lo, int64_t own_hi) {
  const int64_t nq = sod_win_n(ctx), q0 = sod_win0(ctx);
  std::swap(ctx->pose, ctx->pose_b);
  std::swap(ctx->msize, ctx->msize_b);
  SOD_TRY(next_parity(ctx, ctx->hpar, ctx->ev_hread, ctx->hread_id));
  SOD_TRY(sod_reserve(ctx, ctx->pose, (size_t)nq * 4));
  SOD_TRY(sod_reserve(ctx, ctx->basekey, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->vmask, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->msize, (size_t)nq * 2));
  SOD_TRY(sod_reserve(ctx, ctx->counts, (size_t)ctx->nbins));
  SOD_TRY(sod_reserve(ctx, ctx->first, (size_t)ctx->nbins));
  SOD_TRY(guard_reserve(ctx, nq));
  const int bs = 256;
  // one thread per query, and enough of them to clear the histogram in a few passes
  const int64_t pgrid = std::max<int64_t>(cdiv(nq, bs), std::min<int64_t>(cdiv(ctx->nbins, 4 * bs), 4096));
  hipLaunchKernelGGL(pose_kernel, dim3((unsigned)pgrid), dim3(bs), 0, ctx->stream, nq,
                     ctx->good.p + q0, ctx->idx1.p + q0, ctx->qx.p + q0, ctx->qy.p + q0,
                     ctx->qang.p + q0, ctx->qoct.p + q0,
                     ctx->mx.p, ctx->my.p, ctx->mang.p, ctx->moct.p, ctx->mimg.p, ctx->cent.p,
                     ctx->qh, ctx->qw, qimg_p(ctx), ctx->n_qimg ? ctx->qshape.p : nullptr,
                     ctx_bins(ctx), ctx->sig_lut.p, own_lo, own_hi, ctx->pose.p,
                     ctx->basekey.p, ctx->vmask.p, ctx->nbins, ctx->counts.p, ctx->first.p,
                     ctx->isize.p, reinterpret_cast<int2*>(ctx->msize.p),
                     ctx->trig_exact ? nullptr : ctx->grec.p, ctx->gstat.p);
  SOD_HIP(ctx, hipGetLastError());
  SOD_TRY(launch_hist(ctx));
  ctx->guard_done = ctx->trig_exact;   // nothing listed: no read-back before the results
  if (ctx->trig_exact) ctx->guard_flagged = ctx->guard_patched = 0;   // (not a stale count)
  ctx->hist_dense = true;
  return SOD_OK;
}

void sod_guard_host_pose(const double r[8], const int32_t bins[4], double* x, double* y,
                         int32_t* ix, int32_t* iy) {
  // HTHF:31-35 with the libm cos / sin CPython's math module calls (glibc), then HTHF:49-58;
  // one rounding per operation (this file is built with -ffp-contract=off)
  const double tx = r[1], ty = r[2], a = r[3];
  const double ca = std::cos(a), sa = std::sin(a);
  *x = (ca * tx - sa * ty) + r[4];
  *y = (sa * tx + ca * ty) + r[5];
  const int H = (int)r[6], W = (int)r[7];
  *ix = xy_index((*x * bins[0]) / W, bins[0]);
  *iy = xy_index((*y * bins[1]) / H, bins[1]);
}

// The x / y PoseBin means of valid bins vbin[0..nb) redone on the host: each member's pose
// x, y with glibc cos / sin (the calls main.py's math.cos / math.sin make, HTHF:31-32) in the
// reference's expression order, then the running mean of PoseBin.py:45-51 -- so they are the
// reference's values bit for bit, where the device's cos / sin may differ by an ulp.  Written
// to means6[6 i + 0 / 1] (the other four means never involve a transcendental: exact already).
int sod_exact_xy_means(sod_ctx* ctx, const int32_t* vbin, int nb, double* means6) {
  if (nb <= 0) return SOD_OK;
  int64_t V, M;
  SOD_TRY(sod_valid_counts(ctx, &V, &M));
  std::vector<int64_t> off((size_t)V + 1);
  SOD_HIP(ctx, hipMemcpyAsync(off.data(), ctx->voff.p, off.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  // bin list and record offsets up (one upload), records gathered on the device, down into a
  // pinned buffer; the buffers stay with the context (a hipFree per call synchronises the
  // device and cost as much as the rest)
  std::vector<int64_t> up((size_t)nb * 2 + 1);   // [roff 0..nb] [vb as int64 0..nb-1]
  up[0] = 0;
  for (int i = 0; i < nb; ++i) {
    const int64_t v = vbin[i];
    if (v < 0 || v >= V) return sod_fail(ctx, SOD_EINVAL, "valid-bin index out of range");
    up[(size_t)i + 1] = up[(size_t)i] + (off[(size_t)v + 1] - off[(size_t)v]);
  }
  const int64_t n = up[(size_t)nb];
  if (!n) return SOD_OK;
  SOD_TRY(sod_reserve(ctx, ctx->xr_idx, (size_t)nb * 3 + 2));   // roff (nb+1 int64) + vb (nb int32)
  SOD_TRY(sod_reserve(ctx, ctx->xr_rec, (size_t)n * 5));
  if (ctx->xr_host_n < (size_t)n * 5) {
    if (ctx->xr_host) (void)hipHostFree(ctx->xr_host);
    ctx->xr_host = nullptr;
    ctx->xr_host_n = 0;
    SOD_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->xr_host), (size_t)n * 5 * 8, hipHostMallocDefault));
    ctx->xr_host_n = (size_t)n * 5;
  }
  int64_t* droff = reinterpret_cast<int64_t*>(ctx->xr_idx.p);
  int32_t* dvb = reinterpret_cast<int32_t*>(droff + nb + 1);
  std::vector<int32_t> vb32(vbin, vbin + nb);
  SOD_HIP(ctx, hipMemcpyAsync(droff, up.data(), ((size_t)nb + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(dvb, vb32.data(), (size_t)nb * 4, hipMemcpyHostToDevice, ctx->stream));
  const int64_t q0 = sod_win0(ctx);
  hipLaunchKernelGGL(pose_rec_bins_kernel, dim3((unsigned)nb), dim3(256), 0, ctx->stream, nb, dvb,
                     droff, ctx->voff.p, ctx->members.p, ctx->idx1.p + q0, ctx->qx.p + q0,
                     ctx->qy.p + q0, ctx->qang.p + q0, ctx->qoct.p + q0, ctx->mx.p, ctx->my.p,
                     ctx->mang.p, ctx->moct.p, ctx->mimg.p, ctx->cent.p, ctx->xr_rec.p);
  SOD_HIP(ctx, hipGetLastError());
  SOD_HIP(ctx, hipMemcpyAsync(ctx->xr_host, ctx->xr_rec.p, (size_t)n * 5 * 8, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  const double* rec = ctx->xr_host;
  std::vector<size_t> j0((size_t)nb + 1, 0);
  for (int i = 0; i <= nb; ++i) j0[(size_t)i] = (size_t)up[(size_t)i];
  // bins are independent: up to 16 host threads over bin ranges of about equal member counts (the
  // two libm calls per member dominate: ~2 ms for C3's survivors on one thread)
  auto run = [&](int b0, int b1) {
    for (int i = b0; i < b1; ++i) {
      double mxv = 0.0, myv = 0.0;
      for (size_t j = j0[(size_t)i]; j < j0[(size_t)i + 1]; ++j) {
        const double* r = rec + 5 * j;
        const double ca = std::cos(r[2]), sa = std::sin(r[2]);
        const double x = (ca * r[0] - sa * r[1]) + r[3];   // HTHF:31, :34
        const double y = (sa * r[0] + ca * r[1]) + r[4];   // HTHF:32, :35
        const size_t t = j - j0[(size_t)i];
        if (t == 0) {
          mxv = x;
          myv = y;
        } else {                                         // PoseBin.py:45-51, n = votes so far
          const double nn = (double)t;
          mxv = (mxv * nn + x) / (nn + 1.0);
          myv = (myv * nn + y) / (nn + 1.0);
        }
      }
      means6[6 * i + 0] = mxv;
      means6[6 * i + 1] = myv;
    }
  };
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nt = (int)std::min<size_t>({(size_t)16, (size_t)hw, (size_t)nb, (size_t)n / 2048 + 1});
  if (nt <= 1) {
    run(0, nb);
    return SOD_OK;
  }
  std::vector<std::thread> th;
  int b = 0;
  for (int k = 0; k < nt && b < nb; ++k) {
    const size_t goal = (size_t)n * (size_t)(k + 1) / (size_t)nt;
    int e = b + 1;
    while (e < nb && j0[(size_t)e] < goal) ++e;
    if (k == nt - 1) e = nb;
    th.emplace_back(run, b, e);
    b = e;
  }
  for (auto& t : th) t.join();
  return SOD_OK;
}

int sod_guard_resolve(sod_ctx* ctx) {
  if (ctx->guard_done || !ctx->houghed) return SOD_OK;
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  // every copy here is ordered on the context stream and waited for on it: a null-stream copy
  // would also wait for the matcher stream (CU-masked streams are blocking streams), i.e. for
  // the next step's matcher when the caller reads step N while step N+1 is in flight
  uint32_t n = 0;
  SOD_HIP(ctx, hipMemcpyAsync(&n, ctx->gstat.p + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->guard_flagged = n;
  ctx->guard_patched = 0;
  ctx->guard_flagged_total += n;
  if (n == 0) {
    ctx->guard_done = true;
    return SOD_OK;
  }
  const int64_t nq = sod_win_n(ctx);
  std::vector<double> rec((size_t)n * kGuardRec);
  std::vector<uint32_t> key((size_t)nq);
  SOD_HIP(ctx, hipMemcpyAsync(rec.data(), ctx->grec.p, rec.size() * 8, hipMemcpyDeviceToHost,
                              ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(key.data(), ctx->basekey.p, key.size() * 4, hipMemcpyDeviceToHost,
                              ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  std::vector<int32_t> pq(n);
  std::vector<uint32_t> pkey(n);
  std::vector<double> pxy(2 * (size_t)n);
  int64_t changed = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const double* r = &rec[(size_t)i * kGuardRec];
    const int64_t q = (int64_t)r[0];
    int32_t ix, iy;
    sod_guard_host_pose(r, ctx->bins, &pxy[2 * i], &pxy[2 * i + 1], &ix, &iy);
    pq[i] = (int32_t)q;
    pkey[i] = (key[q] & 0xFFFF0000u) | (uint32_t)ix | ((uint32_t)iy << 8);
    changed += pkey[i] != key[q];
  }
  // every listed match takes the host's x, y (and key); the histogram and the stages after
  // it are done again only when a bin changed
  DevBuf<int32_t> dq;
  DevBuf<uint32_t> dk;
  DevBuf<double> dxy;
  int rc = sod_reserve(ctx, dq, n);
  if (rc == SOD_OK) rc = sod_reserve(ctx, dk, n);
  if (rc == SOD_OK) rc = sod_reserve(ctx, dxy, 2 * (size_t)n);
  // (the host vectors outlive the stream synchronisation below)
  if (rc == SOD_OK &&
      (hipMemcpyAsync(dq.p, pq.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
       hipMemcpyAsync(dk.p, pkey.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
       hipMemcpyAsync(dxy.p, pxy.data(), (size_t)n * 16, hipMemcpyHostToDevice, ctx->stream) != hipSuccess))
    rc = sod_fail(ctx, SOD_EHIP, "guard patch upload failed");
  if (rc == SOD_OK) {
    hipLaunchKernelGGL(guard_patch_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, ctx->stream,
                       (int)n, dq.p, dk.p, dxy.p, ctx_bins(ctx), ctx->basekey.p, ctx->vmask.p,
                       ctx->pose.p);
    if (hipGetLastError() != hipSuccess) rc = sod_fail(ctx, SOD_EHIP, "guard_patch_kernel launch");
  }
  if (rc == SOD_OK && changed) {
    // the all-reduced histogram of a sharded run is rebuilt here from every rank's votes
    // (each rank holds every good match and the whole keypoint table)
    hipLaunchKernelGGL(own_all_kernel, dim3((unsigned)std::min<int64_t>(cdiv(nq, 256), 1024)),
                       dim3(256), 0, ctx->stream, nq, ctx->vmask.p);
    if (hipGetLastError() != hipSuccess) rc = sod_fail(ctx, SOD_EHIP, "own_all_kernel launch");
    if (rc == SOD_OK) rc = sod_reserve(ctx, ctx->counts, (size_t)ctx->nbins);
    if (rc == SOD_OK) rc = sod_reserve(ctx, ctx->first, (size_t)ctx->nbins);
    if (rc == SOD_OK &&
        (hipMemsetAsync(ctx->counts.p, 0, (size_t)ctx->nbins * 4, ctx->stream) != hipSuccess ||
         hipMemsetAsync(ctx->first.p, 0xFF, (size_t)ctx->nbins * 4, ctx->stream) != hipSuccess))
      rc = sod_fail(ctx, SOD_EHIP, "guard histogram reset failed");
    if (rc == SOD_OK) rc = launch_hist(ctx);
    if (rc == SOD_OK) ctx->hist_dense = true;
    if (rc == SOD_OK && ctx->selected) rc = launch_select(ctx, ctx->vote_thr);
    if (rc == SOD_OK && ctx->affined) rc = launch_affine_gather(ctx);
    if (rc == SOD_OK && ctx->affined)
      rc = launch_affine(ctx, 0, true, ctx->voff.p, ctx->amx.p, ctx->amy.p, ctx->aqx.p, ctx->aqy.p,
                         ctx->aisig.p, ctx->aff_qw, ctx->aff_qh, ctx->n_qimg ? ctx->bwh.p : nullptr,
                         ctx->aff_xf, ctx->aff_yf, ctx->aff_thr, 1 << 30, nullptr, ctx->surv.p,
                         ctx->fvotes.p, ctx->params.p, ctx->alive.p, ctx->scal.p);
  }
  if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
    rc = sod_fail(ctx, SOD_EHIP, "guard re-run failed");
  (void)sod_stream_sync(ctx->stream);
  sod_release(dq);
  sod_release(dk);
  sod_release(dxy);
  SOD_TRY(rc);
  if (ctx->side_pending) {   // the re-done PoseBin means: joined like every result read
    SOD_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    ctx->side_pending = false;
    ctx->means_waited = ctx->means_id;
  }
  ctx->guard_patched = changed;
  ctx->guard_patched_total += changed;
  ctx->guard_done = true;
  return SOD_OK;
}

static int run_compaction(sod_ctx* ctx, uint32_t thr, uint32_t* out, uint32_t* total_slot,
                          uint32_t* vidx) {
  const int64_t nq = sod_win_n(ctx);
  const int64_t nblk = std::max<int64_t>(1, cdiv(nq, kSelThreads));
  if (ctx->selstat.n < (size_t)nblk) {   // look-back words: zero = never published
    SOD_TRY(sod_reserve(ctx, ctx->selstat, (size_t)nblk));
    SOD_HIP(ctx, hipMemsetAsync(ctx->selstat.p, 0, ctx->selstat.n * 8, ctx->stream));
  }
  if (!ctx->selticket.p) {   // block tickets: a counter that is never reset
    SOD_TRY(sod_reserve(ctx, ctx->selticket, 1));
    SOD_HIP(ctx, hipMemsetAsync(ctx->selticket.p, 0, 8, ctx->stream));
    ctx->sel_tickets = 0;
  }
  ctx->sel_epoch = ctx->sel_epoch >= (1u << 30) - 1 ? 1u : ctx->sel_epoch + 1;
  hipLaunchKernelGGL(select_kernel, dim3((unsigned)nblk), dim3(kSelThreads), 0, ctx->stream, nq,
                     ctx->basekey.p, ctx->vmask.p, ctx->counts.p, ctx->first.p, ctx_bins(ctx),
                     qimg_p(ctx), ctx->nbins1, thr, ctx->selstat.p, ctx->sel_epoch,
                     ctx->selticket.p, (unsigned long long)ctx->sel_tickets, out, vidx,
                     total_slot);
  ctx->sel_tickets += (uint64_t)nblk;
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

static int launch_members_multi(sod_ctx* ctx, uint32_t thr, int64_t nq);
static int launch_means(sod_ctx* ctx, bool on_main = false);
// option select_multi = 1: small windows take the multi-kernel path too (parity tests of both)
static bool select_multi_forced(const sod_ctx* ctx) { return ctx->opt.select_multi == 1; }

int launch_select(sod_ctx* ctx, int32_t thr, bool may_defer_means) {
  const int64_t nq = sod_win_n(ctx);
  std::swap(ctx->scal, ctx->scal_b);
  std::swap(ctx->voff, ctx->voff_b);
  std::swap(ctx->members, ctx->members_b);
  std::swap(ctx->means, ctx->means_b);
  SOD_TRY(next_parity(ctx, ctx->spar, ctx->ev_sread, ctx->sread_id));
  ctx->gathered = false;
  if (thr < 1) thr = 1;  // a bin exists only once voted for
  ctx->vmax = std::max<int64_t>(1, std::min<int64_t>(ctx->nbins, 16 * nq));
  ctx->mmax = std::max<int64_t>(1, 16 * nq);
  SOD_TRY(sod_reserve(ctx, ctx->scal, 4));
  SOD_TRY(sod_reserve(ctx, ctx->vbin, (size_t)ctx->vmax));
  SOD_TRY(sod_reserve(ctx, ctx->voff, (size_t)ctx->vmax + 1));
  SOD_TRY(sod_reserve(ctx, ctx->members, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->means, (size_t)ctx->vmax * 6));
  SOD_TRY(sod_reserve(ctx, ctx->cursor, (size_t)ctx->vmax));
  if (ctx->vidx.n < (size_t)ctx->nbins) {   // bin -> valid index, all-ones between calls
    SOD_TRY(sod_reserve(ctx, ctx->vidx, (size_t)ctx->nbins));
    SOD_HIP(ctx, hipMemsetAsync(ctx->vidx.p, 0xFF, ctx->vidx.n * 4, ctx->stream));
  }
  if (nq <= kSmallQ && !select_multi_forced(ctx)) {   // one work-group, one launch
    hipLaunchKernelGGL(select_small_kernel, dim3(1), dim3(kSmallT), 0, ctx->stream, nq,
                       ctx->basekey.p, ctx->vmask.p, ctx->counts.p, ctx->first.p, ctx_bins(ctx),
                       qimg_p(ctx), ctx->nbins1, (uint32_t)thr, ctx->vbin.p, ctx->scal.p,
                       ctx->voff.p, ctx->members.p);
    SOD_HIP(ctx, hipGetLastError());
  } else {
    SOD_TRY(launch_members_multi(ctx, (uint32_t)thr, nq));
  }
  if (may_defer_means && ctx->mk_main && !ctx->n_qimg) {
    // nothing to overlap (the matcher ran on the context stream): the means wait for the
    // affine enqueue and run in its launch (means_affine_kernel), with no fork to the side
    // stream and join back (~8 us of marker on the context stream, and the reader's
    // cross-stream wait); any other next call runs them alone first (sod_means_flush)
    ctx->means_deferred = true;
    return SOD_OK;
  }
  return launch_means(ctx);
}

// select + members over several work-groups (any window size)
static int launch_members_multi(sod_ctx* ctx, uint32_t thr, int64_t nq) {
  SOD_TRY(run_compaction(ctx, thr, ctx->vbin.p, ctx->scal.p + 0, ctx->vidx.p));
  hipLaunchKernelGGL(member_offsets_kernel, dim3(1), dim3(1024), 0, ctx->stream, ctx->vbin.p,
                     ctx->counts.p, ctx->scal.p, ctx->voff.p, ctx->cursor.p);
  SOD_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(member_fill_lds_kernel, dim3((unsigned)std::max<int64_t>(1, cdiv(nq, 256))),
                     dim3(256), 0, ctx->stream, nq, ctx->scal.p, ctx->basekey.p, ctx->vmask.p,
                     ctx_bins(ctx), qimg_p(ctx), ctx->nbins1, ctx->vidx.p, ctx->voff.p,
                     ctx->cursor.p, ctx->members.p);
  SOD_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(member_order_small_kernel, dim3(std::max(1, ctx->tail_cus() * 8)), dim3(256),
                     0, ctx->stream, ctx->scal.p, ctx->vbin.p, ctx->voff.p, ctx->vidx.p,
                     ctx->members.p);
  SOD_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(member_order_kernel, dim3(std::max(1, ctx->tail_cus() * 2)), dim3(kOrderT), 0,
                     ctx->stream, ctx->scal.p, ctx->voff.p, nq, ctx->members.p);
  SOD_HIP(ctx, hipGetLastError());
  if (nq > kBitQ) {   // beyond the LDS bitmap of member_order_kernel only (a no-op otherwise)
    const int wg = std::max(1, ctx->tail_cus() * 4);
    hipLaunchKernelGGL(members_kernel, dim3(wg), dim3(256), 0, ctx->stream, nq, ctx->scal.p,
                       ctx->vbin.p, ctx->voff.p, ctx->counts.p, ctx->first.p, ctx->basekey.p,
                       ctx->vmask.p, ctx_bins(ctx), qimg_p(ctx), ctx->nbins1, ctx->members.p);
    SOD_HIP(ctx, hipGetLastError());
  }
  return SOD_OK;
}

static int launch_means(sod_ctx* ctx, bool on_main) {
  // PoseBin means depend only on the member lists: they run on the side stream, beside the
  // affine verification and the next step's matcher tail (their inputs are double-buffered);
  // entry points that read results join them (set_dev)
  // 1/(n+1) for every n a member list of this capacity can reach: built once per capacity
  // (a bin's chain reads entry n for its member n)
  const bool new_rtab = ctx->rtab.n < (size_t)ctx->mmax;
  SOD_TRY(sod_reserve(ctx, ctx->rtab, (size_t)ctx->mmax));
  if (on_main) {
    // the fused one-image path: on the context stream, no fork / join events (an event on a
    // dispatch delays the next kernel ~5 us, about what these means take at this size); the
    // buffers it reads are then ordered before every later writer by the stream itself
    if (new_rtab) {
      hipLaunchKernelGGL(recip_table_kernel, dim3((unsigned)std::min<int64_t>(cdiv(ctx->rtab.n, 256), 4096)),
                         dim3(256), 0, ctx->stream, (int64_t)ctx->rtab.n, ctx->rtab.p);
      SOD_HIP(ctx, hipGetLastError());
    }
    hipLaunchKernelGGL(means_kernel, dim3(std::max(1, ctx->tail_cus() * 11)), dim3(64), 0,
                       ctx->stream, ctx->scal.p, ctx->voff.p, ctx->members.p, ctx->pose.p,
                       reinterpret_cast<const int2*>(ctx->msize.p), ctx->rtab.p, ctx->means.p);
    SOD_HIP(ctx, hipGetLastError());
    ++ctx->means_id;
    ctx->hread_id[ctx->hpar] = 0;   // nothing to wait for: stream order
    ctx->sread_id[ctx->spar] = 0;
    return SOD_OK;
  }
  SOD_HIP(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
  SOD_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
  if (new_rtab) {
    hipLaunchKernelGGL(recip_table_kernel, dim3((unsigned)std::min<int64_t>(cdiv(ctx->rtab.n, 256), 4096)),
                       dim3(256), 0, ctx->side, (int64_t)ctx->rtab.n, ctx->rtab.p);
    SOD_HIP(ctx, hipGetLastError());
  }
  // one wave per bin, each a serial f64 chain: as many chains in flight as LDS allows
  // (14 KiB per wave: 11 per CU)
  hipLaunchKernelGGL(means_kernel, dim3(std::max(1, ctx->tail_cus() * 11)), dim3(64), 0, ctx->side,
                     ctx->scal.p, ctx->voff.p, ctx->members.p, ctx->pose.p,
                     reinterpret_cast<const int2*>(ctx->msize.p), ctx->rtab.p, ctx->means.p);
  SOD_HIP(ctx, hipGetLastError());
  ++ctx->means_id;
  SOD_TRY(mark_read(ctx, ctx->side, ctx->hpar, ctx->ev_hread, ctx->hread_id));
  SOD_TRY(mark_read(ctx, ctx->side, ctx->spar, ctx->ev_sread, ctx->sread_id));
  SOD_HIP(ctx, hipEventRecord(ctx->ev_join, ctx->side));
  ctx->side_pending = true;
  return SOD_OK;
}

// The fused one-image path (hough_small_kernel): what launch_hough + launch_select +
// launch_affine_gather do for a window of <= kFusedQ queries of one image on one rank, in one
// launch; the dense histogram is built only if something reads it (sod_hist_dense).
bool sod_hough_small_ok(const sod_ctx* ctx) {
  if (ctx->opt.hough_fused == 0) return false;
  return ctx->nranks <= 1 && !ctx->comm && ctx->n_qimg == 0 && sod_win_n(ctx) <= kFusedQ &&
         sod_win_n(ctx) >= 1;
}

int launch_hough_small(sod_ctx* ctx, int32_t thr) {
  const int64_t nq = sod_win_n(ctx), q0 = sod_win0(ctx);
  // launch_hough's buffers (pose / model sizes alternate per step, see next_parity)
  std::swap(ctx->pose, ctx->pose_b);
  std::swap(ctx->msize, ctx->msize_b);
  SOD_TRY(next_parity(ctx, ctx->hpar, ctx->ev_hread, ctx->hread_id));
  SOD_TRY(sod_reserve(ctx, ctx->pose, (size_t)nq * 4));
  SOD_TRY(sod_reserve(ctx, ctx->basekey, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->vmask, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->msize, (size_t)nq * 2));
  SOD_TRY(guard_reserve(ctx, nq));
  // launch_select's
  std::swap(ctx->scal, ctx->scal_b);
  std::swap(ctx->voff, ctx->voff_b);
  std::swap(ctx->members, ctx->members_b);
  std::swap(ctx->means, ctx->means_b);
  SOD_TRY(next_parity(ctx, ctx->spar, ctx->ev_sread, ctx->sread_id));
  if (thr < 1) thr = 1;
  ctx->vmax = std::max<int64_t>(1, std::min<int64_t>(ctx->nbins, 16 * nq));
  ctx->mmax = std::max<int64_t>(1, 16 * nq);
  SOD_TRY(sod_reserve(ctx, ctx->scal, 4));
  SOD_TRY(sod_reserve(ctx, ctx->vbin, (size_t)ctx->vmax));
  SOD_TRY(sod_reserve(ctx, ctx->voff, (size_t)ctx->vmax + 1));
  SOD_TRY(sod_reserve(ctx, ctx->members, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->means, (size_t)ctx->vmax * 6));
  SOD_TRY(sod_reserve(ctx, ctx->cursor, (size_t)ctx->vmax));   // counts past the LDS copy
  SOD_TRY(sod_reserve(ctx, ctx->vfirst_s, (size_t)ctx->vmax)); // first queries past it
  // launch_affine_gather's
  SOD_TRY(sod_reserve(ctx, ctx->amx, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->amy, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->aqx, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->aqy, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->aisig, (size_t)ctx->vmax));
  hipLaunchKernelGGL(hough_small_kernel, dim3(1), dim3(kFusedT), 0, ctx->stream, nq,
                        ctx->good.p + q0, ctx->idx1.p + q0, ctx->qx.p + q0, ctx->qy.p + q0, ctx->qang.p + q0, ctx->qoct.p + q0, ctx->mx.p, ctx->my.p,
                        ctx->mang.p, ctx->moct.p, ctx->mimg.p, ctx->cent.p, ctx->isize.p, ctx->qh,
                        ctx->qw, ctx_bins(ctx), ctx->sig_lut.p, (uint32_t)thr, ctx->pose.p,
                        ctx->basekey.p, ctx->vmask.p, reinterpret_cast<int2*>(ctx->msize.p),
                        ctx->trig_exact ? nullptr : ctx->grec.p, ctx->gstat.p, ctx->vbin.p,
                        ctx->cursor.p, ctx->vfirst_s.p,
                        ctx->scal.p, ctx->voff.p, ctx->members.p, ctx->amx.p, ctx->amy.p,
                        ctx->aqx.p, ctx->aqy.p, ctx->aisig.p);
  SOD_HIP(ctx, hipGetLastError());
  ctx->guard_done = ctx->trig_exact;
  if (ctx->trig_exact) ctx->guard_flagged = ctx->guard_patched = 0;
  ctx->hist_dense = false;
  ctx->gathered = true;
  // the PoseBin means wait for the affine enqueue, which runs them in the same launch
  // (means_affine_kernel); any other next call runs them alone first (sod_means_flush)
  ctx->means_deferred = true;
  return SOD_OK;
}

int sod_means_flush(sod_ctx* ctx) {
  if (!ctx->means_deferred) return SOD_OK;
  ctx->means_deferred = false;
  return launch_means(ctx, true);
}

// the fused path's affine verification with its deferred PoseBin means in one launch
int launch_means_affine(sod_ctx* ctx, int32_t qw, int32_t qh, double xf, double yf, int32_t thr) {
  ctx->means_deferred = false;
  const bool new_rtab = ctx->rtab.n < (size_t)ctx->mmax;
  SOD_TRY(sod_reserve(ctx, ctx->rtab, (size_t)ctx->mmax));
  if (new_rtab) {
    hipLaunchKernelGGL(recip_table_kernel, dim3((unsigned)std::min<int64_t>(cdiv(ctx->rtab.n, 256), 4096)),
                       dim3(256), 0, ctx->stream, (int64_t)ctx->rtab.n, ctx->rtab.p);
    SOD_HIP(ctx, hipGetLastError());
  }
  const int nA = std::max(1, ctx->tail_cus() * 8), nM = std::max(1, ctx->tail_cus() * 8);
  hipLaunchKernelGGL(means_affine_kernel, dim3((unsigned)(nA + nM)), dim3(64), 0, ctx->stream, nM,
                     ctx->scal.p, ctx->voff.p, ctx->members.p, ctx->pose.p,
                     reinterpret_cast<const int2*>(ctx->msize.p), ctx->rtab.p, ctx->means.p,
                     ctx->amx.p, ctx->amy.p, ctx->aqx.p, ctx->aqy.p, ctx->aisig.p, qw, qh, xf, yf,
                     thr, ctx->surv.p, ctx->fvotes.p, ctx->params.p, ctx->alive.p,
                     ctx->opt.affine_fma);
  SOD_HIP(ctx, hipGetLastError());
  ++ctx->means_id;
  ctx->hread_id[ctx->hpar] = 0;   // stream order, as launch_means(ctx, true)
  ctx->sread_id[ctx->spar] = 0;
  return SOD_OK;
}

// the dense histogram (counts / first touch of every bin) after the fused path, for the
// readers that need it: all bins, another vote threshold, the host exchange
int sod_hist_dense(sod_ctx* ctx) {
  if (ctx->hist_dense) return SOD_OK;
  // the guard reads the record count the fused kernel handed over; hist_kernel hands over
  // again (0 records), so resolve first (a changed bin builds the dense table itself)
  SOD_TRY(sod_guard_resolve(ctx));
  if (ctx->hist_dense) return SOD_OK;
  SOD_TRY(sod_reserve(ctx, ctx->counts, (size_t)ctx->nbins));
  SOD_TRY(sod_reserve(ctx, ctx->first, (size_t)ctx->nbins));
  SOD_HIP(ctx, hipMemsetAsync(ctx->counts.p, 0, (size_t)ctx->nbins * 4, ctx->stream));
  SOD_HIP(ctx, hipMemsetAsync(ctx->first.p, 0xFF, (size_t)ctx->nbins * 4, ctx->stream));
  SOD_TRY(launch_hist(ctx));
  ctx->hist_dense = true;
  return SOD_OK;
}

int launch_all_bins(sod_ctx* ctx) {
  const int64_t bmax = std::max<int64_t>(1, std::min<int64_t>(ctx->nbins, 16 * sod_win_n(ctx)));
  SOD_TRY(sod_reserve(ctx, ctx->scal, 4));
  SOD_TRY(sod_reserve(ctx, ctx->allbin, (size_t)bmax));
  return run_compaction(ctx, 1u, ctx->allbin.p, ctx->scal.p + 2, nullptr);
}

int launch_affine_gather(sod_ctx* ctx) {
  SOD_TRY(sod_reserve(ctx, ctx->amx, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->amy, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->aqx, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->aqy, (size_t)ctx->mmax));
  SOD_TRY(sod_reserve(ctx, ctx->aisig, (size_t)ctx->vmax));
  if (ctx->n_qimg) SOD_TRY(sod_reserve(ctx, ctx->bwh, (size_t)ctx->vmax * 2));
  hipLaunchKernelGGL(affine_gather_kernel, dim3(std::max(1, ctx->tail_cus() * 4)), dim3(256), 0,
                     ctx->stream, ctx->scal.p, ctx->members.p, ctx->idx1.p + sod_win0(ctx),
                     ctx->mx.p, ctx->my.p, ctx->qx.p + sod_win0(ctx), ctx->qy.p + sod_win0(ctx),
                     ctx->vbin.p, ctx_bins(ctx), ctx->nbins1, ctx->n_qimg ? ctx->qshape.p : nullptr,
                     ctx->amx.p, ctx->amy.p, ctx->aqx.p, ctx->aqy.p, ctx->aisig.p, ctx->bwh.p);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

int launch_affine(sod_ctx* ctx, int64_t nb_host, bool count_on_device, const int64_t* offsets,
                  const float* mx, const float* my, const float* qx, const float* qy,
                  const int32_t* isig, int32_t qw, int32_t qh, const int32_t* bwh, double xf,
                  double yf, int32_t thr, int32_t max_iter, const double* params_in, uint8_t* surv,
                  int32_t* votes, double* params, uint8_t* alive, const uint32_t* dev_count) {
  const int wg = std::max(1, ctx->tail_cus() * 4);
  hipLaunchKernelGGL(affine_kernel, dim3(wg), dim3(256), 0, ctx->stream, nb_host,
                     count_on_device ? dev_count : nullptr, offsets, mx, my, qx, qy, isig, qw, qh,
                     bwh, xf, yf, thr, max_iter, params_in, surv, votes, params, alive,
                     ctx->opt.affine_fma);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

