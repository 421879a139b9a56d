// sift.hip -- SIFT detect + describe on the device (the step before
// matching; the reference calls `cv2.SIFT_create().detectAndCompute(gray, None)` at
// main.py:43 and GenerateDatabaseInfo.py:32, OpenCV >= 4.4, default parameters).
//
// The algorithm is OpenCV's (features2d/src/sift.simd.hpp, restated in
// oracle/sift_oracle.c); the arithmetic OpenCV leaves to SIMD/IPP/its math kernels is
// fixed to one definition shared by both sides, so device and oracle agree bit for bit:
// separable blur as row pass then column pass with symmetric-pair sums in increasing
// tap order, no FMA (this file is compiled with -ffp-contract=off), exp / sin / cos /
// 2^y through double-precision Cody-Waite + Taylor kernels, correctly rounded float sqrt,
// OpenCV's fastAtan2 polynomial.
//
// Device pipeline for one image (all on the context stream, one host sync at the end):
//   upscale x2 (exact) -> blur -> per octave: 5 incremental blurs, the column pass also
//   writing the DoG layer -> nearest /2 for the next octave ->
//   extrema (one thread per pixel of DoG layers 1..L, 26-neighbour test, compacted by an
//   atomic counter) -> refine (one thread per candidate: Newton steps, contrast / edge
//   tests, 36-bin orientation histogram, one keypoint per peak) ->
//   order (OpenCV sorts and removes duplicates, so the output order is the sort order and
//   independent of discovery order: rank = number of keypoints before it) ->
//   descriptors (one thread per keypoint, 4x4x8 trilinear histogram).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "sod_internal.h"

namespace {

// Histogram adds (orientation and descriptor): by a whole wave with same-bin lanes applied
// in lane order (wave_order, fast) or by one lane per sample in sample order (ordered, the
// fallback).  The first relies on a property gfx950 shows but does not document -- the
// same-address lanes of one ds_add_f32 are applied in lane order -- so it is compiled for
// gfx950 only and used only after the context's self-check (lds_order_probe_kernel, on the
// first SIFT call) confirmed it on this device; sod_sift_set_lane_order forces the fallback.
#if defined(__gfx950__)
#define SOD_SIFT_WAVE_ORDER_ARCH 1
#else
#define SOD_SIFT_WAVE_ORDER_ARCH 0
#endif
constexpr int kBorder = 5;              // SIFT_IMG_BORDER
constexpr int kMaxInterp = 5;           // SIFT_MAX_INTERP_STEPS
constexpr int kOriBins = 36;            // SIFT_ORI_HIST_BINS
constexpr float kOriSigFctr = 1.5f;     // SIFT_ORI_SIG_FCTR
constexpr float kOriRadius = 3 * kOriSigFctr;
constexpr float kOriPeakRatio = 0.8f;
constexpr int kD = 4, kN = 8;           // SIFT_DESCR_WIDTH, SIFT_DESCR_HIST_BINS
constexpr float kDescrSclFctr = 3.f, kDescrMagThr = 0.2f, kIntDescrFctr = 512.f;
constexpr int kFirstOctave = -1;
constexpr int kMaxOct = 24;
constexpr int kMaxLayers = 8;           // nOctaveLayers + 3 <= kMaxLayers
constexpr int kMaxTaps = 64;

struct Oct {
  int w, h;
  int64_t g;   // offset of layer 0 of this octave in the Gaussian buffer
  int64_t d;   // offset of layer 0 in the DoG buffer
};
struct Pyr {
  Oct o[kMaxOct];
  int n, L;
};

struct Kp {   // final form (firstOctave rescale applied)
  float x, y, size, angle, response;
  int octave;
  int pad0, pad1;
};

// ---- arithmetic shared with oracle/sift_oracle.c --------------------------------------
__host__ __device__ inline int reflect101(int p, int len) {
  if ((unsigned)p < (unsigned)len) return p;
  if (len == 1) return 0;
  do {
    p = p < 0 ? -p : len - 1 - (p - len) - 1;
  } while ((unsigned)p >= (unsigned)len);
  return p;
}

__device__ inline int rnd(float v) { return (int)__builtin_rintf(v); }   // cvRound
__device__ inline int flo(float v) {                                     // cvFloor
  const int i = (int)v;
  return i - (i > v);
}

// e^x: Cody-Waite reduction by ln2 and a Taylor polynomial to r^13 (|r| <= 0.35)
__device__ inline double s_exp(double x) {
  if (x < -740.0) return 0.0;
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double n = __builtin_rint(x * 1.44269504088896338700e+00);
  const double r = (x - n * ln2_hi) - n * ln2_lo;
  double p = 1.0 / 6227020800.0;
  p = p * r + 1.0 / 479001600.0;
  p = p * r + 1.0 / 39916800.0;
  p = p * r + 1.0 / 3628800.0;
  p = p * r + 1.0 / 362880.0;
  p = p * r + 1.0 / 40320.0;
  p = p * r + 1.0 / 5040.0;
  p = p * r + 1.0 / 720.0;
  p = p * r + 1.0 / 120.0;
  p = p * r + 1.0 / 24.0;
  p = p * r + 1.0 / 6.0;
  p = p * r + 0.5;
  p = p * r + 1.0;
  p = p * r + 1.0;
  return __builtin_ldexp(p, (int)n);
}

// sin and cos: reduction by pi/2 (two-part constant), Taylor polynomials to r^21 / r^22
// (|r| <= pi/4: truncation below 1e-24)
__device__ inline void s_sincos(double a, double* sn, double* cs) {
  const double pio2_hi = 1.57079632673412561417e+00, pio2_lo = 6.07710050650619224932e-11;
  const double k = __builtin_rint(a * 6.36619772367581382433e-01);
  const double r = (a - k * pio2_hi) - k * pio2_lo;
  const double r2 = r * r;
  double s = 1.0 / 51090942171709440000.0;   // 1/21!
  s = s * r2 - 1.0 / 121645100408832000.0;   // 1/19!
  s = s * r2 + 1.0 / 355687428096000.0;      // 1/17!
  s = s * r2 - 1.0 / 1307674368000.0;        // 1/15!
  s = s * r2 + 1.0 / 6227020800.0;           // 1/13!
  s = s * r2 - 1.0 / 39916800.0;             // 1/11!
  s = s * r2 + 1.0 / 362880.0;               // 1/9!
  s = s * r2 - 1.0 / 5040.0;                 // 1/7!
  s = s * r2 + 1.0 / 120.0;                  // 1/5!
  s = s * r2 - 1.0 / 6.0;                    // 1/3!
  s = r + r * r2 * s;
  double c = -1.0 / 1124000727777607680000.0;   // 1/22!
  c = c * r2 + 1.0 / 2432902008176640000.0;     // 1/20!
  c = c * r2 - 1.0 / 6402373705728000.0;        // 1/18!
  c = c * r2 + 1.0 / 20922789888000.0;          // 1/16!
  c = c * r2 - 1.0 / 87178291200.0;             // 1/14!
  c = c * r2 + 1.0 / 479001600.0;               // 1/12!
  c = c * r2 - 1.0 / 3628800.0;                 // 1/10!
  c = c * r2 + 1.0 / 40320.0;                   // 1/8!
  c = c * r2 - 1.0 / 720.0;                     // 1/6!
  c = c * r2 + 1.0 / 24.0;                      // 1/4!
  c = c * r2 - 0.5;
  c = 1.0 + r2 * c;
  switch (((int)k) & 3) {
    case 0: *sn = s; *cs = c; break;
    case 1: *sn = c; *cs = -s; break;
    case 2: *sn = -s; *cs = -c; break;
    default: *sn = -c; *cs = s; break;
  }
}

// floor(sqrt(v)) exactly
__host__ __device__ inline int isqrt64(int64_t v) {
  int64_t d = (int64_t)__builtin_sqrt((double)v);
  while (d > 0 && d * d > v) --d;
  while ((d + 1) * (d + 1) <= v) ++d;
  return (int)d;
}

// correctly rounded float sqrt: double estimate, then the exact midpoint tests (a float
// midpoint has 25 significant bits, its square is exact in double)
__device__ inline float sqrt_rn(float x) {
  if (!(x > 0.f)) return x == 0.f ? 0.f : __builtin_nanf("");
  float s = (float)__builtin_sqrt((double)x);
  const double xd = (double)x;
  const unsigned bits = __float_as_uint(s);   // s > 0 and finite
  const float up = __uint_as_float(bits + 1u), dn = __uint_as_float(bits - 1u);
  const double mu = ((double)s + (double)up) * 0.5, md = ((double)s + (double)dn) * 0.5;
  if (mu * mu < xd) s = up;
  else if (md * md > xd) s = dn;
  return s;
}

__device__ inline float fexp(float x) { return (float)s_exp((double)x); }
__device__ inline float fmag(float x, float y) { return sqrt_rn(x * x + y * y); }

// cv::hal::fastAtan2 (degrees), scalar form
__device__ inline float fast_atan2(float y, float x) {
  const float d2r = (float)(180 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * d2r, p3 = -0.3258083974640975f * d2r,
              p5 = 0.1555786518463281f * d2r, p7 = -0.04432655554792128f * d2r;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)2.220446049250313e-16);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)2.220446049250313e-16);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// ---- pyramid kernels ------------------------------------------------------------------
// x2 INTER_LINEAR of an 8-bit image (every value is a multiple of 1/16: exact)
__device__ inline float up_row(const uint8_t* g, int w, int y, int d) {
  const int i = d >> 1;
  const uint8_t* r = g + (size_t)y * w;
  if (d & 1) return i + 1 < w ? 0.75f * r[i] + 0.25f * r[i + 1] : (float)r[i];
  return i > 0 ? 0.25f * r[i - 1] + 0.75f * r[i] : (float)r[i];
}
__global__ void upscale_kernel(const uint8_t* __restrict__ g, int w, int h, float* __restrict__ u) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, d = blockIdx.y;
  if (x >= 2 * w) return;
  const int i = d >> 1;
  float v;
  if (d & 1)
    v = i + 1 < h ? 0.75f * up_row(g, w, i, x) + 0.25f * up_row(g, w, i + 1, x) : up_row(g, w, i, x);
  else
    v = i > 0 ? 0.25f * up_row(g, w, i - 1, x) + 0.75f * up_row(g, w, i, x) : up_row(g, w, i, x);
  u[(size_t)d * 2 * w + x] = v;
}

// row pass: out = k0*x + sum_i k_i * (x[-i] + x[+i]), BORDER_REFLECT_101
__global__ void blur_rows_kernel(const float* __restrict__ src, float* __restrict__ dst, int w,
                                 const float* __restrict__ k, int r) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const float* row = src + (size_t)y * w;
  float s = k[0] * row[x];
  if (x >= r && x + r < w) {
    for (int i = 1; i <= r; ++i) s += k[i] * (row[x - i] + row[x + i]);
  } else {
    for (int i = 1; i <= r; ++i) s += k[i] * (row[reflect101(x - i, w)] + row[reflect101(x + i, w)]);
  }
  dst[(size_t)y * w + x] = s;
}

// column pass; with `dog` it also writes dog = out - prev (the layer the blur started from)
__global__ void blur_cols_kernel(const float* __restrict__ src, float* __restrict__ dst, int w,
                                 int h, const float* __restrict__ k, int r,
                                 const float* __restrict__ prev, float* __restrict__ dog) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  float s = k[0] * src[(size_t)y * w + x];
  if (y >= r && y + r < h) {
    for (int i = 1; i <= r; ++i)
      s += k[i] * (src[(size_t)(y - i) * w + x] + src[(size_t)(y + i) * w + x]);
  } else {
    for (int i = 1; i <= r; ++i)
      s += k[i] * (src[(size_t)reflect101(y - i, h) * w + x] + src[(size_t)reflect101(y + i, h) * w + x]);
  }
  const size_t o = (size_t)y * w + x;
  dst[o] = s;
  if (dog) dog[o] = s - prev[o];
}

// fused separable blur of one kTW x kTH output tile, radius R a template parameter: the
// source tile with an R-pixel halo (rows and columns reflected, BORDER_REFLECT_101) is
// staged in LDS; the row pass (each thread a run of kSeg outputs from a register window)
// writes its results over the source row it read, as the intermediate (one LDS tile per
// work-group: more work-groups per CU) -- a row's runs are 8 lanes of one wave, whose LDS
// reads all precede its writes; the column pass (runs of kSeg down a column) writes the
// output and the DoG = output - source (the source values read before the row pass).  Per output the
// arithmetic is exactly blur_rows_kernel's then blur_cols_kernel's:
// k0*x + sum_{i=1..R} k_i*(x[-i] + x[+i]) in increasing i.
constexpr int kTW = 64, kTH = 32, kSeg = 8, kMaxR = 16;
template <int R>
__global__ __launch_bounds__(256) void blur_tile_kernel(const float* __restrict__ src,
                                                        float* __restrict__ dst, int w, int h,
                                                        const float* __restrict__ kern,
                                                        float* __restrict__ dog) {
  // IP: the LDS row pitch, odd, so the row pass's windows (8 rows x 8 runs per wave) spread
  // over the banks
  constexpr int IW = kTW + 2 * R, IH = kTH + 2 * R, IP = IW | 1, NS = (IW * IH + 255) / 256;
  static_assert(kTW * (kTH / kSeg) == 256, "one column run per thread");
  static_assert(kTW / kSeg == 8 && 64 % (kTW / kSeg) == 0, "a row's runs in one wave");
  __shared__ float in[IH * IP];   // the source tile, then the row pass's output (pitch IP)
  const int x0 = blockIdx.x * kTW, y0 = blockIdx.y * kTH;
  const int tid = threadIdx.x;
  float k[R + 1];
#pragma unroll
  for (int i = 0; i <= R; ++i) k[i] = kern[i];
  const bool interior = x0 >= R && x0 + kTW + R <= w && y0 >= R && y0 + kTH + R <= h;
  // staging: all NS loads of a thread in flight together (a load-then-store loop waits on
  // each load in turn), the tail index clamped
  float sv[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int t = min(tid + 256 * j, IW * IH - 1);
    const int u = t % IW, v = t / IW;
    int gx = x0 - R + u, gy = y0 - R + v;
    if (!interior) {
      gx = reflect101(gx, w);
      gy = reflect101(gy, h);
    }
    sv[j] = src[(size_t)gy * w + gx];
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int t = tid + 256 * j;
    if (t < IW * IH) in[(t / IW) * IP + t % IW] = sv[j];
  }
  __syncthreads();
  // this thread's column run (u, cr): its source values, for the DoG
  const int u = tid % kTW, cr = tid / kTW;
  float dv[kSeg];
#pragma unroll
  for (int o = 0; o < kSeg; ++o) dv[o] = in[(cr * kSeg + o + R) * IP + R + u];
  __syncthreads();   // before any row is overwritten
  // row pass: IH rows x (kTW / kSeg) runs, each row's output over its own source row
  for (int t = tid; t < IH * (kTW / kSeg); t += 256) {   // (wave-uniform trip count per row)
    const int run = t % (kTW / kSeg), v = t / (kTW / kSeg);
    float* row = in + v * IP + run * kSeg;   // window starts R left of the first output
    float win[kSeg + 2 * R];
#pragma unroll
    for (int j = 0; j < kSeg + 2 * R; ++j) win[j] = row[j];
    float res[kSeg];
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      float s = k[0] * win[o + R];
#pragma unroll
      for (int i = 1; i <= R; ++i) s += k[i] * (win[o + R - i] + win[o + R + i]);
      res[o] = s;
    }
    // the row's other lanes read these words too: no write moves above this wave's reads
    asm volatile("" ::: "memory");
#pragma unroll
    for (int o = 0; o < kSeg; ++o) row[o] = res[o];
  }
  __syncthreads();
  // column pass: kTW columns x (kTH / kSeg) runs, one per thread
  {
    const float* col = in + cr * kSeg * IP + u;
    float win[kSeg + 2 * R];
#pragma unroll
    for (int j = 0; j < kSeg + 2 * R; ++j) win[j] = col[j * IP];
    const int x = x0 + u;
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      const int y = y0 + cr * kSeg + o;
      float s = k[0] * win[o + R];
#pragma unroll
      for (int i = 1; i <= R; ++i) s += k[i] * (win[o + R - i] + win[o + R + i]);
      if (x < w && y < h) {
        const size_t oo = (size_t)y * w + x;
        dst[oo] = s;
        if (dog) dog[oo] = s - dv[o];
      }
    }
  }
}

using BlurFn = void (*)(const float*, float*, int, int, const float*, float*);
constexpr BlurFn kBlurFns[kMaxR + 1] = {
    nullptr, blur_tile_kernel<1>, blur_tile_kernel<2>, blur_tile_kernel<3>, blur_tile_kernel<4>,
    blur_tile_kernel<5>, blur_tile_kernel<6>, blur_tile_kernel<7>, blur_tile_kernel<8>,
    blur_tile_kernel<9>, blur_tile_kernel<10>, blur_tile_kernel<11>, blur_tile_kernel<12>,
    blur_tile_kernel<13>, blur_tile_kernel<14>, blur_tile_kernel<15>, blur_tile_kernel<16>};

// OpenCV's test: val >= all 26 neighbours (val > 0) or <= all (val < 0); the 26 loads
// are issued together (max / min of the neighbours, no short-circuit chain of loads)
__device__ inline bool is_extremum(const float* cur, size_t plane, size_t c, int step, float val) {
  float mx = -3.4e38f, mn = 3.4e38f;
#pragma unroll
  for (int dl = -1; dl <= 1; ++dl)
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        if (!dl && !dy && !dx) continue;
        const float v = cur[(ptrdiff_t)plane * dl + (ptrdiff_t)c + (ptrdiff_t)dy * step + dx];
        mx = fmaxf(mx, v);
        mn = fminf(mn, v);
      }
  return val > 0 ? val >= mx : val <= mn;
}

// ---- the small octaves in ONE work-group: from octave o0 (<= kChainPixels pixels) to
// the last, the /2 base, the incremental blurs (row pass, column pass + DoG; the same
// arithmetic as above) on LDS copies of the current layer, each layer also written to the
// pyramid, then the extrema of those octaves.  Replaces ~6 launches per small octave.
constexpr int kChainPixels = 4096;
constexpr int kChainDog = 5;     // DoG layers held in LDS: the chain runs for nOctaveLayers <= 3
constexpr int kTabMax = 64;   // dimensions up to this use an LDS reflection table
// BORDER_REFLECT_101 index for the chain: a table for small dimensions (several
// reflections when the kernel is wider than the image), one reflection otherwise
__device__ inline int refl(int p, int len, const int* tab) {
  if (len <= kTabMax) return tab[p + kMaxR];
  return p < 0 ? -p : (p >= len ? 2 * len - 2 - p : p);
}
// The passes run over runs of kChainSeg consecutive outputs (along x for the row pass, along
// y for the column pass) from a register window of kChainSeg + 2R inputs: ~1/3 the LDS reads
// of one output per thread at R 13.  The window holds the same (reflected) inputs the
// per-tap form reads, and every output is still k0*x + sum_{i=1..R} k_i*(x[-i] + x[+i]) in
// increasing i (blur_rows_kernel / blur_cols_kernel's arithmetic).
constexpr int kChainSeg = 4;
template <int R>
__device__ __forceinline__ void chain_rows(const float* cur, float* T, int w, int h, const float* k, const int* tabx,
                           const int* taby, int tid) {
  const int runs = (w + kChainSeg - 1) / kChainSeg;
  for (int t = tid; t < runs * h; t += 1024) {
    const int y = t / runs, x0 = (t - y * runs) * kChainSeg;
    const float* p = cur + y * w;
    float win[kChainSeg + 2 * R];
    if (x0 >= R && x0 + kChainSeg + R <= w) {
#pragma unroll
      for (int j = 0; j < kChainSeg + 2 * R; ++j) win[j] = p[x0 - R + j];
    } else {
#pragma unroll
      for (int j = 0; j < kChainSeg + 2 * R; ++j)   // (past x + R: feeds no stored output)
        win[j] = p[refl(min(x0 - R + j, w - 1 + R), w, tabx)];
    }
#pragma unroll
    for (int o = 0; o < kChainSeg; ++o) {
      float s = k[0] * win[o + R];
#pragma unroll
      for (int i = 1; i <= R; ++i) s += k[i] * (win[o + R - i] + win[o + R + i]);
      if (x0 + o < w) T[y * w + x0 + o] = s;
    }
  }
}
template <int R>
__device__ __forceinline__ void chain_cols(const float* T, const float* cur, float* nxt, float* dst, float* dg,
                           float* dgl, float* keep, int w, int h, const float* k, const int* tabx,
                           const int* taby, int tid) {
  const int runs = (h + kChainSeg - 1) / kChainSeg;
  for (int t = tid; t < runs * w; t += 1024) {
    const int x = t / runs, y0 = (t - x * runs) * kChainSeg;
    const float* p = T + x;
    float win[kChainSeg + 2 * R];
    if (y0 >= R && y0 + kChainSeg + R <= h) {
#pragma unroll
      for (int j = 0; j < kChainSeg + 2 * R; ++j) win[j] = p[(y0 - R + j) * w];
    } else {
#pragma unroll
      for (int j = 0; j < kChainSeg + 2 * R; ++j)
        win[j] = p[refl(min(y0 - R + j, h - 1 + R), h, taby) * w];
    }
#pragma unroll
    for (int o = 0; o < kChainSeg; ++o) {
      float s = k[0] * win[o + R];
#pragma unroll
      for (int i = 1; i <= R; ++i) s += k[i] * (win[o + R - i] + win[o + R + i]);
      const int y = y0 + o;
      if (y < h) {
        const int tt = y * w + x;
        const float d = s - cur[tt];
        nxt[tt] = s;
        dst[tt] = s;
        dg[tt] = d;
        dgl[tt] = d;
        if (keep) keep[tt] = s;
      }
    }
  }
}
// octaves of at most 1024 pixels: one output per thread, taps read straight from LDS (one
// run per thread either way, and a run's cost is its instruction count); r is a run-time
// value, the arithmetic the same as above
__device__ __forceinline__ void chain_rows1(const float* cur, float* T, int w, int h, int r,
                                            const float* k, const int* tabx, int tid) {
  if (tid >= w * h) return;
  const int y = tid / w, x = tid - y * w;
  const float* p = cur + y * w;
  float s = k[0] * p[x];
  for (int i = 1; i <= r; ++i) s += k[i] * (p[refl(x - i, w, tabx)] + p[refl(x + i, w, tabx)]);
  T[tid] = s;
}
__device__ __forceinline__ void chain_cols1(const float* T, const float* cur, float* nxt, float* dst,
                                            float* dg, float* dgl, float* keep, int w, int h, int r,
                                            const float* k, const int* taby, int tid) {
  if (tid >= w * h) return;
  const int y = tid / w, x = tid - y * w;
  const float* p = T + x;
  float s = k[0] * p[y * w];
  for (int i = 1; i <= r; ++i) s += k[i] * (p[refl(y - i, h, taby) * w] + p[refl(y + i, h, taby) * w]);
  const float d = s - cur[tid];
  nxt[tid] = s;
  dst[tid] = s;
  dg[tid] = d;
  dgl[tid] = d;
  if (keep) keep[tid] = s;
}
#define SOD_CHAIN_CASES(F, ...)                                                         \
  switch (r) {                                                                          \
    case 1: F<1>(__VA_ARGS__); break;   case 2: F<2>(__VA_ARGS__); break;               \
    case 3: F<3>(__VA_ARGS__); break;   case 4: F<4>(__VA_ARGS__); break;               \
    case 5: F<5>(__VA_ARGS__); break;   case 6: F<6>(__VA_ARGS__); break;               \
    case 7: F<7>(__VA_ARGS__); break;   case 8: F<8>(__VA_ARGS__); break;               \
    case 9: F<9>(__VA_ARGS__); break;   case 10: F<10>(__VA_ARGS__); break;             \
    case 11: F<11>(__VA_ARGS__); break; case 12: F<12>(__VA_ARGS__); break;             \
    case 13: F<13>(__VA_ARGS__); break; case 14: F<14>(__VA_ARGS__); break;             \
    case 15: F<15>(__VA_ARGS__); break; default: F<16>(__VA_ARGS__); break;             \
  }


// barrier for LDS traffic only: the pyramid's global stores drain in the background (no
// pass of the chain reads them back)
__device__ inline void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- the small octaves (<= kChainPixels pixels each) in ONE work-group, entirely in LDS:
// the /2 base (from the pyramid for the first, from the LDS copy of layer L after that),
// the incremental blurs (row pass, column pass + DoG), every layer also written to the
// pyramid, and the extrema of each octave from its LDS DoG layers.  Replaces ~7 launches
// per small octave.
__global__ __launch_bounds__(1024) void small_octaves_kernel(float* __restrict__ gauss,
                                                             float* __restrict__ dogs, Pyr P, int o0,
                                                             const float* __restrict__ kern,
                                                             const int* __restrict__ radius,
                                                             float thr, int4* __restrict__ cand,
                                                             unsigned* __restrict__ ncand, int cap) {
  __shared__ float A[kChainPixels], T[kChainPixels], C[kChainPixels], Bl[kChainPixels];
  __shared__ float Dg[kChainDog][kChainPixels];
  __shared__ float kk[kMaxLayers][kMaxTaps];
  __shared__ int tabx[kTabMax + 2 * kMaxR], taby[kTabMax + 2 * kMaxR];
  const int L = P.L, tid = threadIdx.x;
  for (int t = tid; t < kMaxLayers * kMaxTaps; t += 1024) kk[t / kMaxTaps][t % kMaxTaps] = kern[t];
  for (int o = o0; o < P.n; ++o) {
    const Oct& q = P.o[o];
    const int w = q.w, h = q.h, np = w * h;
    float* g0 = gauss + q.g;
    const Oct& pq = P.o[o - 1];
    if (o == o0) {
      const float* base = gauss + pq.g + (size_t)pq.w * pq.h * L;   // written by earlier launches
      for (int t = tid; t < np; t += 1024) {
        const int y = t / w, x = t - y * w;
        A[t] = base[(size_t)(2 * y) * pq.w + 2 * x];
      }
    } else {
      for (int t = tid; t < np; t += 1024) {
        const int y = t / w, x = t - y * w;
        A[t] = Bl[(2 * y) * pq.w + 2 * x];
      }
    }
    for (int t = tid; t < kTabMax + 2 * kMaxR; t += 1024) {
      if (w <= kTabMax) tabx[t] = reflect101(t - kMaxR, w);
      if (h <= kTabMax) taby[t] = reflect101(t - kMaxR, h);
    }
    lds_barrier();
    for (int t = tid; t < np; t += 1024) g0[t] = A[t];
    float* cur = A;
    float* nxt = C;
    for (int i = 1; i < L + 3; ++i) {
      const int r = radius[i];
      if (np <= 1024)
        chain_rows1(cur, T, w, h, r, kk[i], tabx, tid);
      else
        SOD_CHAIN_CASES(chain_rows, cur, T, w, h, kk[i], tabx, taby, tid)
      lds_barrier();
      float* dst = g0 + (size_t)np * i;
      float* dg = dogs + q.d + (size_t)np * (i - 1);
      if (np <= 1024)
        chain_cols1(T, cur, nxt, dst, dg, Dg[i - 1], i == L ? Bl : nullptr, w, h, r, kk[i], taby, tid);
      else
        SOD_CHAIN_CASES(chain_cols, T, cur, nxt, dst, dg, Dg[i - 1], i == L ? Bl : nullptr, w, h,
                        kk[i], tabx, taby, tid)
      lds_barrier();
      float* t2 = cur;
      cur = nxt;
      nxt = t2;
    }
    // extrema of this octave (extrema_all_kernel's test) on the LDS DoG layers
    const int iw = w - 2 * kBorder, ih = h - 2 * kBorder;
    if (iw > 0 && ih > 0) {
      for (int t = tid; t < iw * ih * L; t += 1024) {
        const int layer = t / (iw * ih) + 1, rem = t - (layer - 1) * (iw * ih);
        const int y = rem / iw + kBorder, x = rem - (y - kBorder) * iw + kBorder;
        const float* cur2 = Dg[layer];
        const int c = y * w + x;
        const float val = cur2[c];
        if (!(fabsf(val) > thr)) continue;
        float mx = -3.4e38f, mn = 3.4e38f;
#pragma unroll
        for (int dl = -1; dl <= 1; ++dl)
#pragma unroll
          for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
              if (!dl && !dy && !dx) continue;
              const float v = Dg[layer + dl][c + dy * w + dx];
              mx = fmaxf(mx, v);
              mn = fminf(mn, v);
            }
        if (!(val > 0 ? val >= mx : val <= mn)) continue;
        const unsigned i = atomicAdd(ncand, 1u);
        if (i < (unsigned)cap) cand[i] = make_int4(o, layer, y, x);
      }
    }
    lds_barrier();
  }
}

__global__ void down2_kernel(const float* __restrict__ src, int sw, float* __restrict__ dst, int dw) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw) return;
  dst[(size_t)y * dw + x] = src[(size_t)(2 * y) * sw + 2 * x];
}

// ---- extrema ------------------------------------------------------------------------
// 3x3x3 extrema of the octaves above the small-octave chain in ONE launch: block b of the
// flat grid is block (b - first[o]) of octave o's (256-pixel x blocks, rows, layers) grid
// (candidates are appended in any order: the keypoint sort orders them)
constexpr int kExtRows = 8;   // rows per work-group: their centre loads are in flight together
struct ExtGrid {
  int first[kMaxOct + 1];   // first flat block of each octave; first[n] = total
  int n;
};
__global__ void extrema_all_kernel(const float* __restrict__ dogs, Pyr P, ExtGrid G, float thr,
                                   int4* __restrict__ cand, unsigned* __restrict__ ncand, int cap) {
  int o = 0;
  while (o + 1 < G.n && (int)blockIdx.x >= G.first[o + 1]) ++o;
  const Oct& q = P.o[o];
  const int bx = (q.w - 2 * kBorder + 255) / 256, rows = q.h - 2 * kBorder;
  const int ry = (rows + kExtRows - 1) / kExtRows;
  const int lb = (int)blockIdx.x - G.first[o];
  const int layer = lb / (bx * ry) + 1, rem = lb % (bx * ry);
  const int x = (rem % bx) * 256 + threadIdx.x + kBorder, y0 = (rem / bx) * kExtRows + kBorder;
  if (x >= q.w - kBorder) return;
  const size_t plane = (size_t)q.w * q.h;
  const float* cur = dogs + q.d + plane * layer;
  float val[kExtRows];
#pragma unroll
  for (int r = 0; r < kExtRows; ++r)   // clamped rows: every load is unconditional
    val[r] = cur[(size_t)min(y0 + r, q.h - kBorder - 1) * q.w + x];
#pragma unroll
  for (int r = 0; r < kExtRows; ++r) {
    const int y = y0 + r;
    if (y >= q.h - kBorder || !(fabsf(val[r]) > thr)) continue;
    if (!is_extremum(cur, plane, (size_t)y * q.w + x, q.w, val[r])) continue;
    const unsigned i = atomicAdd(ncand, 1u);
    if (i < (unsigned)cap) cand[i] = make_int4(o, layer, y, x);
  }
}

// ---- refine + orientation -------------------------------------------------------------
__device__ inline float at(const float* img, int w, int y, int x) { return img[(size_t)y * w + x]; }

__device__ bool adjust_local_extrema(const float* dogs, const Pyr& P, int octv, int& layer,
                                     int& r, int& c, float contrastThreshold,
                                     float edgeThreshold, float sigma, Kp& kpt) {
  const int L = P.L;
  const Oct& q = P.o[octv];
  const size_t plane = (size_t)q.w * q.h;
  const int w = q.w;
  const float img_scale = 1.f / (255 * 1);
  const float deriv_scale = img_scale * 0.5f;
  const float second_deriv_scale = img_scale;
  const float cross_deriv_scale = img_scale * 0.25f;
  float xi = 0, xr = 0, xc = 0, contr = 0;
  int i = 0;
  for (; i < kMaxInterp; i++) {
    const float* img = dogs + q.d + plane * layer;
    const float* prev = img - plane;
    const float* next = img + plane;
    const float dD0 = (at(img, w, r, c + 1) - at(img, w, r, c - 1)) * deriv_scale;
    const float dD1 = (at(img, w, r + 1, c) - at(img, w, r - 1, c)) * deriv_scale;
    const float dD2 = (at(next, w, r, c) - at(prev, w, r, c)) * deriv_scale;
    const float v2 = at(img, w, r, c) * 2;
    const float dxx = (at(img, w, r, c + 1) + at(img, w, r, c - 1) - v2) * second_deriv_scale;
    const float dyy = (at(img, w, r + 1, c) + at(img, w, r - 1, c) - v2) * second_deriv_scale;
    const float dss = (at(next, w, r, c) + at(prev, w, r, c) - v2) * second_deriv_scale;
    const float dxy = (at(img, w, r + 1, c + 1) - at(img, w, r + 1, c - 1) -
                       at(img, w, r - 1, c + 1) + at(img, w, r - 1, c - 1)) * cross_deriv_scale;
    const float dxs = (at(next, w, r, c + 1) - at(next, w, r, c - 1) - at(prev, w, r, c + 1) +
                       at(prev, w, r, c - 1)) * cross_deriv_scale;
    const float dys = (at(next, w, r + 1, c) - at(next, w, r - 1, c) - at(prev, w, r + 1, c) +
                       at(prev, w, r - 1, c)) * cross_deriv_scale;
    // Matx33f::solve(DECOMP_LU): Cramer's rule in float, zero vector when det == 0
    const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs,
                a21 = dys, a22 = dss;
    float det = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) +
                a02 * (a10 * a21 - a20 * a11);
    float X0 = 0, X1 = 0, X2 = 0;
    if (det != 0) {
      det = 1 / det;
      X0 = det * (dD0 * (a11 * a22 - a12 * a21) - a01 * (dD1 * a22 - a12 * dD2) +
                  a02 * (dD1 * a21 - a11 * dD2));
      X1 = det * (a00 * (dD1 * a22 - a12 * dD2) - dD0 * (a10 * a22 - a12 * a20) +
                  a02 * (a10 * dD2 - dD1 * a20));
      X2 = det * (a00 * (a11 * dD2 - dD1 * a21) - a01 * (a10 * dD2 - dD1 * a20) +
                  dD0 * (a10 * a21 - a11 * a20));
    }
    xi = -X2;
    xr = -X1;
    xc = -X0;
    if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
    if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) ||
        fabsf(xc) > (float)(INT_MAX / 3))
      return false;
    c += rnd(xc);
    r += rnd(xr);
    layer += rnd(xi);
    if (layer < 1 || layer > L || c < kBorder || c >= q.w - kBorder || r < kBorder ||
        r >= q.h - kBorder)
      return false;
  }
  if (i >= kMaxInterp) return false;
  {
    const float* img = dogs + q.d + plane * layer;
    const float* prev = img - plane;
    const float* next = img + plane;
    const float dD0 = (at(img, w, r, c + 1) - at(img, w, r, c - 1)) * deriv_scale;
    const float dD1 = (at(img, w, r + 1, c) - at(img, w, r - 1, c)) * deriv_scale;
    const float dD2 = (at(next, w, r, c) - at(prev, w, r, c)) * deriv_scale;
    float t = 0;
    t += dD0 * xc;
    t += dD1 * xr;
    t += dD2 * xi;
    contr = at(img, w, r, c) * img_scale + t * 0.5f;
    if (fabsf(contr) * L < contrastThreshold) return false;
    const float v2 = at(img, w, r, c) * 2.f;
    const float dxx = (at(img, w, r, c + 1) + at(img, w, r, c - 1) - v2) * second_deriv_scale;
    const float dyy = (at(img, w, r + 1, c) + at(img, w, r - 1, c) - v2) * second_deriv_scale;
    const float dxy = (at(img, w, r + 1, c + 1) - at(img, w, r + 1, c - 1) -
                       at(img, w, r - 1, c + 1) + at(img, w, r - 1, c - 1)) * cross_deriv_scale;
    const float tr = dxx + dyy;
    const float dt = dxx * dyy - dxy * dxy;
    if (dt <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * dt)
      return false;
  }
  kpt.x = (c + xc) * (1 << octv);
  kpt.y = (r + xr) * (1 << octv);
  kpt.octave = octv + (layer << 8) + ((int)__builtin_rint(((double)xi + 0.5) * 255) << 16);
  kpt.size = sigma * (float)s_exp((double)((layer + xi) / L) * 0.6931471805599453) * (1 << octv) * 2;
  kpt.response = fabsf(contr);
  return true;
}

// a candidate that passed adjustLocalExtrema: its keypoint (pyramid coordinates) and
// the Gaussian layer / pixel its orientation histogram is taken at
struct Surv {
  Kp k;
  int o, layer, r, c;
};

// one thread per candidate: adjustLocalExtrema
__global__ void refine_kernel(const float* __restrict__ dogs, Pyr P, const int4* __restrict__ cand,
                              const unsigned* __restrict__ ncand, int cap, float contrastThreshold,
                              float edgeThreshold, float sigma, Surv* __restrict__ surv,
                              unsigned* __restrict__ nsurv) {
  const unsigned id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= min(*ncand, (unsigned)cap)) return;
  const int4 cd = cand[id];
  const int o = cd.x;
  int layer = cd.y, r = cd.z, c = cd.w;
  Kp kpt;
  if (!adjust_local_extrema(dogs, P, o, layer, r, c, contrastThreshold, edgeThreshold, sigma, kpt))
    return;
  const unsigned k = atomicAdd(nsurv, 1u);   // at most one survivor per candidate
  surv[k] = Surv{kpt, o, layer, r, c};
}

// one 256-thread block per survivor: calcOrientationHist + one keypoint per histogram
// peak.  The window's samples are computed 256 at a time (one per thread, in OpenCV's
// row-major order), compacted in that order, and added to the LDS histogram by one lane
// in order (LDS operations of a wave retire in order), so every bin sums in OpenCV's order.
constexpr int kOT = 256;
__device__ inline int block_compact_slot(bool ok, int* wcnt, int& total) {
  // position of this thread's item among the block's valid items (thread order)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
  if (lane == 0) wcnt[wave] = __builtin_popcountll(m);
  __syncthreads();
  int base = 0;
  total = 0;
  for (int w2 = 0; w2 < (int)(blockDim.x >> 6); ++w2) {
    base += w2 < wave ? wcnt[w2] : 0;
    total += wcnt[w2];
  }
  return base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__global__ __launch_bounds__(kOT) void orient_kernel(const float* __restrict__ gauss, Pyr P,
                                                     const Surv* __restrict__ surv,
                                                     const unsigned* __restrict__ nsurv, int cap,
                                                     Kp* __restrict__ kps, unsigned* __restrict__ nkp,
                                                     int kcap, int lane_order) {
#if SOD_SIFT_WAVE_ORDER_ARCH
  const bool wave_order = lane_order != 0;
#else
  const bool wave_order = false;
#endif
  __shared__ float tmp[kOriBins + 4 + 1];   // + a dummy bin for the padding samples
  __shared__ __attribute__((aligned(16))) int sbin[kOT + 16];
  __shared__ __attribute__((aligned(16))) float sval[kOT + 16];
  __shared__ int wcnt[kOT / 64];
  const int nsv = (int)min(*nsurv, (unsigned)cap);
  const int tid = threadIdx.x;
  for (int sid = blockIdx.x; sid < nsv; sid += gridDim.x) {
    const Surv sv = surv[sid];
    const Kp& kpt = sv.k;
    const int o = sv.o, r = sv.r, c = sv.c;
    const Oct& q = P.o[o];
    const float* img = gauss + q.g + (size_t)q.w * q.h * sv.layer;
    const float scl_octv = kpt.size * 0.5f / (1 << o);
    const int radius = rnd(kOriRadius * scl_octv);
    const float osig = kOriSigFctr * scl_octv;
    const float expf_scale = -1.f / (2.f * osig * osig);
    if (tid < kOriBins + 5) tmp[tid] = 0.f;
    float* temphist = tmp + 2;
    const int side = 2 * radius + 1, total = side * side;
    for (int p0 = 0; p0 < total; p0 += kOT) {
      const int p = p0 + tid;
      const int i = p / side - radius, j = p % side - radius;
      const int y = r + i, x = c + j;
      const bool ok = p < total && y > 0 && y < q.h - 1 && x > 0 && x < q.w - 1;
      int bin = 0;
      float val = 0.f;
      if (ok) {
        const float dx = at(img, q.w, y, x + 1) - at(img, q.w, y, x - 1);
        const float dy = at(img, q.w, y - 1, x) - at(img, q.w, y + 1, x);
        const float wgt = fexp((i * i + j * j) * expf_scale);
        const float ori = fast_atan2(dy, dx);
        const float mag = fmag(dx, dy);
        bin = rnd((kOriBins / 360.f) * ori);
        if (bin >= kOriBins) bin -= kOriBins;
        if (bin < 0) bin += kOriBins;
        val = wgt * mag;
      }
      int nv;
      const int slot = block_compact_slot(ok, wcnt, nv);
      if (ok) {
        sbin[slot] = bin;
        sval[slot] = val;
      }
      if (tid < 16) {   // pad to a multiple of 16 with zero adds to the dummy bin
        sbin[nv + tid] = kOriBins + 2;
        sval[nv + tid] = 0.f;
      }
      __syncthreads();
      if (wave_order) {
      // wave 0 adds 64 samples per LDS atomic instruction, sample k on lane k: lanes of one
      // ds_add_f32 that hit the same bin are applied in lane order on gfx950 (probed:
      // tools/lds_atomic_order.hip, 2000 order-sensitive trials; checked again per context by
      // lds_order_probe_kernel), and the instructions of a wave in program order -- so every
      // bin still sums in OpenCV's sample order
      if (tid < 64) {
        for (int t0 = 0; t0 < nv; t0 += 64)
          if (t0 + tid < nv) atomicAdd(&temphist[sbin[t0 + tid]], sval[t0 + tid]);
      }
      } else if (tid == 0) {
        for (int t0 = 0; t0 < nv; t0 += 16) {
          int4 b4[4];
          float4 v4[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            b4[u] = *reinterpret_cast<const int4*>(&sbin[t0 + 4 * u]);
            v4[u] = *reinterpret_cast<const float4*>(&sval[t0 + 4 * u]);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            atomicAdd(&temphist[b4[u].x], v4[u].x);
            atomicAdd(&temphist[b4[u].y], v4[u].y);
            atomicAdd(&temphist[b4[u].z], v4[u].z);
            atomicAdd(&temphist[b4[u].w], v4[u].w);
          }
        }
      }
      __syncthreads();
    }
    if (tid == 0) {
      temphist[-1] = temphist[kOriBins - 1];
      temphist[-2] = temphist[kOriBins - 2];
      temphist[kOriBins] = temphist[0];
      temphist[kOriBins + 1] = temphist[1];
      float hist[kOriBins];
      for (int i = 0; i < kOriBins; i++)
        hist[i] = (temphist[i - 2] + temphist[i + 2]) * (1.f / 16.f) +
                  (temphist[i - 1] + temphist[i + 1]) * (4.f / 16.f) + temphist[i] * (6.f / 16.f);
      float omax = hist[0];
      for (int i = 1; i < kOriBins; i++) omax = fmaxf(omax, hist[i]);
      const float mag_thr = omax * kOriPeakRatio;
      // firstOctave = -1 rescale (exact, so it commutes with OpenCV's later sort / dedup)
      const float scale = 1.f / (float)(1 << -kFirstOctave);
      Kp out = kpt;
      out.octave = (kpt.octave & ~255) | ((kpt.octave + kFirstOctave) & 255);
      out.x = kpt.x * scale;
      out.y = kpt.y * scale;
      out.size = kpt.size * scale;
      out.pad0 = out.pad1 = 0;
      for (int j = 0; j < kOriBins; j++) {
        const int l = j > 0 ? j - 1 : kOriBins - 1;
        const int r2 = j < kOriBins - 1 ? j + 1 : 0;
        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
          float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
          bin = bin < 0 ? kOriBins + bin : bin >= kOriBins ? bin - kOriBins : bin;
          out.angle = 360.f - (float)((360.f / kOriBins) * bin);
          if (fabsf(out.angle - 360.f) < 1.1920928955078125e-07f) out.angle = 0.f;
          const unsigned k = atomicAdd(nkp, 1u);
          if (k < (unsigned)kcap) kps[k] = out;
        }
      }
    }
    __syncthreads();   // tmp is reused by the next survivor
  }
}

// ---- OpenCV order: KeyPointsFilter::removeDuplicatedSorted ----------------------------
// KeyPoint12_LessThan, with the array index as the last key (a total order)
__device__ inline bool kp_less(const Kp& a, int ia, const Kp& b, int ib) {
  if (a.x != b.x) return a.x < b.x;
  if (a.y != b.y) return a.y < b.y;
  if (a.size != b.size) return a.size > b.size;
  if (a.angle != b.angle) return a.angle < b.angle;
  if (a.response != b.response) return a.response > b.response;
  if (a.octave != b.octave) return a.octave > b.octave;
  return ia < ib;
}
__device__ inline bool kp_same(const Kp& a, const Kp& b) {
  return a.x == b.x && a.y == b.y && a.size == b.size && a.angle == b.angle;
}

constexpr int kRankTile = 64;
constexpr int kSortMax = 3072;   // keypoint lists up to this size: sort_dedup_kernel
// images up to this size leave the rank path to a second enqueue, after the host saw a list
// longer than kSortMax (textured 1000 x 800 images hold ~1 450 keypoints)
constexpr int64_t kEagerRankPixels = 1200000;
constexpr int kSortPow2 = 4096;  // its bitonic network (the next power of two)
// (i tile, j tile) pairs, strided over the grid.  pass 0: dup[i] |= an equal (x, y, size,
// angle) keypoint precedes i; pass 1: before[i] += kept keypoints preceding i (the sorted
// position)
__global__ __launch_bounds__(kRankTile) void rank_kernel(const Kp* __restrict__ kps,
                                                         const unsigned* __restrict__ nkp, int kcap,
                                                         int pass, unsigned* __restrict__ dup,
                                                         unsigned* __restrict__ before, int smax) {
  __shared__ Kp tile[kRankTile];
  __shared__ unsigned tdup[kRankTile];
  const int n = (int)min(*nkp, (unsigned)kcap);
  if (n <= smax) return;   // sort_dedup_kernel took it
  const int tiles = (n + kRankTile - 1) / kRankTile;
  for (int tp = blockIdx.x; tp < tiles * tiles; tp += gridDim.x) {
    const int i = (tp % tiles) * kRankTile + threadIdx.x;
    const int j0 = (tp / tiles) * kRankTile;
    __syncthreads();
    if (j0 + (int)threadIdx.x < n) {
      tile[threadIdx.x] = kps[j0 + threadIdx.x];
      tdup[threadIdx.x] = pass ? dup[j0 + threadIdx.x] : 0u;
    }
    __syncthreads();
    if (i >= n) continue;
    const Kp me = kps[i];
    const int m = min(kRankTile, n - j0);
    unsigned cnt = 0;
    bool d = false;
    for (int j = 0; j < m; ++j) {
      const bool lt = kp_less(tile[j], j0 + j, me, i);
      if (pass == 0)
        d = d || (lt && kp_same(tile[j], me));
      else
        cnt += (lt && !tdup[j]) ? 1u : 0u;
    }
    if (pass == 0) {
      if (d) atomicOr(&dup[i], 1u);
    } else if (cnt) {
      atomicAdd(&before[i], cnt);
    }
  }
}

__global__ void scatter_kernel(const Kp* __restrict__ kps, const unsigned* __restrict__ nkp, int kcap,
                               const unsigned* __restrict__ dup, const unsigned* __restrict__ before,
                               Kp* __restrict__ sorted, unsigned* __restrict__ nfinal, int smax,
                               int* __restrict__ src) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = (int)min(*nkp, (unsigned)kcap);
  if (n <= smax || i >= n || dup[i]) return;
  sorted[before[i]] = kps[i];
  if (src) src[before[i]] = i;
  atomicAdd(nfinal, 1u);
}

// Lists of up to kSortMax keypoints: OpenCV's order and dedup in ONE work-group instead of
// the two O(n^2) rank passes and the scatter.  A bitonic sort of the indices under
// kp_less (its index tie-break makes it a strict total order, so any correct sort gives the
// rank kernels' order), then a keypoint is kept unless the one before it is kp_same (equal
// (x, y, size, angle) keypoints are adjacent in that order: nothing sorts between them), and
// the kept ones are compacted in order -- the output rank_kernel + scatter_kernel produce.
// (x, y) as one 64-bit key that orders like kp_less's first two fields (IEEE order of the
// float bits: flip the negatives, set the sign of the positives); equal keys (rare) fall back
// to the full comparison
__device__ inline uint32_t f32_order(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline bool key_less(const Kp* sk, uint64_t ka, int a, uint64_t kb, int b, int n) {
  if (a >= n || b >= n) return a < b;   // padding sorts last (a < n <= b: real first)
  if (ka != kb) return ka < kb;
  return kp_less(sk[a], a, sk[b], b);
}
__global__ __launch_bounds__(1024) void sort_dedup_kernel(const Kp* __restrict__ kps,
                                                          const unsigned* __restrict__ nkp, int kcap,
                                                          Kp* __restrict__ sorted,
                                                          unsigned* __restrict__ nfinal, int smax,
                                                          int* __restrict__ src) {
  __shared__ Kp sk[kSortMax];
  __shared__ uint64_t k64[kSortPow2];   // the (x, y) keys, sorted with their indices
  __shared__ unsigned short ix[kSortPow2];
  __shared__ int wsum[16];
  __shared__ int carry_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = (int)min(*nkp, (unsigned)kcap);
  if (n > smax) return;   // rank_kernel / scatter_kernel take it
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int t = tid; t < n; t += 1024) {
    const Kp kp = kps[t];
    sk[t] = kp;
    // -0.0 and +0.0 compare equal under kp_less: fold them (one key for both)
    const float x = kp.x == 0.f ? 0.f : kp.x, y = kp.y == 0.f ? 0.f : kp.y;
    k64[t] = (uint64_t)f32_order(x) << 32 | f32_order(y);
  }
  for (int t = tid; t < np2; t += 1024) {
    ix[t] = (unsigned short)t;
    if (t >= n) k64[t] = ~0ull;
  }
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int q = tid; q < (np2 >> 1); q += 1024) {   // pair q: t with bit j clear, p = t | j
        const int t = ((q & ~(j - 1)) << 1) | (q & (j - 1)), p = t | j;
        const int a = ix[t], b = ix[p];
        const uint64_t ka = k64[t], kb = k64[p];
        const bool asc = (t & k) == 0;
        if (asc ? key_less(sk, kb, b, ka, a, n) : key_less(sk, ka, a, kb, b, n)) {
          ix[t] = (unsigned short)b;
          ix[p] = (unsigned short)a;
          k64[t] = kb;
          k64[p] = ka;
        }
      }
      // a wave's 64 pairs of stage (k, j <= 64) lie in its own 128 elements, and one wave's
      // LDS operations complete in order: only stages that cross waves need the barrier
      const int jn = j > 1 ? j >> 1 : k;
      if (j > 64 || jn > 64) __syncthreads();
    }
  __syncthreads();
  for (int p0 = 0; p0 < n; p0 += 1024) {
    const int p = p0 + tid;
    const bool kept = p < n && (p == 0 || !kp_same(sk[ix[p - 1]], sk[ix[p]]));
    const uint64_t m = __ballot(kept);
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int off = carry_s, tot = 0;
    for (int i = 0; i < 16; ++i) {
      off += i < w ? wsum[i] : 0;
      tot += wsum[i];
    }
    if (kept) {
      const int o = off + __popcll(m & ((1ull << lane) - 1ull));
      sorted[o] = sk[ix[p]];
      if (src) src[o] = ix[p];   // raw index (early descriptors)
    }
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  if (tid == 0) *nfinal = (unsigned)carry_s;
}

// final descriptors from the ones computed early on the raw keypoint list (the sort's
// source index per kept keypoint): one float4 per thread
__global__ void gather_desc_kernel(const float4* __restrict__ rdesc, const int* __restrict__ src,
                                   const unsigned* __restrict__ nfinal, float4* __restrict__ desc) {
  const int64_t n = (int64_t)*nfinal * 32;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    desc[t] = rdesc[(int64_t)src[t >> 5] * 32 + (t & 31)];
}

// ---- descriptors: calcSIFTDescriptor, one 256-thread block per keypoint ---------------
// The window's samples are computed 192 at a time by waves 1-3 (one per thread, OpenCV's
// row-major order), compacted in that order, and their eight trilinear contributions added
// to the LDS histogram by wave 0 one chunk behind, sample by sample (the eight bins of a
// sample are distinct), so every bin sums in OpenCV's order.
constexpr int kHistLen = (kD + 2) * (kD + 2) * (kN + 2);
constexpr int kDT = 256;
constexpr int kDP = kDT - 64;   // window samples per chunk: waves 1-3 produce, wave 0 adds
constexpr int kDescSide = kDT;  // windows up to this many rows enumerate per-row j ranges
// a histogram index in one of the d x d inner cells: the only bins the descriptor reads (the
// border ring, ~1/3 of the trilinear contributions, and the dummy padding bins are skipped;
// every inner bin still receives its adds in sample order)
__device__ __forceinline__ bool inner_bin(int b) {
  const int cell = b / (kN + 2), r = cell / (kD + 2), c = cell - r * (kD + 2);
  return r >= 1 && r <= kD && c >= 1 && c <= kD;
}
__global__ __launch_bounds__(kDT) void descriptor_kernel(const float* __restrict__ gauss, Pyr P,
                                                         const Kp* __restrict__ sorted,
                                                         const unsigned* __restrict__ nfinal,
                                                         float* __restrict__ desc, int lane_order,
                                                         int range_max, int ncap) {
  __shared__ float hist[kHistLen];
  __shared__ int sidx[2][kDP / 64][64];           // [buffer][producer wave][compacted slot]
  __shared__ float svalT[2][kDP / 64][8][64];     // the 8 contributions of each slot
  __shared__ int nseg[2][kDP / 64];
  __shared__ int rlo[kDescSide], roff[kDescSide + 1];   // per window row: first j, first sample
  __shared__ int wsum[kDT / 64];
  __shared__ float raw[kD * kD * kN];
  __shared__ float scal[2];
  const int tid = threadIdx.x;
  const int nf = (int)min(*nfinal, (unsigned)ncap);   // (a raw list may exceed its capacity)
#if SOD_SIFT_WAVE_ORDER_ARCH
  const bool wave_order = lane_order != 0;
#else
  const bool wave_order = false;
#endif
  // the eight bins of a sample relative to its first (lanes 0-7 of the ordered adds)
  const int off = tid == 0 ? 0 : tid == 1 ? 1 : tid == 2 ? kN + 2 : tid == 3 ? kN + 3
                : tid == 4 ? (kD + 2) * (kN + 2) : tid == 5 ? (kD + 2) * (kN + 2) + 1
                : tid == 6 ? (kD + 3) * (kN + 2) : (kD + 3) * (kN + 2) + 1;
  for (int id = blockIdx.x; id < nf; id += gridDim.x) {
    const Kp k = sorted[id];
    int octave = k.octave & 255;
    const int layer = (k.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    const float sc = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
    const float size = k.size * sc;
    const Oct& q = P.o[octave - kFirstOctave];
    const float* img = gauss + q.g + (size_t)q.w * q.h * layer;
    float ori = 360.f - k.angle;
    if (fabsf(ori - 360.f) < 1.1920928955078125e-07f) ori = 0.f;
    const float scl = size * 0.5f;
    const float ptx = k.x * sc, pty = k.y * sc;
    const int px = rnd(ptx), py = rnd(pty);
    double sd, cd;
    s_sincos((double)(ori * (float)(3.14159265358979323846 / 180)), &sd, &cd);
    float cos_t = (float)cd, sin_t = (float)sd;
    const float bins_per_rad = kN / 360.f;
    const float exp_scale = -1.f / (kD * kD * 0.5f);
    const float hist_width = kDescrSclFctr * scl;
    int radius = rnd(hist_width * 1.4142135623730951f * (kD + 1) * 0.5f);
    const int diag = isqrt64((int64_t)q.w * q.w + (int64_t)q.h * q.h);
    radius = min(radius, diag);
    cos_t /= hist_width;
    sin_t /= hist_width;
    const int rows = q.h, cols = q.w;
    for (int t = tid; t < kHistLen; t += kDT) hist[t] = 0.f;
    const int side = 2 * radius + 1;
    // The samples enumerated: per window row i, a j range that holds every position the
    // test below can accept (rbin, cbin in (-1, d): |r_rot|, |c_rot| < d/2 + 0.5, widened by
    // 1e-3 and one column each side; r, c inside the image), in row-major order -- about
    // half the window's positions.  The per-sample test still decides, so the samples and
    // their order are OpenCV's.  Windows over range_max (<= kDescSide) rows enumerate every
    // position.
    const bool ranged = side <= range_max;
    int64_t total = (int64_t)side * side;
    if (ranged) {
      int cnt = 0, jl = 0;
      if (tid < side) {
        const int i = tid - radius, r = py + i;
        double lo = max(-radius, 1 - px), hi = min(radius, cols - 2 - px);
        if (r <= 0 || r >= rows - 1) hi = lo - 1;
        constexpr double E = kD * 0.5 + 0.5 + 1e-3;
        const double ab[2][2] = {{(double)sin_t, (double)i * cos_t}, {(double)cos_t, -(double)i * sin_t}};
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {   // a j + b in (-E, E)
          const double a = ab[k2][0], b = ab[k2][1];
          if (fabs(a) < 1e-12) {
            if (fabs(b) >= E) hi = lo - 1;
          } else {
            const double j1 = (-E - b) / a, j2 = (E - b) / a;
            lo = fmax(lo, floor(fmin(j1, j2)) - 1);
            hi = fmin(hi, ceil(fmax(j1, j2)) + 1);
          }
        }
        if (hi >= lo) {
          jl = (int)lo;
          cnt = (int)hi - jl + 1;
        }
      }
      // exclusive scan of the row counts over the block
      int x = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if ((tid & 63) >= d) x += y;
      }
      if ((tid & 63) == 63) wsum[tid >> 6] = x;
      __syncthreads();
      int before = 0, tot = 0;
#pragma unroll
      for (int k2 = 0; k2 < kDT / 64; ++k2) {
        before += k2 < (tid >> 6) ? wsum[k2] : 0;
        tot += wsum[k2];
      }
      roff[tid] = before + x - cnt;
      rlo[tid] = jl;
      if (tid == 0) roff[kDescSide] = tot;
      total = tot;
      __syncthreads();
    }
    // Waves 1-3 compute chunk c (192 window samples, one per thread, OpenCV's row-major
    // order) while wave 0 adds chunk c-1 into the histogram: two buffers, one barrier per
    // chunk.  Each producer wave compacts its 64 samples into its own segment (ballot, no
    // barrier); segments 1, 2, 3 in turn are the chunk's samples in order.
    const int64_t nch = (total + kDP - 1) / kDP;
    const int wv = tid >> 6, lane = tid & 63;
    for (int64_t ch = 0; ch <= nch; ++ch) {
      const int buf = (int)(ch & 1);
      if (wv > 0 && ch < nch) {
        const int64_t p = ch * kDP + (tid - 64);
        int i, j;
        if (ranged) {   // the row holding sample p: last t with roff[t] <= p
          int t = 0;
#pragma unroll
          for (int st = kDescSide / 2; st >= 1; st >>= 1)
            if (roff[t + st] <= p) t += st;
          i = t - radius;
          j = rlo[t] + (int)(p - roff[t]);
        } else {
          i = (int)(p / side) - radius;
          j = (int)(p % side) - radius;
        }
        const float c_rot = j * cos_t - i * sin_t;
        const float r_rot = j * sin_t + i * cos_t;
        float rbin = r_rot + kD / 2 - 0.5f;
        float cbin = c_rot + kD / 2 - 0.5f;
        const int r = py + i, c = px + j;
        const bool ok = p < total && rbin > -1 && rbin < kD && cbin > -1 && cbin < kD && r > 0 &&
                        r < rows - 1 && c > 0 && c < cols - 1;
        int idx = 0;
        float v8[8];
        if (ok) {
          const float dx = at(img, cols, r, c + 1) - at(img, cols, r, c - 1);
          const float dy = at(img, cols, r - 1, c) - at(img, cols, r + 1, c);
          const float wexp = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
          const float o_k = fast_atan2(dy, dx);
          const float mag_k = fmag(dx, dy);
          const float w_k = fexp(wexp);
          float obin = (o_k - ori) * bins_per_rad;
          const float mag = mag_k * w_k;
          const int r0 = flo(rbin), c0 = flo(cbin);
          int o0 = flo(obin);
          rbin -= r0;
          cbin -= c0;
          obin -= o0;
          if (o0 < 0) o0 += kN;
          if (o0 >= kN) o0 -= kN;
          const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
          const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
          const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
          v8[7] = v_rc11 * obin;            // v_rco111
          v8[6] = v_rc11 - v8[7];           // v_rco110
          v8[5] = v_rc10 * obin;            // v_rco101
          v8[4] = v_rc10 - v8[5];           // v_rco100
          v8[3] = v_rc01 * obin;            // v_rco011
          v8[2] = v_rc01 - v8[3];           // v_rco010
          v8[1] = v_rc00 * obin;            // v_rco001
          v8[0] = v_rc00 - v8[1];           // v_rco000
          idx = ((r0 + 1) * (kD + 2) + c0 + 1) * (kN + 2) + o0;
        }
        const uint64_t m = __ballot(ok);
        const int sg = wv - 1;
        if (ok) {
          const int slot = __popcll(m & ((1ull << lane) - 1ull));
          sidx[buf][sg][slot] = idx;
#pragma unroll
          for (int e = 0; e < 8; ++e) svalT[buf][sg][e][slot] = v8[e];
        }
        if (lane == 0) nseg[buf][sg] = __popcll(m);
      }
      if (wv == 0 && ch > 0) {
        const int pb = buf ^ 1;
        if (wave_order) {
          // 8 samples per LDS atomic instruction: lane 8 s + e carries contribution e of
          // sample s (same-bin lanes apply in lane order = sample order, see orient_kernel);
          // the next group's operands are read before this group's atomic goes out (a wave's
          // LDS operations complete in order: reads issued after the atomic would wait on it)
          const int s8 = lane >> 3, e = lane & 7;
          const int offe = e == 0 ? 0 : e == 1 ? 1 : e == 2 ? kN + 2 : e == 3 ? kN + 3
                         : e == 4 ? (kD + 2) * (kN + 2) : e == 5 ? (kD + 2) * (kN + 2) + 1
                         : e == 6 ? (kD + 3) * (kN + 2) : (kD + 3) * (kN + 2) + 1;
          for (int sg = 0; sg < kDP / 64; ++sg) {
            const int n = nseg[pb][sg];
            int b = sidx[pb][sg][min(s8, 63)] + offe;
            float v = svalT[pb][sg][e][min(s8, 63)];
            for (int t0 = 0; t0 < n; t0 += 8) {
              const int tn = min(t0 + 8 + s8, 63);
              const int bn = sidx[pb][sg][tn] + offe;
              const float vn = svalT[pb][sg][e][tn];
              if (t0 + s8 < n && inner_bin(b)) {
                atomicAdd(&hist[b], v);
              }
              b = bn;
              v = vn;
            }
          }
        } else if (lane < 8) {
          // ordered single-lane adds: lane e adds contribution e, one sample per instruction
          for (int sg = 0; sg < kDP / 64; ++sg) {
            const int n = nseg[pb][sg];
            for (int t = 0; t < n; ++t) {
              const int b = sidx[pb][sg][t] + off;
              if (inner_bin(b)) atomicAdd(&hist[b], svalT[pb][sg][lane][t]);
            }
          }
        }
      }
      __syncthreads();   // chunk ch written, chunk ch-1 added: the buffers swap roles
    }
    // finalize: fold the circular orientation bins, then OpenCV's sequential norms
    if (tid < kD * kD) {
      const int i = tid / kD, j = tid % kD;
      const int idx = ((i + 1) * (kD + 2) + (j + 1)) * (kN + 2);
      hist[idx] += hist[idx + kN];
      hist[idx + 1] += hist[idx + kN + 1];
      for (int k2 = 0; k2 < kN; k2++) raw[(i * kD + j) * kN + k2] = hist[idx + k2];
    }
    __syncthreads();
    constexpr int len = kD * kD * kN;
    if (tid == 0) {
      float nrm2 = 0;
      for (int k2 = 0; k2 < len; k2++) nrm2 += raw[k2] * raw[k2];
      const float thr = sqrt_rn(nrm2) * kDescrMagThr;
      nrm2 = 0;
      for (int i = 0; i < len; i++) {
        const float val = fminf(raw[i], thr);
        raw[i] = val;
        nrm2 += val * val;
      }
      scal[0] = kIntDescrFctr / fmaxf(sqrt_rn(nrm2), 1.1920928955078125e-07f);
    }
    __syncthreads();
    const float nrm = scal[0];
    float* dst = desc + (size_t)id * 128;
    if (tid < len) {
      const int v = rnd(raw[tid] * nrm);
      dst[tid] = (float)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    __syncthreads();   // LDS reused by the next keypoint
  }
}

// Self-check of the property the wave-order histogram adds rely on: one wave's ds_add_f32
// with same-address lanes, applied in lane order.  Per trial 64 values whose float sum
// depends on the order (large / small / cancelling magnitudes) go to 1, 2 or 8 LDS
// addresses with one atomic instruction; the host compares with the lane-order sums.
__global__ __launch_bounds__(64) void lds_order_probe_kernel(const float* __restrict__ vals,
                                                             const int* __restrict__ addr,
                                                             float* __restrict__ out, int trials) {
  __shared__ float h[8];
  const int l = threadIdx.x;
  for (int t = 0; t < trials; ++t) {
    if (l < 8) h[l] = 0.f;
    __syncthreads();
    atomicAdd(&h[addr[t * 64 + l]], vals[t * 64 + l]);
    __syncthreads();
    if (l < 8) out[t * 8 + l] = h[l];
    __syncthreads();
  }
}

__global__ void bgr2gray_kernel(const uint8_t* __restrict__ bgr, int64_t n, uint8_t* __restrict__ g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g[i] = (uint8_t)((bgr[3 * i] * 1868 + bgr[3 * i + 1] * 9617 + bgr[3 * i + 2] * 4899 + (1 << 13)) >> 14);
}

__global__ void unpack_kp_kernel(const Kp* __restrict__ sorted, const unsigned* __restrict__ nfinal,
                                 float* __restrict__ x, float* __restrict__ y,
                                 float* __restrict__ ang, int32_t* __restrict__ oct) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int)*nfinal) return;
  const Kp k = sorted[i];
  x[i] = k.x;
  y[i] = k.y;
  ang[i] = k.angle;
  oct[i] = k.octave;
}

// ---- host side ------------------------------------------------------------------------
// cv::getGaussianKernel(n, sigma, CV_32F) with the GaussianBlur size rule for float images
int gauss_kernel(double sigma, float* k) {
  const int n = (int)std::lrint(sigma * 4 * 2 + 1) | 1;
  const int r = n / 2;
  if (r + 1 > kMaxTaps) return -1;
  std::vector<float> cf((size_t)n);
  const double scale2X = -0.5 / (sigma * sigma);
  double sum = 0;
  for (int i = 0; i < n; i++) {
    const double x = i - (n - 1) * 0.5;
    cf[(size_t)i] = (float)std::exp(scale2X * x * x);
    sum += cf[(size_t)i];
  }
  sum = 1. / sum;
  for (int i = 0; i < n; i++) cf[(size_t)i] = (float)(cf[(size_t)i] * sum);
  for (int i = 0; i <= r; i++) k[i] = cf[(size_t)(r + i)];
  return r;
}

}  // namespace

// one in-flight image: its pyramid, candidate / keypoint lists and descriptors, on its
// own stream (a batch keeps several images in flight)
struct SiftSlot {
  hipStream_t stream = nullptr;
  // a lone image runs the big octaves' extrema on `side`, beside the small-octave chain
  // (one work-group) on `stream`; a batch keeps to one stream per image
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  Pyr P{};
  DevBuf<uint8_t> gray, bgr;
  DevBuf<float> gauss, dogs, tmp, up;
  DevBuf<int4> cand;
  DevBuf<Surv> surv;
  DevBuf<Kp> kps, sorted;
  DevBuf<unsigned> dup, before;
  DevBuf<unsigned> cnt;        // [0] candidates, [1] raw keypoints, [2] final, [3] survivors
  DevBuf<float> desc;          // [cap * 128]
  unsigned* hcnt = nullptr;    // pinned copy of cnt
  int cap = 1 << 16;
  bool rank_deferred = false;   // the rank path was left out of the last enqueue
  // a lone image writes its final keypoints / descriptors straight into the context's
  // result arrays (no copy after the host sync); null: into `sorted` / `desc`
  Kp* out_kp = nullptr;
  float* out_desc = nullptr;
  // a lone image computes the descriptors of the raw keypoint list on `side` while the sort
  // runs, into `rdesc`; the sort's source indices (`src`) then gather the final ones
  bool early_desc = false;
  DevBuf<float> rdesc;
  DevBuf<int> src;
  Kp* final_kp() { return out_kp ? out_kp : sorted.p; }
  float* final_desc() { return out_desc ? out_desc : desc.p; }
};

struct SiftWork {
  // histogram adds: 1 = wave order, 0 = ordered single lane; -1 = not decided yet (the
  // self-check runs on the first SIFT call); mode = sod_sift_set_lane_order's request
  int lane_order = -1, lane_mode = -1, probe_ok = -1;
  int L = 3;
  double contrast = 0.04, edge = 10.0, sigma = 1.6;
  int radius[kMaxLayers] = {};
  DevBuf<float> kern;          // [kMaxLayers][kMaxTaps]
  DevBuf<int> rad;             // [kMaxLayers]
  bool kern_ok = false;
  std::vector<SiftSlot*> slots;
  // results of the last detect / batch, concatenated in image order
  DevBuf<Kp> all_kp;
  DevBuf<float> all_desc;
  std::vector<int64_t> off{0};
  std::vector<int32_t> shapes;   // (h, w) per image
  bool valid = false;
};

static void free_slot(SiftSlot* S) {
  if (S->stream) (void)sod_stream_drain(S->stream);
  sod_release(S->gray);
  sod_release(S->bgr);
  sod_release(S->gauss);
  sod_release(S->dogs);
  sod_release(S->tmp);
  sod_release(S->up);
  sod_release(S->cand);
  sod_release(S->surv);
  sod_release(S->kps);
  sod_release(S->sorted);
  sod_release(S->dup);
  sod_release(S->before);
  sod_release(S->cnt);
  sod_release(S->desc);
  sod_release(S->rdesc);
  sod_release(S->src);
  if (S->hcnt) (void)hipHostFree(S->hcnt);
  if (S->side) (void)sod_stream_drain(S->side);
  if (S->fork) (void)hipEventDestroy(S->fork);
  if (S->join) (void)hipEventDestroy(S->join);
  if (S->side) (void)hipStreamDestroy(S->side);
  if (S->stream) (void)hipStreamDestroy(S->stream);
  delete S;
}

void sod_sift_free(sod_ctx* ctx) {
  SiftWork* W = ctx->sift;
  if (!W) return;
  for (SiftSlot* S : W->slots) free_slot(S);
  sod_release(W->kern);
  sod_release(W->rad);
  sod_release(W->all_kp);
  sod_release(W->all_desc);
  delete W;
  ctx->sift = nullptr;
}

namespace {

// images in flight in a batch (measured, 16 images of 1000 x 800: 2 slots 0.68 ms per image,
// 4 slots 0.64, 8 slots 0.95 -- more streams than hardware queues serialise; replaying each
// image's launches as a HIP graph changed nothing: the GPU, not the host, is the limit)
constexpr int kSlots = 4;

SiftWork* work(sod_ctx* ctx) {
  if (!ctx->sift) ctx->sift = new SiftWork();
  return ctx->sift;
}

int get_slot(sod_ctx* ctx, SiftWork& W, int i, SiftSlot** out) {
  while ((int)W.slots.size() <= i) {
    SiftSlot* S = new SiftSlot();
    W.slots.push_back(S);
    // a CU-masked stream gets a hardware queue of its own (unmasked streams share a pool of
    // GPU_MAX_HW_QUEUES with every other stream of the process -- the contexts' matcher and
    // tail streams among them -- and the image's stream and its side stream on ONE queue
    // serialise and stall on their cross-stream events: 0.65 -> 1.2-1.5 ms per image
    // measured); the mask leaves out CU 0, the side stream's leaves out the last CU.  Only
    // slot kSlots, the lone image's (the one with the side stream): batches run on slots
    // 0..kSlots-1, unmasked -- in a bench-like process (r04 siftmask1, 3 interleaved rounds)
    // a batch of 16 took 5.8-7.3 ms with no slot masked, 7.6-7.9 ms with its slot 0 masked
    // (round 3's layout: the lone image and the batches shared slot 0) and 7.3-7.5 ms with all
    // masked (SOD_SIFT_STREAM_MASK=0: none masked, 2: all)
    int masked = (int)W.slots.size() == kSlots + 1 ? 1 : 0;
    if (ctx->opt.sift_stream_mask == 2 || ctx->opt.sift_stream_mask == 0)
      masked = ctx->opt.sift_stream_mask == 2 ? 1 : 0;
    if (masked && ctx->num_cus > 2) {
      std::vector<uint32_t> mask((size_t)(ctx->num_cus + 31) / 32, 0u);
      for (int i = 1; i < ctx->num_cus; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
      SOD_HIP(ctx, hipExtStreamCreateWithCUMask(&S->stream, (uint32_t)mask.size(), mask.data()));
    } else {
      SOD_HIP(ctx, hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking));
    }
    SOD_HIP(ctx, hipHostMalloc((void**)&S->hcnt, 16, hipHostMallocDefault));
  }
  *out = W.slots[(size_t)i];
  return SOD_OK;
}

// lds_order_probe_kernel over 512 trials (a fixed LCG: the same on every run); 1 when every
// trial came out in lane order, 0 otherwise
int lds_order_probe(sod_ctx* ctx, int* ok) {
  constexpr int kTrials = 512;
  std::vector<float> v((size_t)kTrials * 64);
  std::vector<int> a((size_t)kTrials * 64);
  uint32_t st = 12345u;
  auto rnd = [&st]() { st = st * 1664525u + 1013904223u; return st >> 8; };
  for (int t = 0; t < kTrials; ++t) {
    const int nb = t % 3 == 0 ? 1 : t % 3 == 1 ? 2 : 8;
    for (int l = 0; l < 64; ++l) {
      const uint32_t k = rnd() % 4;
      v[(size_t)t * 64 + l] = k == 0 ? 1.0e8f * (rnd() % 2 ? 1.f : -1.f)
                            : k == 1 ? 1.0f + (float)(rnd() % 1000) * 1e-3f
                            : k == 2 ? 3.1e-5f * (float)(rnd() % 100) : 7.7e7f;
      a[(size_t)t * 64 + l] = (int)(rnd() % nb);
    }
  }
  DevBuf<float> dv, dout;
  DevBuf<int> da;
  std::vector<float> o((size_t)kTrials * 8);
  int rc = sod_reserve(ctx, dv, v.size());
  if (rc == SOD_OK) rc = sod_reserve(ctx, da, a.size());
  if (rc == SOD_OK) rc = sod_reserve(ctx, dout, o.size());
  // copies on the context stream (the synchronisation below covers them): a null-stream copy
  // would wait for every blocking stream of the process, the CU-masked ones included
  if (rc == SOD_OK &&
      (hipMemcpyAsync(dv.p, v.data(), v.size() * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
       hipMemcpyAsync(da.p, a.data(), a.size() * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess))
    rc = sod_fail(ctx, SOD_EHIP, "lds order probe upload failed");
  if (rc == SOD_OK) {
    hipLaunchKernelGGL(lds_order_probe_kernel, dim3(1), dim3(64), 0, ctx->stream, dv.p, da.p,
                       dout.p, kTrials);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(o.data(), dout.p, o.size() * 4, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        sod_stream_sync(ctx->stream) != hipSuccess)
      rc = sod_fail(ctx, SOD_EHIP, "lds order probe failed");
  }
  sod_release(dv);
  sod_release(da);
  sod_release(dout);
  SOD_TRY(rc);
  int good = 1;
  for (int t = 0; t < kTrials && good; ++t) {
    float ref[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int l = 0; l < 64; ++l) ref[a[(size_t)t * 64 + l]] += v[(size_t)t * 64 + l];
    for (int b = 0; b < 8; ++b) good &= o[(size_t)t * 8 + b] == ref[b];
  }
  *ok = good;
  return SOD_OK;
}

int set_lane_order(sod_ctx* ctx, SiftWork& W) {
  if (W.lane_order >= 0) return SOD_OK;
  if (W.probe_ok < 0) {
    if (ctx->gfx950) SOD_TRY(lds_order_probe(ctx, &W.probe_ok));
    else W.probe_ok = 0;   // the wave-order adds are compiled for gfx950 only
  }
  W.lane_order = (W.lane_mode != 0 && W.probe_ok == 1) ? 1 : 0;
  return SOD_OK;
}

int set_kernels(sod_ctx* ctx, SiftWork& W) {
  SOD_TRY(set_lane_order(ctx, W));
  if (W.kern_ok) return SOD_OK;
  // sig[0] = the base blur sqrt(max(sigma^2 - 4 * 0.5^2, 0.01)) in float (createInitialImage);
  // sig[i] as buildGaussianPyramid (double)
  double sig[kMaxLayers];
  const float s = (float)W.sigma;
  sig[0] = (double)std::sqrt(std::max(s * s - 0.5f * 0.5f * 4, 0.01f));
  const double k = std::pow(2., 1. / W.L);
  for (int i = 1; i < W.L + 3; i++) {
    const double sig_prev = std::pow(k, (double)(i - 1)) * W.sigma;
    const double sig_total = sig_prev * k;
    sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
  }
  std::vector<float> h((size_t)kMaxLayers * kMaxTaps, 0.f);
  for (int i = 0; i < W.L + 3; i++) {
    W.radius[i] = gauss_kernel(sig[i], h.data() + (size_t)i * kMaxTaps);
    if (W.radius[i] < 0) return sod_fail(ctx, SOD_EINVAL, "sigma too large for the blur kernel");
  }
  SOD_TRY(sod_reserve(ctx, W.kern, h.size()));
  SOD_TRY(sod_reserve(ctx, W.rad, (size_t)kMaxLayers));
  SOD_HIP(ctx, hipMemcpyAsync(W.kern.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(W.rad.p, W.radius, sizeof(W.radius), hipMemcpyHostToDevice, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  W.kern_ok = true;
  return SOD_OK;
}

int blur(sod_ctx* ctx, const SiftWork& W, SiftSlot& S, const float* src, float* dst, int w, int h,
         int layer, const float* prev, float* dog, hipStream_t bs = nullptr) {
  const float* k = W.kern.p + (size_t)layer * kMaxTaps;
  const int r = W.radius[layer];
  if (r >= 1 && r <= kMaxR) {   // (no scratch: the one path `bs` may name another stream for)
    dim3 gt((unsigned)((w + kTW - 1) / kTW), (unsigned)((h + kTH - 1) / kTH));
    hipLaunchKernelGGL(kBlurFns[r], gt, dim3(256), 0, bs ? bs : S.stream, src, dst, w, h, k, dog);
    return SOD_OK;
  }
  dim3 g((unsigned)((w + 255) / 256), (unsigned)h);
  hipLaunchKernelGGL(blur_rows_kernel, g, dim3(256), 0, S.stream, src, S.tmp.p, w, k, r);
  hipLaunchKernelGGL(blur_cols_kernel, g, dim3(256), 0, S.stream, S.tmp.p, dst, w, h, k, r, prev,
                     dog);
  return SOD_OK;
}

constexpr int kOrientGrid = 4096, kRankGrid = 2048, kDescGrid = 4096;

// geometry of the pyramid of a w x h image (OpenCV: nOctaves = cvRound(log2(min(2w, 2h)) - 2)
// - firstOctave); returns the Gaussian / DoG element counts
void plan_pyramid(int L, int w, int h, Pyr& P, int64_t& go, int64_t& dof, int& o_small) {
  P.L = L;
  const int bw = 2 * w, bh = 2 * h;
  int nOct = (int)std::lrint(std::log((double)std::min(bw, bh)) / std::log(2.) - 2) - kFirstOctave;
  nOct = std::max(1, std::min(nOct, kMaxOct));
  P.n = nOct;
  go = dof = 0;
  int ow = bw, oh = bh;
  for (int o = 0; o < nOct; ++o) {
    P.o[o] = Oct{ow, oh, go, dof};
    go += (int64_t)(L + 3) * ow * oh;
    dof += (int64_t)(L + 2) * ow * oh;
    ow /= 2;
    oh /= 2;
    if (ow < 1 || oh < 1) {   // OpenCV would build empty layers here; none hold keypoints
      P.n = nOct = o + 1;
      break;
    }
  }
  o_small = nOct;   // first octave handled by small_octaves_kernel
  for (int o = 1; o < nOct && L + 2 <= kChainDog; ++o)
    if ((int64_t)P.o[o].w * P.o[o].h <= kChainPixels) {
      o_small = o;
      break;
    }
}

// option sift_sort_max (tests): a lower one-work-group limit, so the rank path runs too
int sort_max(const sod_ctx* ctx) {
  int smax = kSortMax;
  if (ctx->opt.sift_sort_max != -2) smax = std::max(-1, std::min(kSortMax, ctx->opt.sift_sort_max));
  return smax;
}

// keypoint order + dedup of lists longer than smax: two O(n^2) rank passes and a scatter
// (each exits at once when sort_dedup_kernel took the list)
int enqueue_rank(sod_ctx* ctx, SiftSlot& S, int smax) {
  hipStream_t st = S.stream;
  const int cap = S.cap;
  SOD_HIP(ctx, hipMemsetAsync(S.dup.p, 0, (size_t)cap * 4, st));
  SOD_HIP(ctx, hipMemsetAsync(S.before.p, 0, (size_t)cap * 4, st));
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(rank_kernel, dim3(kRankGrid), dim3(kRankTile), 0, st, S.kps.p, S.cnt.p + 1, cap,
                       pass, S.dup.p, S.before.p, smax);
  hipLaunchKernelGGL(scatter_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, st, S.kps.p,
                     S.cnt.p + 1, cap, S.dup.p, S.before.p, S.final_kp(), S.cnt.p + 2, smax,
                     S.early_desc ? S.src.p : nullptr);
  return SOD_OK;
}

// descriptors of the final list, then the counts to the host
int enqueue_describe(sod_ctx* ctx, SiftSlot& S, int lane_order) {
  hipStream_t st = S.stream;
  // option sift_desc_range_max (tests): a lower window-row limit of the ranged enumeration
  int rmax = kDescSide;
  if (ctx->opt.sift_desc_range_max >= 0) rmax = std::min(kDescSide, ctx->opt.sift_desc_range_max);
  if (S.early_desc)
    hipLaunchKernelGGL(gather_desc_kernel, dim3(1024), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(S.rdesc.p), S.src.p, S.cnt.p + 2,
                       reinterpret_cast<float4*>(S.final_desc()));
  else
    hipLaunchKernelGGL(descriptor_kernel, dim3(kDescGrid), dim3(kDT), 0, st, S.gauss.p, S.P, S.final_kp(),
                       S.cnt.p + 2, S.final_desc(), lane_order, rmax, S.cap);
  SOD_HIP(ctx, hipGetLastError());
  SOD_HIP(ctx, hipMemcpyAsync(S.hcnt, S.cnt.p, 16, hipMemcpyDeviceToHost, st));
  return SOD_OK;
}

// enqueue detect + describe of the image in S.gray on S.stream (no host sync); the counts
// land in S.hcnt.  `pyramid` false re-runs only the stages after it (list overflow).
int slot_enqueue(sod_ctx* ctx, const SiftWork& W, SiftSlot& S, int w, int h, bool pyramid, bool lone) {
  const int L = W.L;
  Pyr& P = S.P;
  int64_t go, dof;
  int o_small;
  plan_pyramid(L, w, h, P, go, dof, o_small);
  const int nOct = P.n, bw = 2 * w, bh = 2 * h;
  SOD_TRY(sod_reserve(ctx, S.gauss, (size_t)go));
  SOD_TRY(sod_reserve(ctx, S.dogs, (size_t)dof));
  SOD_TRY(sod_reserve(ctx, S.tmp, (size_t)bw * bh));
  SOD_TRY(sod_reserve(ctx, S.up, (size_t)bw * bh));
  SOD_TRY(sod_reserve(ctx, S.cnt, 4));
  const int cap = S.cap;
  SOD_TRY(sod_reserve(ctx, S.cand, (size_t)cap));
  SOD_TRY(sod_reserve(ctx, S.surv, (size_t)cap));
  SOD_TRY(sod_reserve(ctx, S.kps, (size_t)cap));
  SOD_TRY(sod_reserve(ctx, S.sorted, (size_t)cap));
  SOD_TRY(sod_reserve(ctx, S.dup, (size_t)cap));
  SOD_TRY(sod_reserve(ctx, S.before, (size_t)cap));
  SOD_TRY(sod_reserve(ctx, S.desc, (size_t)cap * 128));
  const float thr = (float)(int)std::floor(0.5 * W.contrast / L * 255 * 1);
  hipStream_t st = S.stream;
  SOD_HIP(ctx, hipMemsetAsync(S.cnt.p, 0, 16, st));
  ExtGrid G{};   // the octaves above the small-octave chain: one extrema launch
  int tot = 0;
  for (int o = 0; o < o_small; ++o) {
    const Oct& q = P.o[o];
    G.first[o] = tot;
    if (q.w > 2 * kBorder && q.h > 2 * kBorder)
      tot += ((q.w - 2 * kBorder + 255) / 256) * ((q.h - 2 * kBorder + kExtRows - 1) / kExtRows) * L;
  }
  G.first[o_small] = tot;
  G.n = o_small;
  // a lone image runs the big octaves' extrema on S.side beside the small-octave chain (both
  // append to the candidate list atomically; the keypoint sort fixes the order) and, when it
  // builds the pyramid, also the top two layers of every big octave: the next octave needs
  // only layer L, so its chain starts while layers L+1, L+2 blur beside it
  const bool split = lone && tot > 0 && o_small < nOct;
  bool lsplit = split && pyramid && W.radius[L + 1] >= 1 && W.radius[L + 1] <= kMaxR &&
                W.radius[L + 2] >= 1 && W.radius[L + 2] <= kMaxR;
  int nsplit = kMaxOct;   // option sift_layer_split = n (A/B): only the first n octaves split
  if (ctx->opt.sift_layer_split >= 0) nsplit = ctx->opt.sift_layer_split;
  if (split && !S.side) {
    // the side stream leaves one CU out of its mask (option sift_side_mask 0: all CUs): the
    // small-octave chain (one 1 024-thread work-group, ~146 KB of LDS) then always finds a
    // free CU instead of waiting for the extrema launch's work-groups to drain
    const int keep_free = ctx->opt.sift_side_mask != 0;
    if (keep_free && ctx->num_cus > 1) {
      std::vector<uint32_t> mask((size_t)(ctx->num_cus + 31) / 32, 0u);
      for (int i = 0; i < ctx->num_cus - 1; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
      SOD_HIP(ctx, hipExtStreamCreateWithCUMask(&S.side, (uint32_t)mask.size(), mask.data()));
    } else {
      SOD_HIP(ctx, hipStreamCreateWithFlags(&S.side, hipStreamNonBlocking));
    }
    SOD_HIP(ctx, hipEventCreateWithFlags(&S.fork, hipEventDisableTiming));
    SOD_HIP(ctx, hipEventCreateWithFlags(&S.join, hipEventDisableTiming));
  }
  if (pyramid) {
    hipLaunchKernelGGL(upscale_kernel, dim3((unsigned)((bw + 255) / 256), (unsigned)bh), dim3(256), 0,
                       st, S.gray.p, w, h, S.up.p);
    for (int o = 0; o < o_small; ++o) {
      const Oct& q = P.o[o];
      const size_t plane = (size_t)q.w * q.h;
      float* g0 = S.gauss.p + q.g;
      if (o == 0) {
        SOD_TRY(blur(ctx, W, S, S.up.p, g0, q.w, q.h, 0, nullptr, nullptr));
      } else {
        const Oct& pq = P.o[o - 1];
        hipLaunchKernelGGL(down2_kernel, dim3((unsigned)((q.w + 255) / 256), (unsigned)q.h), dim3(256),
                           0, st, S.gauss.p + pq.g + (size_t)pq.w * pq.h * L, pq.w, g0, q.w);
      }
      for (int i = 1; i < L + 3; ++i) {
        hipStream_t bs = st;
        if (lsplit && o < nsplit && i == L + 1) {   // layer L is done on st: fork
          SOD_HIP(ctx, hipEventRecord(S.fork, st));
          SOD_HIP(ctx, hipStreamWaitEvent(S.side, S.fork, 0));
        }
        if (lsplit && o < nsplit && i > L) bs = S.side;
        SOD_TRY(blur(ctx, W, S, g0 + plane * (i - 1), g0 + plane * i, q.w, q.h, i, g0 + plane * (i - 1),
                     S.dogs.p + q.d + plane * (i - 1), bs));
      }
    }
  }
  {
    hipStream_t xs = st;
    if (split) {   // the side stream holds the top layers (lsplit) and waits for the rest
      // (when the last big octave split, the side stream already waits for every layer the
      // image's stream blurs: no second event right before the small-octave chain)
      if (!(lsplit && o_small - 1 < nsplit) || ctx->opt.sift_fork2) {
        SOD_HIP(ctx, hipEventRecord(S.fork, st));
        SOD_HIP(ctx, hipStreamWaitEvent(S.side, S.fork, 0));
      }
      xs = S.side;
    }
    if (tot > 0)
      hipLaunchKernelGGL(extrema_all_kernel, dim3((unsigned)tot), dim3(256), 0, xs, S.dogs.p, P, G,
                         thr, S.cand.p, S.cnt.p, cap);
    if (split) SOD_HIP(ctx, hipEventRecord(S.join, S.side));
    if (o_small < nOct)   // re-running it re-blurs the small octaves identically
      hipLaunchKernelGGL(small_octaves_kernel, dim3(1), dim3(1024), 0, st, S.gauss.p, S.dogs.p, P,
                         o_small, W.kern.p, W.rad.p, thr, S.cand.p, S.cnt.p, cap);
    if (split) SOD_HIP(ctx, hipStreamWaitEvent(st, S.join, 0));
  }
  hipLaunchKernelGGL(refine_kernel, dim3((unsigned)((cap + 127) / 128)), dim3(128), 0, st, S.dogs.p, P,
                     S.cand.p, S.cnt.p, cap, (float)W.contrast, (float)W.edge, (float)W.sigma, S.surv.p,
                     S.cnt.p + 3);
  hipLaunchKernelGGL(orient_kernel, dim3(kOrientGrid), dim3(kOT), 0, st, S.gauss.p, P, S.surv.p,
                     S.cnt.p + 3, cap, S.kps.p, S.cnt.p + 1, cap, W.lane_order);
  // lone image: descriptors of the raw list on the side stream, beside the keypoint sort
  // (a descriptor depends on its keypoint only; the few duplicates the sort drops cost their
  // work-groups); option sift_early_desc 0: after the sort, of the final list
  S.early_desc = split && ctx->opt.sift_early_desc != 0;
  if (S.early_desc) {
    SOD_TRY(sod_reserve(ctx, S.rdesc, (size_t)cap * 128));
    SOD_TRY(sod_reserve(ctx, S.src, (size_t)cap));
    int rmax = kDescSide;
    if (ctx->opt.sift_desc_range_max >= 0) rmax = std::min(kDescSide, ctx->opt.sift_desc_range_max);
    SOD_HIP(ctx, hipEventRecord(S.fork, st));
    SOD_HIP(ctx, hipStreamWaitEvent(S.side, S.fork, 0));
    hipLaunchKernelGGL(descriptor_kernel, dim3(kDescGrid), dim3(kDT), 0, S.side, S.gauss.p, P, S.kps.p,
                       S.cnt.p + 1, S.rdesc.p, W.lane_order, rmax, cap);
    SOD_HIP(ctx, hipEventRecord(S.join, S.side));
  }
  const int smax = sort_max(ctx);
  hipLaunchKernelGGL(sort_dedup_kernel, dim3(1), dim3(1024), 0, st, S.kps.p, S.cnt.p + 1, cap,
                     S.final_kp(), S.cnt.p + 2, smax, S.early_desc ? S.src.p : nullptr);
  // lists longer than smax take the rank path; an image small enough that its list most
  // likely fits leaves those launches (two memsets, three kernels that would exit at once:
  // ~25 us of a ~660 us image) to a second enqueue after the host sees the count
  S.rank_deferred = (int64_t)w * h <= kEagerRankPixels;
  S.rank_deferred = S.rank_deferred && ctx->opt.sift_eager_rank == 0;   // option: 1 = always eager
  if (!S.rank_deferred) SOD_TRY(enqueue_rank(ctx, S, smax));
  if (S.early_desc) SOD_HIP(ctx, hipStreamWaitEvent(st, S.join, 0));
  return enqueue_describe(ctx, S, W.lane_order);
}

// upload one image (8-bit gray, or BGR converted on the device) into S.gray
int slot_upload(sod_ctx* ctx, SiftSlot& S, const uint8_t* img, int w, int h, int channels) {
  const size_t np = (size_t)w * h;
  SOD_TRY(sod_reserve(ctx, S.gray, np));
  if (channels == 1) {
    SOD_HIP(ctx, hipMemcpyAsync(S.gray.p, img, np, hipMemcpyHostToDevice, S.stream));
  } else {
    SOD_TRY(sod_reserve(ctx, S.bgr, np * 3));
    SOD_HIP(ctx, hipMemcpyAsync(S.bgr.p, img, np * 3, hipMemcpyHostToDevice, S.stream));
    hipLaunchKernelGGL(bgr2gray_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, S.stream,
                       S.bgr.p, (int64_t)np, S.gray.p);
  }
  return SOD_OK;
}

int grow_results(sod_ctx* ctx, SiftWork& W, int64_t need) {
  if ((int64_t)W.all_kp.n >= need && (int64_t)W.all_desc.n >= need * 128) return SOD_OK;
  const int64_t have = W.off.back();
  const int64_t n = std::max<int64_t>(need, 2 * (int64_t)W.all_kp.n);
  DevBuf<Kp> nk;
  DevBuf<float> nd;
  SOD_TRY(sod_reserve(ctx, nk, (size_t)n));
  SOD_TRY(sod_reserve(ctx, nd, (size_t)n * 128));
  for (SiftSlot* S : W.slots) SOD_HIP(ctx, sod_stream_sync(S->stream));
  if (have > 0) {   // on slot 0's stream, not the null stream (see lds_order_probe)
    hipStream_t s0 = W.slots[0]->stream;
    SOD_HIP(ctx, hipMemcpyAsync(nk.p, W.all_kp.p, (size_t)have * sizeof(Kp), hipMemcpyDeviceToDevice, s0));
    SOD_HIP(ctx, hipMemcpyAsync(nd.p, W.all_desc.p, (size_t)have * 512, hipMemcpyDeviceToDevice, s0));
    SOD_HIP(ctx, sod_stream_sync(s0));
  }
  sod_release(W.all_kp);
  sod_release(W.all_desc);
  W.all_kp = nk;
  W.all_desc = nd;
  return SOD_OK;
}

// point a lone image's final lists at the result arrays (grown to hold its capacity at the
// next offset), or back at the slot's own buffers
int set_direct(sod_ctx* ctx, SiftWork& W, SiftSlot& S, bool on) {
  S.out_kp = nullptr;
  S.out_desc = nullptr;
  if (!on) return SOD_OK;
  const int64_t at = W.off.back();
  SOD_TRY(grow_results(ctx, W, at + S.cap));
  S.out_kp = W.all_kp.p + at;
  S.out_desc = W.all_desc.p + at * 128;
  return SOD_OK;
}

// detect + describe n images, kSlots in flight on their own streams; the results are
// appended to W.all_kp / W.all_desc in image order (W.off = prefix counts)
int run_batch(sod_ctx* ctx, int n, const uint8_t* const* imgs, const int32_t* ws, const int32_t* hs,
              const int32_t* chans, int32_t* counts) {
  SiftWork& W = *work(ctx);
  W.valid = false;
  for (int i = 0; i < n; ++i)
    if (!imgs[i] || ws[i] < 1 || hs[i] < 1 || (int64_t)ws[i] * hs[i] > (1LL << 28) ||
        (chans && chans[i] != 1 && chans[i] != 3))
      return sod_fail(ctx, SOD_EINVAL, "bad image arguments (image " + std::to_string(i) + ")");
  SOD_TRY(set_kernels(ctx, W));
  W.off.assign(1, 0);
  W.shapes.clear();
  const int K = std::min(n, kSlots);
  // option sift_direct 0 (A/B): a lone image's results copied after the sync too
  const bool direct = ctx->opt.sift_direct != 0;
  for (int i0 = 0; i0 < n; i0 += K) {
    const int m = std::min(K, n - i0);
    // a lone image (a round of one) on its own CU-masked slot, batches on the unmasked ones
    auto slot_of = [&](int j) { return m == 1 ? kSlots : j; };
    for (int j = 0; j < m; ++j) {
      SiftSlot* S;
      SOD_TRY(get_slot(ctx, W, slot_of(j), &S));
      const int i = i0 + j;
      SOD_TRY(slot_upload(ctx, *S, imgs[i], ws[i], hs[i], chans ? chans[i] : 1));
      SOD_TRY(set_direct(ctx, W, *S, m == 1 && direct));
      SOD_TRY(slot_enqueue(ctx, W, *S, ws[i], hs[i], true, m == 1));
    }
    for (int j = 0; j < m; ++j) {
      SiftSlot* S = W.slots[(size_t)slot_of(j)];
      const int i = i0 + j;
      for (int attempt = 0;; ++attempt) {
        SOD_HIP(ctx, sod_stream_sync(S->stream));
        const unsigned c0 = S->hcnt[0], c1 = S->hcnt[1];
        if (c0 <= (unsigned)S->cap && c1 <= (unsigned)S->cap) break;
        if (attempt >= 3) return sod_fail(ctx, SOD_ENOMEM, "SIFT: candidate list did not fit after growing");
        // grow and redo after the pyramid (the result does not depend on discovery order)
        S->cap = (int)std::min<int64_t>(1 << 26, 2 * (int64_t)std::max(c0, c1));
        SOD_TRY(set_direct(ctx, W, *S, S->out_kp != nullptr));   // room for the grown list
        SOD_TRY(slot_enqueue(ctx, W, *S, ws[i], hs[i], false, m == 1));
      }
      if (S->rank_deferred && (int64_t)S->hcnt[1] > sort_max(ctx)) {   // the list did not fit one work-group
        SOD_TRY(enqueue_rank(ctx, *S, sort_max(ctx)));
        SOD_TRY(enqueue_describe(ctx, *S, W.lane_order));
        SOD_HIP(ctx, sod_stream_sync(S->stream));
      }
      const int64_t cnt = S->hcnt[2];
      const int64_t at = W.off.back();
      SOD_TRY(grow_results(ctx, W, at + cnt));
      if (cnt > 0 && !S->out_kp) {
        SOD_HIP(ctx, hipMemcpyAsync(W.all_kp.p + at, S->sorted.p, (size_t)cnt * sizeof(Kp),
                                    hipMemcpyDeviceToDevice, S->stream));
        SOD_HIP(ctx, hipMemcpyAsync(W.all_desc.p + at * 128, S->desc.p, (size_t)cnt * 512,
                                    hipMemcpyDeviceToDevice, S->stream));
      }
      W.off.push_back(at + cnt);
      W.shapes.push_back(hs[i]);
      W.shapes.push_back(ws[i]);
      if (counts) counts[i] = (int32_t)cnt;
    }
  }
  for (SiftSlot* S : W.slots) SOD_HIP(ctx, sod_stream_sync(S->stream));
  W.valid = true;
  return SOD_OK;
}

}  // namespace

// ---- C ABI ----------------------------------------------------------------------------
extern "C" {

int sod_sift_set_params(sod_ctx* ctx, int32_t n_octave_layers, double contrast_threshold,
                        double edge_threshold, double sigma) {
  if (!ctx) return SOD_EINVAL;
  if (n_octave_layers < 1 || n_octave_layers + 3 > kMaxLayers || !(sigma > 0) ||
      !(contrast_threshold >= 0) || !(edge_threshold > 0))
    return sod_fail(ctx, SOD_EINVAL, "SIFT parameters out of range");
  SiftWork& W = *work(ctx);
  if (W.L == n_octave_layers && W.contrast == contrast_threshold && W.edge == edge_threshold &&
      W.sigma == sigma)
    return SOD_OK;
  W.L = n_octave_layers;
  W.contrast = contrast_threshold;
  W.edge = edge_threshold;
  W.sigma = sigma;
  W.kern_ok = false;
  W.valid = false;
  return SOD_OK;
}

int sod_sift_set_lane_order(sod_ctx* ctx, int mode) {
  if (!ctx) return SOD_EINVAL;
  if (mode != -1 && mode != 0) return sod_fail(ctx, SOD_EINVAL, "lane order mode must be -1 or 0");
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  SiftWork& W = *work(ctx);
  W.lane_mode = mode;
  W.lane_order = -1;   // decided again (the self-check result is kept)
  W.valid = false;
  return SOD_OK;
}

int sod_sift_lane_order(sod_ctx* ctx, int* active, int* probe_ok) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  SiftWork& W = *work(ctx);
  SOD_TRY(set_lane_order(ctx, W));
  if (active) *active = W.lane_order;
  if (probe_ok) *probe_ok = W.probe_ok;
  return SOD_OK;
}

int sod_sift_detect(sod_ctx* ctx, const uint8_t* gray, int32_t width, int32_t height,
                    int32_t* n_keypoints) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  if (!n_keypoints) return sod_fail(ctx, SOD_EINVAL, "null output");
  const uint8_t* imgs[1] = {gray};
  const int32_t one = 1;
  return run_batch(ctx, 1, imgs, &width, &height, &one, n_keypoints);
}

int sod_sift_detect_bgr(sod_ctx* ctx, const uint8_t* bgr, int32_t width, int32_t height,
                        int32_t* n_keypoints) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  if (!n_keypoints) return sod_fail(ctx, SOD_EINVAL, "null output");
  const uint8_t* imgs[1] = {bgr};
  const int32_t three = 3;
  return run_batch(ctx, 1, imgs, &width, &height, &three, n_keypoints);
}

int sod_sift_detect_batch(sod_ctx* ctx, int32_t n_images, const uint8_t* const* images,
                          const int32_t* widths, const int32_t* heights, const int32_t* channels,
                          int32_t* counts) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  if (n_images < 1 || !images || !widths || !heights)
    return sod_fail(ctx, SOD_EINVAL, "bad batch arguments");
  return run_batch(ctx, n_images, images, widths, heights, channels, counts);
}

int sod_sift_get(sod_ctx* ctx, int64_t cap, float* x, float* y, float* size, float* angle,
                 float* response, int32_t* octave, float* descriptors) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  SiftWork* W = ctx->sift;
  if (!W || !W->valid) return sod_fail(ctx, SOD_ESTATE, "no SIFT result: call sod_sift_detect first");
  const int64_t n = std::min<int64_t>(W->off.back(), std::max<int64_t>(cap, 0));
  if (n > 0) {
    std::vector<Kp> h((size_t)n);
    // the detection's streams are done (its count sync); the copies go on slot 0's stream
    // rather than the null stream, which would wait for every blocking stream of the process
    for (SiftSlot* S : W->slots) SOD_HIP(ctx, sod_stream_sync(S->stream));
    hipStream_t s0 = W->slots[0]->stream;
    SOD_HIP(ctx, hipMemcpyAsync(h.data(), W->all_kp.p, (size_t)n * sizeof(Kp), hipMemcpyDeviceToHost, s0));
    if (descriptors)
      SOD_HIP(ctx, hipMemcpyAsync(descriptors, W->all_desc.p, (size_t)n * 512, hipMemcpyDeviceToHost, s0));
    SOD_HIP(ctx, sod_stream_sync(s0));
    for (int64_t i = 0; i < n; ++i) {
      const Kp& k = h[(size_t)i];
      if (x) x[i] = k.x;
      if (y) y[i] = k.y;
      if (size) size[i] = k.size;
      if (angle) angle[i] = k.angle;
      if (response) response[i] = k.response;
      if (octave) octave[i] = k.octave;
    }
  }
  return SOD_OK;
}

// the last detection (one image or a batch) becomes the query set of the matcher / Hough
// stages, without a host round trip (descriptors are packed from device memory); a batch
// is declared as query images (sod_query_images) for the fused per-image stages
int sod_sift_to_queries(sod_ctx* ctx) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  SiftWork* W = ctx->sift;
  if (!W || !W->valid) return sod_fail(ctx, SOD_ESTATE, "no SIFT result: call sod_sift_detect first");
  const int64_t nq64 = W->off.back();
  if (nq64 < 1) return sod_fail(ctx, SOD_ESTATE, "the image(s) have no SIFT keypoints");
  if (nq64 > (1 << 27)) return sod_fail(ctx, SOD_EINVAL, "query count out of range");
  const int32_t nq = (int32_t)nq64;
  SOD_TRY(sod_reserve(ctx, ctx->flags, 4));
  // invalid-value count and the query max norm (flags[1], the DB's, stays)
  SOD_HIP(ctx, hipMemsetAsync(ctx->flags.p, 0, 4, ctx->stream));
  SOD_HIP(ctx, hipMemsetAsync(ctx->flags.p + 2, 0, 4, ctx->stream));
  SOD_TRY(sod_inputs_begin(ctx));
  SOD_TRY(ctx->impl != 0 ? launch_pack_i8(ctx, W->all_desc.p, SOD_DTYPE_F32, nq, false)
                         : launch_pack_queries(ctx, W->all_desc.p, SOD_DTYPE_F32, nq));
  SOD_TRY(sod_inputs_end(ctx));
  SOD_TRY(sod_reserve(ctx, ctx->qx, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->qy, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->qang, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->qoct, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->scal, 4));
  // the final count as a device scalar for unpack_kp_kernel
  const unsigned un = (unsigned)nq;
  SOD_HIP(ctx, hipMemcpyAsync(ctx->scal.p + 3, &un, 4, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(unpack_kp_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, ctx->stream,
                     W->all_kp.p, ctx->scal.p + 3, ctx->qx.p, ctx->qy.p, ctx->qang.p, ctx->qoct.p);
  SOD_HIP(ctx, hipGetLastError());
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->nq = nq;
  ctx->win0 = 0;
  ctx->winn = -1;
  ctx->n_qimg = 0;
  ctx->matched = ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  ++ctx->res_epoch;   // staged results (sod_results_fetch) are stale now
  const int nimg = (int)W->shapes.size() / 2;
  if (nimg > 1) {
    std::vector<int32_t> off(W->off.begin(), W->off.end());
    SOD_TRY(sod_query_images(ctx, nimg, off.data(), W->shapes.data()));
  }
  return SOD_OK;
}

}  // extern "C"

