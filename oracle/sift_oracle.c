/* CPU restatement of SIFT detect + describe -- TEST INFRASTRUCTURE ONLY (SURVEY.md 8(f)
 * row 4).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline load this.
 *
 * The reference calls OpenCV: `sift = cv2.SIFT_create()` (main.py:179,
 * GenerateDatabaseInfo.py:16) and `sift.detectAndCompute(gray, None)` (main.py:43,
 * GenerateDatabaseInfo.py:32).  OpenCV is a third-party dependency absent here
 * (opencv-python >= 4.4 -- SIFT_create moved to the main module in 4.4.0 -- version
 * unpinned by the reference); this file restates its published algorithm,
 * modules/features2d/src/sift.dispatch.cpp + sift.simd.hpp (defaults nfeatures 0,
 * nOctaveLayers 3, contrastThreshold 0.04, edgeThreshold 10, sigma 1.6, float DoG):
 *
 *   createInitialImage  -> x2 INTER_LINEAR upscale (exact: weights 1/4, 3/4 of integers)
 *                          + GaussianBlur(sqrt(sigma^2 - 4 * 0.5^2))
 *   buildGaussianPyramid -> nOctaveLayers + 3 layers per octave, incremental blurs,
 *                          next octave = every 2nd pixel of layer nOctaveLayers
 *   buildDoGPyramid      -> layer differences
 *   findScaleSpaceExtrema -> 26-neighbour extrema (>= / <=) above floor(0.5 * ct / L * 255),
 *                          adjustLocalExtrema (<= 5 Newton steps, 3x3 Cramer solve as
 *                          Matx33f::solve, contrast + edge tests), calcOrientationHist
 *                          (36 bins, [1 4 6 4 1]/16 smoothing, peaks >= 0.8 max,
 *                          parabolic interpolation)
 *   KeyPointsFilter::removeDuplicatedSorted -> sort by (x, y, -size, angle, -response,
 *                          -octave), drop equal (x, y, size, angle)
 *   firstOctave = -1 rescale, calcSIFTDescriptor (4x4x8, trilinear, clip 0.2, x512,
 *                          saturate_cast<uchar> into a float row)
 *
 * PARITY UNPINNED AGAINST OPENCV: no OpenCV and no reference fixture exists at this
 * boundary.  Arithmetic that OpenCV leaves to SIMD / IPP / its own math kernels is fixed
 * here (and identically in the device code, sift.hip), so the device path is compared
 * with THIS restatement bit for bit:
 *   - separable blur: row pass then column pass, out = k0*x + sum_{i=1..r} k_i*(x[-i]+x[+i])
 *     in increasing i, BORDER_REFLECT_101, no FMA (OpenCV: its SIMD row/column filters);
 *   - exp(x), sin, cos and 2^y through the double-precision Cody-Waite + Taylor kernels
 *     s_exp / s_sincos below (OpenCV: cv::hal::exp32f, cosf, sinf, powf), rounded to float;
 *   - |v| = correctly rounded float sqrt of x*x + y*y (OpenCV: magnitude32f);
 *   - fastAtan2: OpenCV's published 7th-order polynomial (scalar form, no FMA);
 *   - sums (histograms, norms) in OpenCV's scalar loop order.
 * Compile with -ffp-contract=off (no FMA), no fast-math.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SIFT_DESCR_WIDTH 4
#define SIFT_DESCR_HIST_BINS 8
#define SIFT_INIT_SIGMA 0.5f
#define SIFT_IMG_BORDER 5
#define SIFT_MAX_INTERP_STEPS 5
#define SIFT_ORI_HIST_BINS 36
#define SIFT_ORI_SIG_FCTR 1.5f
#define SIFT_ORI_RADIUS (3 * SIFT_ORI_SIG_FCTR)
#define SIFT_ORI_PEAK_RATIO 0.8f
#define SIFT_DESCR_SCL_FCTR 3.f
#define SIFT_DESCR_MAG_THR 0.2f
#define SIFT_INT_DESCR_FCTR 512.f
#define FIRST_OCTAVE (-1)

typedef struct {
  int w, h;
  float* p;
} img_t;

static int cv_round_d(double v) { return (int)lrint(v); }   /* round half to even */
static int cv_round_f(float v) { return (int)lrintf(v); }
static int cv_floor_f(float v) {
  int i = (int)v;
  return i - (i > v);
}
static int cv_floor_d(double v) {
  int i = (int)v;
  return i - (i > v);
}

static img_t img_new(int w, int h) {
  img_t m = {w, h, (float*)calloc((size_t)w * h > 0 ? (size_t)w * h : 1, sizeof(float))};
  return m;
}
#define AT(m, y, x) ((m).p[(size_t)(y) * (m).w + (x)])

/* cv::borderInterpolate(p, len, BORDER_REFLECT_101) */
static int reflect101(int p, int len) {
  if ((unsigned)p < (unsigned)len) return p;
  if (len == 1) return 0;
  do {
    if (p < 0)
      p = -p - 1 + 1;
    else
      p = len - 1 - (p - len) - 1;
  } while ((unsigned)p >= (unsigned)len);
  return p;
}

/* cv::getGaussianKernel(n, sigma, CV_32F) with n = cvRound(sigma * 4 * 2 + 1) | 1 (the
 * GaussianBlur size rule for float images); returns the radius, k[0..r] = centre..edge */
int sift_gauss_kernel(double sigma, float* k, int kmax) {
  const int n = cv_round_d(sigma * 4 * 2 + 1) | 1;
  const int r = n / 2;
  if (r + 1 > kmax) return -1;
  float* cf = (float*)malloc(sizeof(float) * n);
  const double scale2X = -0.5 / (sigma * sigma);
  double sum = 0;
  for (int i = 0; i < n; i++) {
    const double x = i - (n - 1) * 0.5;
    cf[i] = (float)exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
  for (int i = 0; i <= r; i++) k[i] = cf[r + i];
  free(cf);
  return r;
}

static void blur(const img_t* src, img_t* dst, double sigma) {
  float k[64];
  const int r = sift_gauss_kernel(sigma, k, 64);
  const int w = src->w, h = src->h;
  img_t t = img_new(w, h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      float s = k[0] * AT(*src, y, x);
      for (int i = 1; i <= r; i++)
        s += k[i] * (AT(*src, y, reflect101(x - i, w)) + AT(*src, y, reflect101(x + i, w)));
      AT(t, y, x) = s;
    }
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      float s = k[0] * AT(t, y, x);
      for (int i = 1; i <= r; i++)
        s += k[i] * (AT(t, reflect101(y - i, h), x) + AT(t, reflect101(y + i, h), x));
      AT(*dst, y, x) = s;
    }
  free(t.p);
}

/* x2 INTER_LINEAR resize of an 8-bit image to float: sample positions (d + 0.5)/2 - 0.5,
 * clamped at the borders; every value is a multiple of 1/16 below 256, hence exact */
static img_t upscale2(const uint8_t* g, int w, int h) {
  img_t t = img_new(2 * w, h), u = img_new(2 * w, 2 * h);
  for (int y = 0; y < h; y++)
    for (int d = 0; d < 2 * w; d++) {
      const int i = d >> 1;
      float v;
      if (d & 1)
        v = i + 1 < w ? 0.75f * g[(size_t)y * w + i] + 0.25f * g[(size_t)y * w + i + 1]
                      : (float)g[(size_t)y * w + i];
      else
        v = i > 0 ? 0.25f * g[(size_t)y * w + i - 1] + 0.75f * g[(size_t)y * w + i]
                  : (float)g[(size_t)y * w + i];
      AT(t, y, d) = v;
    }
  for (int d = 0; d < 2 * h; d++) {
    const int i = d >> 1;
    for (int x = 0; x < 2 * w; x++) {
      float v;
      if (d & 1)
        v = i + 1 < h ? 0.75f * AT(t, i, x) + 0.25f * AT(t, i + 1, x) : AT(t, i, x);
      else
        v = i > 0 ? 0.25f * AT(t, i - 1, x) + 0.75f * AT(t, i, x) : AT(t, i, x);
      AT(u, d, x) = v;
    }
  }
  free(t.p);
  return u;
}

typedef struct {
  int nOct, L;
  img_t* g;   /* nOct * (L + 3) */
  img_t* d;   /* nOct * (L + 2) */
} pyr_t;

int sift_num_octaves(int w, int h) {
  const int bw = 2 * w, bh = 2 * h;
  return cv_round_d(log((double)(bw < bh ? bw : bh)) / log(2.) - 2) - FIRST_OCTAVE;
}

/* the per-layer blur sigmas of buildGaussianPyramid (sig[0] = the base blur) */
void sift_layer_sigmas(int L, double sigma, double* sig) {
  const float s = (float)sigma;
  sig[0] = (double)sqrtf(fmaxf(s * s - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA * 4, 0.01f));
  const double k = pow(2., 1. / L);
  for (int i = 1; i < L + 3; i++) {
    const double sig_prev = pow(k, (double)(i - 1)) * sigma;
    const double sig_total = sig_prev * k;
    sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
  }
}

static pyr_t build_pyramid(const uint8_t* gray, int w, int h, int L, double sigma) {
  pyr_t P;
  P.L = L;
  P.nOct = sift_num_octaves(w, h);
  double sig[64];
  sift_layer_sigmas(L, sigma, sig);
  P.g = (img_t*)calloc((size_t)P.nOct * (L + 3), sizeof(img_t));
  P.d = (img_t*)calloc((size_t)P.nOct * (L + 2), sizeof(img_t));
  for (int o = 0; o < P.nOct; o++)
    for (int i = 0; i < L + 3; i++) {
      img_t* dst = &P.g[o * (L + 3) + i];
      if (o == 0 && i == 0) {
        img_t u = upscale2(gray, w, h);
        *dst = img_new(u.w, u.h);
        blur(&u, dst, sig[0]);
        free(u.p);
      } else if (i == 0) {
        const img_t* src = &P.g[(o - 1) * (L + 3) + L];
        *dst = img_new(src->w / 2, src->h / 2);
        for (int y = 0; y < dst->h; y++)
          for (int x = 0; x < dst->w; x++) AT(*dst, y, x) = AT(*src, 2 * y, 2 * x);
      } else {
        const img_t* src = &P.g[o * (L + 3) + i - 1];
        *dst = img_new(src->w, src->h);
        blur(src, dst, sig[i]);
      }
    }
  for (int o = 0; o < P.nOct; o++)
    for (int i = 0; i < L + 2; i++) {
      const img_t* a = &P.g[o * (L + 3) + i];
      const img_t* b = &P.g[o * (L + 3) + i + 1];
      img_t* dst = &P.d[o * (L + 2) + i];
      *dst = img_new(a->w, a->h);
      for (size_t j = 0; j < (size_t)a->w * a->h; j++) dst->p[j] = b->p[j] - a->p[j];
    }
  return P;
}

static void free_pyramid(pyr_t* P) {
  for (int i = 0; i < P->nOct * (P->L + 3); i++) free(P->g[i].p);
  for (int i = 0; i < P->nOct * (P->L + 2); i++) free(P->d[i].p);
  free(P->g);
  free(P->d);
}

/* cv::hal::fastAtan2 (degrees), scalar form */
float sift_fast_atan2(float y, float x) {
  const float d2r = (float)(180 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * d2r, p3 = -0.3258083974640975f * d2r,
              p5 = 0.1555786518463281f * d2r, p7 = -0.04432655554792128f * d2r;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)DBL_EPSILON);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)DBL_EPSILON);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

/* e^x: Cody-Waite reduction by ln2 and a Taylor polynomial to r^13 (|r| <= 0.35) */
static double s_exp(double x) {
  if (x < -740.0) return 0.0;
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double n = rint(x * 1.44269504088896338700e+00);
  const double r = (x - n * ln2_hi) - n * ln2_lo;
  static const double inv_fact[14] = {1.0,           1.0,           0.5,
                                      1.0 / 6.0,     1.0 / 24.0,    1.0 / 120.0,
                                      1.0 / 720.0,   1.0 / 5040.0,  1.0 / 40320.0,
                                      1.0 / 362880.0, 1.0 / 3628800.0, 1.0 / 39916800.0,
                                      1.0 / 479001600.0, 1.0 / 6227020800.0};
  double p = inv_fact[13];
  for (int k = 12; k >= 0; k--) p = p * r + inv_fact[k];
  return ldexp(p, (int)n);
}

/* sin and cos: reduction by pi/2 (two-part constant), Taylor polynomials to r^21 / r^22 */
static void s_sincos(double a, double* sn, double* cs) {
  const double pio2_hi = 1.57079632673412561417e+00, pio2_lo = 6.07710050650619224932e-11;
  const double k = rint(a * 6.36619772367581382433e-01);
  const double r = (a - k * pio2_hi) - k * pio2_lo;
  const double r2 = r * r;
  /* odd / even Taylor coefficients, signs alternating from the top term down */
  static const double fs[10] = {1.0 / 51090942171709440000.0, 1.0 / 121645100408832000.0,
                                1.0 / 355687428096000.0,     1.0 / 1307674368000.0,
                                1.0 / 6227020800.0,          1.0 / 39916800.0,
                                1.0 / 362880.0,              1.0 / 5040.0,
                                1.0 / 120.0,                 1.0 / 6.0};
  static const double fc[11] = {1.0 / 1124000727777607680000.0, 1.0 / 2432902008176640000.0,
                                1.0 / 6402373705728000.0,       1.0 / 20922789888000.0,
                                1.0 / 87178291200.0,            1.0 / 479001600.0,
                                1.0 / 3628800.0,                1.0 / 40320.0,
                                1.0 / 720.0,                    1.0 / 24.0,
                                0.5};
  double s = fs[0];
  for (int i = 1; i < 10; i++) s = (i & 1) ? s * r2 - fs[i] : s * r2 + fs[i];
  s = r + r * r2 * s;
  double c = -fc[0];
  for (int i = 1; i < 11; i++) c = (i & 1) ? c * r2 + fc[i] : c * r2 - fc[i];
  c = 1.0 + r2 * c;
  switch (((int)k) & 3) {
    case 0: *sn = s; *cs = c; break;
    case 1: *sn = c; *cs = -s; break;
    case 2: *sn = -s; *cs = -c; break;
    default: *sn = -c; *cs = s; break;
  }
}

static float fexp(float x) { return (float)s_exp((double)x); }
static float fmag(float x, float y) { return (float)sqrt((double)(x * x + y * y)); }

typedef struct {
  float x, y, size, angle, response;
  int octave;
} kp_t;

/* adjustLocalExtrema (sift.simd.hpp) */
static int adjust_local_extrema(const pyr_t* P, kp_t* kpt, int octv, int* layer, int* r, int* c,
                                float contrastThreshold, float edgeThreshold, float sigma) {
  const int L = P->L;
  const float img_scale = 1.f / (255 * 1);
  const float deriv_scale = img_scale * 0.5f;
  const float second_deriv_scale = img_scale;
  const float cross_deriv_scale = img_scale * 0.25f;
  float xi = 0, xr = 0, xc = 0, contr = 0;
  int i = 0;
  for (; i < SIFT_MAX_INTERP_STEPS; i++) {
    const int idx = octv * (L + 2) + *layer;
    const img_t img = P->d[idx], prev = P->d[idx - 1], next = P->d[idx + 1];
    const int R = *r, C = *c;
    const float dD0 = (AT(img, R, C + 1) - AT(img, R, C - 1)) * deriv_scale;
    const float dD1 = (AT(img, R + 1, C) - AT(img, R - 1, C)) * deriv_scale;
    const float dD2 = (AT(next, R, C) - AT(prev, R, C)) * deriv_scale;
    const float v2 = AT(img, R, C) * 2;
    const float dxx = (AT(img, R, C + 1) + AT(img, R, C - 1) - v2) * second_deriv_scale;
    const float dyy = (AT(img, R + 1, C) + AT(img, R - 1, C) - v2) * second_deriv_scale;
    const float dss = (AT(next, R, C) + AT(prev, R, C) - v2) * second_deriv_scale;
    const float dxy = (AT(img, R + 1, C + 1) - AT(img, R + 1, C - 1) - AT(img, R - 1, C + 1) +
                       AT(img, R - 1, C - 1)) * cross_deriv_scale;
    const float dxs = (AT(next, R, C + 1) - AT(next, R, C - 1) - AT(prev, R, C + 1) +
                       AT(prev, R, C - 1)) * cross_deriv_scale;
    const float dys = (AT(next, R + 1, C) - AT(next, R - 1, C) - AT(prev, R + 1, C) +
                       AT(prev, R - 1, C)) * cross_deriv_scale;
    /* Matx33f H(dxx dxy dxs / dxy dyy dys / dxs dys dss); X = H.solve(dD, DECOMP_LU):
     * the 3x3 fast path (Cramer's rule in float, zero vector when det == 0) */
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
      return 0;
    *c += cv_round_f(xc);
    *r += cv_round_f(xr);
    *layer += cv_round_f(xi);
    if (*layer < 1 || *layer > L || *c < SIFT_IMG_BORDER || *c >= img.w - SIFT_IMG_BORDER ||
        *r < SIFT_IMG_BORDER || *r >= img.h - SIFT_IMG_BORDER)
      return 0;
  }
  if (i >= SIFT_MAX_INTERP_STEPS) return 0;
  {
    const int idx = octv * (L + 2) + *layer;
    const img_t img = P->d[idx], prev = P->d[idx - 1], next = P->d[idx + 1];
    const int R = *r, C = *c;
    const float dD0 = (AT(img, R, C + 1) - AT(img, R, C - 1)) * deriv_scale;
    const float dD1 = (AT(img, R + 1, C) - AT(img, R - 1, C)) * deriv_scale;
    const float dD2 = (AT(next, R, C) - AT(prev, R, C)) * deriv_scale;
    float t = 0;
    t += dD0 * xc;
    t += dD1 * xr;
    t += dD2 * xi;
    contr = AT(img, R, C) * img_scale + t * 0.5f;
    if (fabsf(contr) * L < contrastThreshold) return 0;
    const float v2 = AT(img, R, C) * 2.f;
    const float dxx = (AT(img, R, C + 1) + AT(img, R, C - 1) - v2) * second_deriv_scale;
    const float dyy = (AT(img, R + 1, C) + AT(img, R - 1, C) - v2) * second_deriv_scale;
    const float dxy = (AT(img, R + 1, C + 1) - AT(img, R + 1, C - 1) - AT(img, R - 1, C + 1) +
                       AT(img, R - 1, C - 1)) * cross_deriv_scale;
    const float tr = dxx + dyy;
    const float det = dxx * dyy - dxy * dxy;
    if (det <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * det)
      return 0;
  }
  kpt->x = (*c + xc) * (1 << octv);
  kpt->y = (*r + xr) * (1 << octv);
  kpt->octave = octv + (*layer << 8) + (cv_round_d((xi + 0.5) * 255) << 16);
  /* powf(2, (layer + xi) / L) as e^(y ln2) through s_exp */
  kpt->size = sigma * (float)s_exp((double)((*layer + xi) / L) * 0.6931471805599453) * (1 << octv) * 2;
  kpt->response = fabsf(contr);
  return 1;
}

/* calcOrientationHist (sift.simd.hpp) -> smoothed hist[n], returns its maximum */
static float calc_orientation_hist(const img_t* img, int px, int py, int radius, float sigma,
                                   float* hist, int n) {
  const float expf_scale = -1.f / (2.f * sigma * sigma);
  float tmp[SIFT_ORI_HIST_BINS + 4];
  float* temphist = tmp + 2;
  for (int i = 0; i < n; i++) temphist[i] = 0.f;
  for (int i = -radius; i <= radius; i++) {
    const int y = py + i;
    if (y <= 0 || y >= img->h - 1) continue;
    for (int j = -radius; j <= radius; j++) {
      const int x = px + j;
      if (x <= 0 || x >= img->w - 1) continue;
      const float dx = AT(*img, y, x + 1) - AT(*img, y, x - 1);
      const float dy = AT(*img, y - 1, x) - AT(*img, y + 1, x);
      const float w = fexp((i * i + j * j) * expf_scale);
      const float ori = sift_fast_atan2(dy, dx);
      const float mag = fmag(dx, dy);
      int bin = cv_round_f((n / 360.f) * ori);
      if (bin >= n) bin -= n;
      if (bin < 0) bin += n;
      temphist[bin] += w * mag;
    }
  }
  temphist[-1] = temphist[n - 1];
  temphist[-2] = temphist[n - 2];
  temphist[n] = temphist[0];
  temphist[n + 1] = temphist[1];
  for (int i = 0; i < n; i++)
    hist[i] = (temphist[i - 2] + temphist[i + 2]) * (1.f / 16.f) +
              (temphist[i - 1] + temphist[i + 1]) * (4.f / 16.f) + temphist[i] * (6.f / 16.f);
  float maxval = hist[0];
  for (int i = 1; i < n; i++) maxval = fmaxf(maxval, hist[i]);
  return maxval;
}

typedef struct {
  kp_t* v;
  int n, cap;
} kpvec_t;

static void kp_push(kpvec_t* V, kp_t k) {
  if (V->n == V->cap) {
    V->cap = V->cap ? 2 * V->cap : 1024;
    V->v = (kp_t*)realloc(V->v, sizeof(kp_t) * V->cap);
  }
  V->v[V->n++] = k;
}

static void find_extrema(const pyr_t* P, kpvec_t* out, float contrastThreshold,
                         float edgeThreshold, float sigma) {
  const int L = P->L, n = SIFT_ORI_HIST_BINS;
  const int threshold = cv_floor_d(0.5 * contrastThreshold / L * 255 * 1);
  float hist[SIFT_ORI_HIST_BINS];
  for (int o = 0; o < P->nOct; o++)
    for (int i = 1; i <= L; i++) {
      const int idx = o * (L + 2) + i;
      const img_t img = P->d[idx], prev = P->d[idx - 1], next = P->d[idx + 1];
      const int rows = img.h, cols = img.w;
      for (int r = SIFT_IMG_BORDER; r < rows - SIFT_IMG_BORDER; r++)
        for (int c = SIFT_IMG_BORDER; c < cols - SIFT_IMG_BORDER; c++) {
          const float val = AT(img, r, c);
          if (!(fabsf(val) > threshold)) continue;
          int ext = 1;
          for (int dl = -1; dl <= 1 && ext; dl++) {
            const img_t* m = dl < 0 ? &prev : dl > 0 ? &next : &img;
            for (int dy = -1; dy <= 1 && ext; dy++)
              for (int dx = -1; dx <= 1; dx++) {
                if (!dl && !dy && !dx) continue;
                const float v = AT(*m, r + dy, c + dx);
                if (val > 0 ? !(val >= v) : !(val <= v)) {
                  ext = 0;
                  break;
                }
              }
          }
          if (!ext) continue;
          kp_t kpt;
          int r1 = r, c1 = c, layer = i;
          if (!adjust_local_extrema(P, &kpt, o, &layer, &r1, &c1, contrastThreshold,
                                    edgeThreshold, sigma))
            continue;
          const float scl_octv = kpt.size * 0.5f / (1 << o);
          const float omax = calc_orientation_hist(&P->g[o * (L + 3) + layer], c1, r1,
                                                   cv_round_f(SIFT_ORI_RADIUS * scl_octv),
                                                   SIFT_ORI_SIG_FCTR * scl_octv, hist, n);
          const float mag_thr = omax * SIFT_ORI_PEAK_RATIO;
          for (int j = 0; j < n; j++) {
            const int l = j > 0 ? j - 1 : n - 1;
            const int r2 = j < n - 1 ? j + 1 : 0;
            if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
              float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
              bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
              kpt.angle = 360.f - (float)((360.f / n) * bin);
              if (fabsf(kpt.angle - 360.f) < FLT_EPSILON) kpt.angle = 0.f;
              kp_push(out, kpt);
            }
          }
        }
    }
}

/* KeyPoint12_LessThan (class_id is -1 for every SIFT keypoint) */
static int kp_cmp(const void* pa, const void* pb) {
  const kp_t* a = (const kp_t*)pa;
  const kp_t* b = (const kp_t*)pb;
  if (a->x != b->x) return a->x < b->x ? -1 : 1;
  if (a->y != b->y) return a->y < b->y ? -1 : 1;
  if (a->size != b->size) return a->size > b->size ? -1 : 1;
  if (a->angle != b->angle) return a->angle < b->angle ? -1 : 1;
  if (a->response != b->response) return a->response > b->response ? -1 : 1;
  if (a->octave != b->octave) return a->octave > b->octave ? -1 : 1;
  return 0;
}

static int remove_duplicated_sorted(kp_t* v, int n) {
  if (n < 2) return n;
  qsort(v, n, sizeof(kp_t), kp_cmp);
  int i = 0;
  for (int j = 1; j < n; ++j) {
    const kp_t* a = &v[i];
    const kp_t* b = &v[j];
    if (a->x != b->x || a->y != b->y || a->size != b->size || a->angle != b->angle) v[++i] = v[j];
  }
  return i + 1;
}

/* calcSIFTDescriptor (sift.simd.hpp), d = 4, n = 8, float output row */
static void calc_descriptor(const img_t* img, float ptx, float pty, float ori, float scl,
                            float* dst) {
  const int d = SIFT_DESCR_WIDTH, n = SIFT_DESCR_HIST_BINS;
  const int px = cv_round_f(ptx), py = cv_round_f(pty);
  double sd, cd;
  s_sincos((double)(ori * (float)(3.14159265358979323846 / 180)), &sd, &cd);
  float cos_t = (float)cd;
  float sin_t = (float)sd;
  const float bins_per_rad = n / 360.f;
  const float exp_scale = -1.f / (d * d * 0.5f);
  const float hist_width = SIFT_DESCR_SCL_FCTR * scl;
  int radius = cv_round_f(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
  const int diag = (int)sqrt(((double)img->w) * img->w + ((double)img->h) * img->h);   /* exact floor */
  if (radius > diag) radius = diag;
  cos_t /= hist_width;
  sin_t /= hist_width;
  const int rows = img->h, cols = img->w;
  float hist[(SIFT_DESCR_WIDTH + 2) * (SIFT_DESCR_WIDTH + 2) * (SIFT_DESCR_HIST_BINS + 2)];
  float raw[SIFT_DESCR_WIDTH * SIFT_DESCR_WIDTH * SIFT_DESCR_HIST_BINS];
  memset(hist, 0, sizeof(hist));
  for (int i = -radius; i <= radius; i++)
    for (int j = -radius; j <= radius; j++) {
      const float c_rot = j * cos_t - i * sin_t;
      const float r_rot = j * sin_t + i * cos_t;
      float rbin = r_rot + d / 2 - 0.5f;
      float cbin = c_rot + d / 2 - 0.5f;
      const int r = py + i, c = px + j;
      if (!(rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < rows - 1 && c > 0 &&
            c < cols - 1))
        continue;
      const float dx = AT(*img, r, c + 1) - AT(*img, r, c - 1);
      const float dy = AT(*img, r - 1, c) - AT(*img, r + 1, c);
      const float wexp = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
      const float o_k = sift_fast_atan2(dy, dx);
      const float mag_k = fmag(dx, dy);
      const float w_k = fexp(wexp);
      float obin = (o_k - ori) * bins_per_rad;
      const float mag = mag_k * w_k;
      const int r0 = cv_floor_f(rbin), c0 = cv_floor_f(cbin);
      int o0 = cv_floor_f(obin);
      rbin -= r0;
      cbin -= c0;
      obin -= o0;
      if (o0 < 0) o0 += n;
      if (o0 >= n) o0 -= n;
      const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
      const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
      const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
      const float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
      const float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
      const float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
      const float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
      const int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
      hist[idx] += v_rco000;
      hist[idx + 1] += v_rco001;
      hist[idx + (n + 2)] += v_rco010;
      hist[idx + (n + 3)] += v_rco011;
      hist[idx + (d + 2) * (n + 2)] += v_rco100;
      hist[idx + (d + 2) * (n + 2) + 1] += v_rco101;
      hist[idx + (d + 3) * (n + 2)] += v_rco110;
      hist[idx + (d + 3) * (n + 2) + 1] += v_rco111;
    }
  for (int i = 0; i < d; i++)
    for (int j = 0; j < d; j++) {
      const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
      hist[idx] += hist[idx + n];
      hist[idx + 1] += hist[idx + n + 1];
      for (int k = 0; k < n; k++) raw[(i * d + j) * n + k] = hist[idx + k];
    }
  const int len = d * d * n;
  float nrm2 = 0;
  for (int k = 0; k < len; k++) nrm2 += raw[k] * raw[k];
  const float thr = (float)sqrt((double)nrm2) * SIFT_DESCR_MAG_THR;
  nrm2 = 0;
  for (int i = 0; i < len; i++) {
    const float val = fminf(raw[i], thr);
    raw[i] = val;
    nrm2 += val * val;
  }
  nrm2 = SIFT_INT_DESCR_FCTR / fmaxf((float)sqrt((double)nrm2), FLT_EPSILON);
  for (int k = 0; k < len; k++) {
    const int v = cv_round_f(raw[k] * nrm2);
    dst[k] = (float)(v < 0 ? 0 : v > 255 ? 255 : v);
  }
}

/* detectAndCompute(gray, None).  Writes min(n, cap) keypoints (+ descriptors when desc is
 * non-null) and returns n (the full count), or -1 on bad arguments. */
int sift_oracle_detect(const uint8_t* gray, int w, int h, int L, double contrastThreshold,
                       double edgeThreshold, double sigma, int cap, float* kx, float* ky,
                       float* ksize, float* kangle, float* kresp, int* koct, float* desc) {
  if (!gray || w < 1 || h < 1 || L < 1 || L > 16) return -1;
  pyr_t P = build_pyramid(gray, w, h, L, sigma);
  kpvec_t V = {0, 0, 0};
  find_extrema(&P, &V, (float)contrastThreshold, (float)edgeThreshold, (float)sigma);
  const int n = remove_duplicated_sorted(V.v, V.n);
  const float scale = 1.f / (float)(1 << -FIRST_OCTAVE);
  for (int i = 0; i < n; i++) {
    kp_t* k = &V.v[i];
    k->octave = (k->octave & ~255) | ((k->octave + FIRST_OCTAVE) & 255);
    k->x *= scale;
    k->y *= scale;
    k->size *= scale;
  }
  const int m = n < cap ? n : cap;
  for (int i = 0; i < m; i++) {
    const kp_t* k = &V.v[i];
    if (kx) kx[i] = k->x;
    if (ky) ky[i] = k->y;
    if (ksize) ksize[i] = k->size;
    if (kangle) kangle[i] = k->angle;
    if (kresp) kresp[i] = k->response;
    if (koct) koct[i] = k->octave;
    if (desc) {
      /* calcDescriptors: unpackOctave, layer image, descriptor at octave scale */
      int octave = k->octave & 255;
      const int layer = (k->octave >> 8) & 255;
      octave = octave < 128 ? octave : (-128 | octave);
      const float sc = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
      const float size = k->size * sc;
      const img_t* img = &P.g[(octave - FIRST_OCTAVE) * (L + 3) + layer];
      float angle = 360.f - k->angle;
      if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
      calc_descriptor(img, k->x * sc, k->y * sc, angle, size * 0.5f, desc + (size_t)i * 128);
    }
  }
  free(V.v);
  free_pyramid(&P);
  return n;
}

/* one Gaussian (kind 0) or DoG (kind 1) layer of the pyramid, for layer-wise parity
 * checks; returns the layer's w*h or -1 (dims via *ow, *oh; out may be null) */
int sift_oracle_layer(const uint8_t* gray, int w, int h, int L, double sigma, int kind,
                      int octave, int layer, float* out, int* ow, int* oh) {
  pyr_t P = build_pyramid(gray, w, h, L, sigma);
  int ret = -1;
  if (octave >= 0 && octave < P.nOct && layer >= 0 && layer < L + 3 - kind) {
    const img_t* m = kind ? &P.d[octave * (L + 2) + layer] : &P.g[octave * (L + 3) + layer];
    if (ow) *ow = m->w;
    if (oh) *oh = m->h;
    if (out) memcpy(out, m->p, sizeof(float) * m->w * m->h);
    ret = m->w * m->h;
  }
  free_pyramid(&P);
  return ret;
}

/* cvtColor(BGR2GRAY) for 8-bit: (B*1868 + G*9617 + R*4899 + 2^13) >> 14 */
void sift_oracle_bgr2gray(const uint8_t* bgr, int64_t npix, uint8_t* gray) {
  for (int64_t i = 0; i < npix; i++)
    gray[i] = (uint8_t)((bgr[3 * i] * 1868 + bgr[3 * i + 1] * 9617 + bgr[3 * i + 2] * 4899 +
                         (1 << 13)) >> 14);
}
