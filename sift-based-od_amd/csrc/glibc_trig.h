// glibc_trig.h -- glibc's double sin / cos, bit for bit, on the host and on the device.
//
// Licence: this file restates the algorithm of the GNU C Library's
// sysdeps/ieee754/dbl-64/s_sin.c (glibc 2.35; Copyright (C) 2001-2022 Free Software
// Foundation, Inc., originally IBM Accurate Mathematical Library, written by International
// Business Machines Corp.), and glibc_trig_tab.h holds that library's constants and sin / cos
// table.  The GNU C Library is free software under the GNU Lesser General Public License,
// version 2.1 or (at your option) any later version; this file and glibc_trig_tab.h are
// distributed under those same terms (LGPL-2.1-or-later), separately from the rest of this
// repository.  See https://www.gnu.org/licenses/old-licenses/lgpl-2.1.html.
//
// Why: HoughTransformHelperFunctions.py:31-35 (estimate_object_pose) rotates each match's
// model offset with Python's math.cos / math.sin, i.e. glibc's libm.  Those results are not
// correctly rounded (about 0.15 % of angles in [0, 2 pi) differ from the correctly rounded
// value, tools/glibc_trig_cr_check.py), so no other implementation -- ocml's, or a correctly
// rounded one -- reproduces them; the PoseBin means of PoseBin.py:20-28 and, through them,
// post-processing's `<=` clusters (PostProcessing.py:22-28) and the final pose follow those
// last bits.  This is a restatement of glibc 2.35's sysdeps/ieee754/dbl-64/s_sin.c as the
// x86_64 libm runs it on an FMA / AVX2 CPU (the __sin_fma / __cos_fma ifunc variants: s_sin.c
// compiled with -mfma -mavx2, where GCC contracted a * b + c into fused multiply-adds); every
// fma() below is one the compiled code has, every other operation is rounded on its own (this
// header must be compiled with -ffp-contract=off).  The constants and the 440-entry table are
// the library's own bit patterns (glibc_trig_tab.h, tools/gen_glibc_trig.py).
// Range: |x| < 105414350 (beyond it glibc reduces with __branred: not restated; the pose
// angles are in [0, 2 pi)); gt_supported() tells.  Checked against the host's glibc on
// 10^8+ arguments by tools/glibc_trig_check.cpp (tests/test_glibc_trig.py).
#pragma once
#include <math.h>
#include <stdint.h>

#include "glibc_trig_tab.h"

#ifdef __HIPCC__
#define GT_HD __host__ __device__ __forceinline__
#else
#define GT_HD static inline
#endif

namespace gtrig {

#if defined(__HIP_DEVICE_COMPILE__)
static __device__ const uint64_t kTab[GT_TAB_N] = GT_TAB_INIT;
#else
static const uint64_t kTab[GT_TAB_N] = GT_TAB_INIT;
#endif

GT_HD double bits(uint64_t u) { return __builtin_bit_cast(double, u); }
GT_HD uint64_t ubits(double d) { return __builtin_bit_cast(uint64_t, d); }
GT_HD double tab(int i) { return bits(kTab[i]); }

// TAYLOR_SIN(a*a, a, da): a - a^3/3! + ... with the da correction, |a| < 0.126
GT_HD double taylor_sin(double a, double da) {
  const double xx = a * a;
  double p = fma(xx, bits(GT_S5), bits(GT_S4));
  p = fma(xx, p, bits(GT_S3));
  p = fma(xx, p, bits(GT_S2));
  p = fma(xx, p, bits(GT_S1));
  const double t1 = fma(p, a, -(da * 0.5));
  return a + fma(xx, t1, da);
}

// do_sin(x, dx): sin(x + dx) from the table entry nearest |x| (x multiple of 1/128)
GT_HD double do_sin(double x, double dx) {
  if (fabs(x) < bits(GT_C0126)) return taylor_sin(x, dx);
  if (x <= 0) dx = -dx;
  const double ax = fabs(x);
  const double u = bits(GT_BIG) + ax;
  const int k = (int)(uint32_t)ubits(u) << 2;
  const double xr = ax - (u - bits(GT_BIG));
  const double xx = xr * xr;
  const double s = xr + fma(xr * xx, fma(xx, bits(GT_SN5), bits(GT_SN3)), dx);
  const double c = fma(xr, dx, xx * fma(xx, fma(xx, bits(GT_CS6), bits(GT_CS4)), bits(GT_CS2)));
  const double sn = tab(k), ssn = tab(k + 1), cs = tab(k + 2), ccs = tab(k + 3);
  const double cor = fma(s, cs, fma(-c, sn, fma(s, ccs, ssn)));
  return copysign(sn + cor, x);
}

// do_cos(x, dx): cos(x + dx)
GT_HD double do_cos(double x, double dx) {
  if (x < 0) dx = -dx;
  const double ax = fabs(x);
  const double u = bits(GT_BIG) + ax;
  const int k = (int)(uint32_t)ubits(u) << 2;
  const double xr = ax - (u - bits(GT_BIG)) + dx;
  const double xx = xr * xr;
  const double s = fma(xr * xx, fma(xx, bits(GT_SN5), bits(GT_SN3)), xr);
  const double c = xx * fma(xx, fma(xx, bits(GT_CS6), bits(GT_CS4)), bits(GT_CS2));
  const double sn = tab(k), ssn = tab(k + 1), cs = tab(k + 2), ccs = tab(k + 3);
  const double cor = fma(-s, sn, fma(-c, cs, fma(-s, ssn, ccs)));
  return cs + cor;
}

// reduce_sincos: x - n pi/2 as a + da, n mod 4 (|x| < 105414350)
GT_HD int reduce(double x, double* a, double* da) {
  const double t = fma(x, bits(GT_HPINV), bits(GT_TOINT));
  const double xn = t - bits(GT_TOINT);
  const int n = (int)(ubits(t) & 3);
  const double y = fma(-xn, bits(GT_MP2), fma(-xn, bits(GT_MP1), x));
  const double t2 = fma(-xn, bits(GT_PP3), y);
  double db = fma(-xn, bits(GT_PP3), y - t2);
  const double b = fma(-xn, bits(GT_PP4), t2);
  db += fma(-xn, bits(GT_PP4), t2 - b);
  *a = b;
  *da = db;
  return n;
}

GT_HD double do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}

GT_HD bool supported(double x) { return fabs(x) < 105414350.0; }

GT_HD double sin(double x) {
  const uint32_t k = (uint32_t)(ubits(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e500000u) return x;
  if (k < 0x3feb6000u) return do_sin(x, 0.0);
  if (k < 0x400368fdu) return copysign(do_cos(bits(GT_HP0) - fabs(x), bits(GT_HP1)), x);
  if (k < 0x419921fbu) {
    double a, da;
    const int n = reduce(x, &a, &da);
    return do_sincos(a, da, n);
  }
  return __builtin_nan("");   // not restated (__branred); callers check supported()
}

GT_HD double cos(double x) {
  const uint32_t k = (uint32_t)(ubits(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e400000u) return 1.0;
  if (k < 0x3feb6000u) return do_cos(x, 0.0);
  if (k < 0x400368fdu) {
    const double y = bits(GT_HP0) - fabs(x);
    const double a = y + bits(GT_HP1);
    const double da = (y - a) + bits(GT_HP1);
    return do_sin(a, da);
  }
  if (k < 0x419921fbu) {
    double a, da;
    const int n = reduce(x, &a, &da);
    return do_sincos(a, da, n + 1);
  }
  return __builtin_nan("");
}

}  // namespace gtrig
