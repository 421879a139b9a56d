// Host check of glibc_trig.h against the host's own glibc sin / cos, bit for bit.
//   g++ -O2 -std=c++17 -ffp-contract=off -mfma tools/glibc_trig_check.cpp -o /tmp/gtc && /tmp/gtc [n]
// Ranges: the pose angles [0, 2 pi); each branch of s_sin.c around its bounds; [-100, 100];
// log-uniform magnitudes 2^-30 .. 2^26.  Prints mismatches per range; exit 1 on any.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../sift-based-od_amd/csrc/glibc_trig.h"

// through volatile pointers: GCC folds sin(x) and cos(x) of one argument into a sincos()
// call, whose last bits differ from sin's and cos's (what Python's math.sin / math.cos call)
static double (*volatile g_sin)(double) = ::sin;
static double (*volatile g_cos)(double) = ::cos;

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  struct R { const char* name; double lo, hi; bool logu; };
  const R ranges[] = {{"[0,2pi)", 0.0, 6.283185307179586, false},
                      {"taylor |x|<0.126", -0.126, 0.126, false},
                      {"[0.126,0.8555)", 0.126, 0.855469, false},
                      {"[0.8555,2.4263)", 0.855469, 2.426265, false},
                      {"[2.4263,100)", 2.426265, 100.0, false},
                      {"[-100,100]", -100.0, 100.0, false},
                      {"log 2^-30..2^26", -30.0, 26.0, true}};
  long bad_total = 0;
  for (const R& r : ranges) {
    long bs = 0, bc = 0;
    for (long i = 0; i < n; ++i) {
      double x = r.logu ? std::ldexp(1.0, 0) * std::exp2(r.lo + (r.hi - r.lo) * u01(rng)) * (rng() & 1 ? 1 : -1)
                        : r.lo + (r.hi - r.lo) * u01(rng);
      const double s0 = g_sin(x), c0 = g_cos(x);
      const double s1 = gtrig::sin(x), c1 = gtrig::cos(x);
      if (__builtin_bit_cast(uint64_t, s0) != __builtin_bit_cast(uint64_t, s1)) {
        if (bs < 3) printf("  sin(%.17g) glibc %.17g replica %.17g\n", x, s0, s1);
        ++bs;
      }
      if (__builtin_bit_cast(uint64_t, c0) != __builtin_bit_cast(uint64_t, c1)) {
        if (bc < 3) printf("  cos(%.17g) glibc %.17g replica %.17g\n", x, c0, c1);
        ++bc;
      }
    }
    printf("%-18s %ld args: sin mismatches %ld, cos mismatches %ld\n", r.name, n, bs, bc);
    bad_total += bs + bc;
  }
  // branch edges: ulp neighbourhoods of every threshold and of k/128 table points
  const double edges[] = {0.126, 0.855469, 2.426265, 1.4901161193847656e-08, 7.450580596923828e-09,
                          0.855468750, 2.4262652397155762, 3.141592653589793, 6.283185307179586,
                          1.5707963267948966, 4.71238898038469};
  long be = 0, ne = 0;
  for (double e : edges)
    for (int s = -1; s <= 1; s += 2) {
      double x = s * e;
      for (int k = 0; k < 2000; ++k) {
        x = std::nextafter(x, s > 0 ? 10.0 : -10.0);
        ++ne;
        be += __builtin_bit_cast(uint64_t, g_sin(x)) != __builtin_bit_cast(uint64_t, gtrig::sin(x));
        be += __builtin_bit_cast(uint64_t, g_cos(x)) != __builtin_bit_cast(uint64_t, gtrig::cos(x));
      }
    }
  for (int i = 0; i < 110; ++i)
    for (int k = -500; k <= 500; ++k) {
      const double x = std::nextafter(i / 128.0, 1.0) + k * 1e-18 * (i + 1);
      ++ne;
      be += __builtin_bit_cast(uint64_t, g_sin(x)) != __builtin_bit_cast(uint64_t, gtrig::sin(x));
      be += __builtin_bit_cast(uint64_t, g_cos(x)) != __builtin_bit_cast(uint64_t, gtrig::cos(x));
    }
  printf("edges / table points: %ld args, mismatches %ld\n", ne, be);
  bad_total += be;
  printf(bad_total ? "FAIL\n" : "OK\n");
  return bad_total ? 1 : 0;
}
