// The solver's transcendental functions on its hot loops (the barrier's log per bounded variable, the stage
// dynamics' sin / cos / tan): plain double arithmetic with explicit fused multiply-adds, so the device and every
// host build return the same doubles (the bit-exact device emulation, csrc/emu_wave.h), within 2 ulp (tan 3) of the
// true value (tests/test_libm_cpu.py) and at the cost of the platform libm -- unlike the double-double
// correctly rounded htp_libm.h, whose log in the barrier cost 13 % of an IPM iteration (profiles/r04g_ab_D.txt).
// Arguments beyond the fast reduction's range go to htp_libm.h.
#pragma once
#include <cmath>

#ifndef HTP_HD
#error "define HTP_HD before including htp_fastm.h"
#endif

#include "htp_libm.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#elif defined(__GNUC__)
#pragma GCC push_options
#pragma GCC optimize("fp-contract=off")
#endif

namespace htp {
namespace fm {

// Polynomials: Chebyshev fits (mpmath.chebyfit, 120 bits) in z = s^2 or r^2, evaluated by Estrin's scheme (three
// dependent fused multiply-adds instead of six: one wavefront per SIMD hides no latency).
// log(m) = 2 atanh(s) = 2 s + 2 s z R(z), s = (m - 1) / (m + 1), z <= ((sqrt 2 - 1) / (sqrt 2 + 1))^2: |R err| 1.6e-16
constexpr double LOG_C[7] = {0.3333333333333335, 0.19999999999949752, 0.14285714312987743, 0.1111110556739754,
                             0.09091444562630861, 0.07665860800278021, 0.07308224842521703};
// sin r = r + r z S(z), cos r = 1 + z C(z), z = r^2 <= (pi / 4)^2: |S err| 2.0e-17, |C err| 2.0e-19
constexpr double SIN_C[6] = {-0.16666666666666666, 0.008333333333330948, -0.00019841269836756774,
                             2.7557316101617874e-06, -2.505113165023518e-08, 1.5918115263265974e-10};
constexpr double COS_C[7] = {-0.5, 0.04166666666666664, -0.001388888888888077, 2.4801587293690305e-05,
                             -2.755731556524682e-07, 2.0875886564482672e-09, -1.1367988423294987e-11};
constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;   // LN2_HI: 32 bits
constexpr double SQRT1_2 = 0.70710678118654752440;

HTP_HD inline double estrin6(const double* c, double z, double z2, double z4) {
  return std::fma(std::fma(c[5], z, c[4]), z4, std::fma(std::fma(c[3], z, c[2]), z2, std::fma(c[1], z, c[0])));
}
HTP_HD inline double estrin7(const double* c, double z, double z2, double z4) {
  return std::fma(std::fma(c[6], z2, std::fma(c[5], z, c[4])), z4,
                  std::fma(std::fma(c[3], z, c[2]), z2, std::fma(c[1], z, c[0])));
}

// The rare arguments go to htp_libm.h through out-of-line calls that return by value, so the fast paths below
// inline into the solver's loops without the double-double code (the compiler would otherwise outline the whole
// function, and every call site pays the caller-saved register spills of a 512-register kernel).
#if defined(__GNUC__) || defined(__clang__)
#define HTP_FM_NOINLINE __attribute__((noinline)) inline
#define HTP_FM_INLINE __attribute__((always_inline)) inline
#else
#define HTP_FM_NOINLINE inline
#define HTP_FM_INLINE inline
#endif
struct SinCos { double s, c; };
HTP_HD HTP_FM_NOINLINE double log_slow(double x) { return hm::log(x); }
HTP_HD HTP_FM_NOINLINE SinCos sincos_slow(double x) { SinCos r; hm::sincos(x, r.s, r.c); return r; }

HTP_HD HTP_FM_INLINE double log(double x) {
  if (!(x > 0.0) || x == __builtin_huge_val()) return log_slow(x);   // 0, negative, NaN, +inf
  int e;
  double m = std::frexp(x, &e);           // x = m 2^e, m in [0.5, 1) (subnormals included)
  if (m < SQRT1_2) { m *= 2.0; --e; }     // m in [sqrt(1/2), sqrt 2)
  const double f = m - 1.0;               // exact (Sterbenz)
  const double s = f / (2.0 + f);
  const double z = s * s, z2 = z * z;
  const double p = estrin7(LOG_C, z, z2, z2 * z2);
  // 2 s (1 + z p) = f - f s + 2 s z p   (f = 2 s + f s: the leading term without the division's rounding)
  const double fs = f * s;
  const double r = std::fma(2.0 * s, z * p, -fs) + f;
  const double ed = (double)e;
  return std::fma(ed, LN2_HI, std::fma(ed, LN2_LO, r));
}

// pi / 2 in three parts of 33, 33 and 53 bits (k * PIO2_A, k * PIO2_B exact for |k| < 2^20)
constexpr double PIO2_A = 1.57079632673412561417e+00, PIO2_B = 6.07710050630396597660e-11,
                 PIO2_C = 2.02226624879595063154e-21, INV_PIO2 = 6.36619772367581382433e-01;

HTP_HD HTP_FM_INLINE void sincos(double x, double& s, double& c) {
  if (!(std::fabs(x) < 0x1p20)) { const SinCos r = sincos_slow(x); s = r.s; c = r.c; return; }   // large, inf, NaN
  const double k = rint(x * INV_PIO2);
  const double r = std::fma(-k, PIO2_C, std::fma(-k, PIO2_B, std::fma(-k, PIO2_A, x)));
  const int q = (int)((long long)k & 3);
  const double z = r * r, z2 = z * z, z4 = z2 * z2;
  const double sr = std::fma(r * z, estrin6(SIN_C, z, z2, z4), r), cr = std::fma(z, estrin7(COS_C, z, z2, z4), 1.0);
  s = (q & 1) ? cr : sr;
  c = (q & 1) ? sr : cr;
  if (q & 2) s = -s;
  if (((q + 1) & 2) != 0) c = -c;
}
HTP_HD HTP_FM_INLINE double sin(double x) { double s, c; sincos(x, s, c); return s; }
HTP_HD HTP_FM_INLINE double cos(double x) { double s, c; sincos(x, s, c); return c; }
HTP_HD HTP_FM_INLINE double tan(double x) { double s, c; sincos(x, s, c); return s / c; }

}  // namespace fm
}  // namespace htp

#if !defined(__clang__) && defined(__GNUC__)
#pragma GCC pop_options
#endif
