// Deterministic double-double libm for the planner cores (sin, cos, tan, atan, atan2, asin, acos, hypot, pow), one
// __host__ __device__ source for the gfx950 kernels and every host build of the same cores.
//
// Why: integer outputs of the reference's planners hang on the last bit of a transcendental.  A spline piece
// has len(np.arange(0, s[-1] + ds, ds)) samples (R/path_planner/utils/cubic_spline.py:102) and pydubins
// samples at the step the spline then resamples at, so s[-1] sits on a multiple of ds and one ulp of a sin or
// hypot flips the count.  ocml (device) and glibc (host) round differently (glibc 2.35 itself misrounds
// ~0.1 % of sin/cos/atan/atan2/asin/acos/pow arguments; numpy's AVX-512 arctan2/hypot/tan differ from
// glibc on 7.8 % / 0.6 % / 0.5 %: tools/libm_check.py, profiles/r04_libm_check.json).  Evaluating every
// function in double-double (error < 2^-100 relative before the final rounding) and rounding once gives the
// same double on both sides of the boundary (the same operations in the same order), so the device and the
// host builds produce the same doubles by construction.  There is no Ziv rounding test with a higher-precision
// fallback: an argument whose exact result lies within 2^-100 of a rounding boundary can still round the wrong
// way -- identically on both sides.  On 10^7 random arguments per function no misrounding was found
// (tools/libm_check.py), so "correctly rounded" below means "in every case tested", not a proof.  Arithmetic: explicit fma only (exact on both sides), no contraction.
//
// HTP_LIBM_PLATFORM (host builds only): forward to the platform libm instead -- the build that reproduces the
// reference's own doubles where they were produced by CPython's math module (golden-vector tests).
//
// Domain: double-double accurate for finite arguments with |x| < 2^30 (sin, cos, tan) and normal results; C99
// special values (zeros, infinities, NaN) follow glibc.  Constants: tools/gen_libm_consts.py (mpmath).
#pragma once
#include <cmath>

#ifndef HTP_HD
#error "define HTP_HD before including htp_libm.h"
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#elif defined(__GNUC__)
#pragma GCC push_options
#pragma GCC optimize("fp-contract=off")
#endif

namespace htp {
namespace hm {

#if defined(HTP_LIBM_PLATFORM) && !defined(__HIP_DEVICE_COMPILE__)
inline double sin(double x) { return std::sin(x); }
inline double cos(double x) { return std::cos(x); }
inline double tan(double x) { return std::tan(x); }
inline double atan(double x) { return std::atan(x); }
inline double atan2(double y, double x) { return std::atan2(y, x); }
inline double asin(double x) { return std::asin(x); }
inline double acos(double x) { return std::acos(x); }
inline double hypot(double x, double y) { return std::hypot(x, y); }
inline double pow(double x, double y) { return std::pow(x, y); }
inline double log(double x) { return std::log(x); }
inline void sincos(double x, double& s, double& c) { s = std::sin(x); c = std::cos(x); }
#else

// ---- constants (tools/gen_libm_consts.py)
// pi/2 = PIO2_1 + PIO2_2 + PIO2_3 (+ 2^-160)
constexpr double PIO2_1 = 1.5707963267948966, PIO2_2 = 6.123233995736766e-17, PIO2_3 = -1.4973849048591698e-33;
constexpr unsigned TWO_OVER_PI_BITS[44] = {  // 2/pi = sum_j limb_j 2^(-32 (j + 1))
    0xa2f9836eu, 0x4e441529u, 0xfc2757d1u, 0xf534ddc0u, 0xdb629599u, 0x3c439041u,
    0xfe5163abu, 0xdebbc561u, 0xb7246e3au, 0x424dd2e0u, 0x06492eeau, 0x09d1921cu,
    0xfe1deb1cu, 0xb129a73eu, 0xe88235f5u, 0x2ebb4484u, 0xe99c7026u, 0xb45f7e41u,
    0x3991d639u, 0x835339f4u, 0x9c845f8bu, 0xbdf9283bu, 0x1ff897ffu, 0xde05980fu,
    0xef2f118bu, 0x5a0a6d1fu, 0x6d367ecfu, 0x27cb09b7u, 0x4f463f66u, 0x9e5fea2du,
    0x7527bac7u, 0xebe5f17bu, 0x3d0739f7u, 0x8a5292eau, 0x6bfb5fb1u, 0x1f8d5d08u,
    0x56033046u, 0xfc7b6babu, 0xf0cfbc20u, 0x9af4361du, 0xa9e39161u, 0x5ee61b08u,
    0x6599855fu, 0x14a06840u,
};
constexpr double PIO2_4 = 5.562271104316826e-50;
constexpr double PI_H = 3.141592653589793, PI_L = 1.2246467991473532e-16;
constexpr double PIO2_H = 1.5707963267948966, PIO2_L = 6.123233995736766e-17;
constexpr double PIO4_H = 0.7853981633974483, PIO4_L = 3.061616997868383e-17;
constexpr double PI34_H = 2.356194490192345, PI34_L = 9.184850993605148e-17;
constexpr double TWO_OVER_PI = 0.6366197723675814;
constexpr double LN2_1 = 0.6931471805599453, LN2_2 = 2.3190468138462996e-17, LN2_3 = 5.707708438416212e-34;
constexpr double INV_LN2 = 1.4426950408889634;
constexpr double SIN_C[14][2] = {
    {1.0, 0.0},
    {-0.16666666666666666, -9.25185853854297e-18},
    {0.008333333333333333, 1.1564823173178714e-19},
    {-0.0001984126984126984, -1.7209558293420705e-22},
    {2.7557319223985893e-06, -1.858393274046472e-22},
    {-2.505210838544172e-08, 1.448814070935912e-24},
    {1.6059043836821613e-10, 1.2585294588752098e-26},
    {-7.647163731819816e-13, -7.03872877733453e-30},
    {2.8114572543455206e-15, 1.6508842730861433e-31},
    {-8.22063524662433e-18, -2.2141894119604265e-34},
    {1.9572941063391263e-20, -1.3643503830087908e-36},
    {-3.868170170630684e-23, 8.843177655482344e-40},
    {6.446950284384474e-26, -1.9330404233703465e-42},
    {-9.183689863795546e-29, -1.4303150396787322e-45},
};
constexpr double COS_C[15][2] = {
    {1.0, 0.0},
    {-0.5, 0.0},
    {0.041666666666666664, 2.3129646346357427e-18},
    {-0.001388888888888889, 5.300543954373577e-20},
    {2.48015873015873e-05, 2.1511947866775882e-23},
    {-2.755731922398589e-07, -2.3767714622250297e-23},
    {2.08767569878681e-09, -1.20734505911326e-25},
    {-1.1470745597729725e-11, -2.0655512752830745e-28},
    {4.779477332387385e-14, 4.399205485834081e-31},
    {-1.5619206968586225e-16, -1.1910679660273754e-32},
    {4.110317623312165e-19, 1.4412973378659527e-36},
    {-8.896791392450574e-22, 7.911402614872376e-38},
    {1.6117375710961184e-24, -3.6846573564509766e-41},
    {-2.4795962632247976e-27, 1.2953730964765229e-43},
    {3.279889237069838e-30, 1.5117542744029879e-46},
};
constexpr double ATAN_C[12][2] = {
    {1.0, 0.0},
    {-0.3333333333333333, -1.850371707708594e-17},
    {0.2, -1.1102230246251566e-17},
    {-0.14285714285714285, -7.93016446160826e-18},
    {0.1111111111111111, 6.1679056923619804e-18},
    {-0.09090909090909091, 2.523234146875356e-18},
    {0.07692307692307693, -4.270088556250602e-18},
    {-0.06666666666666667, -9.251858538542971e-19},
    {0.058823529411764705, 8.163404592832033e-19},
    {-0.05263157894736842, -2.921639538487254e-18},
    {0.047619047619047616, 2.64338815386942e-18},
    {-0.043478260869565216, -1.206764157201257e-18},
};
constexpr double ATANH_C[12][2] = {
    {1.0, 0.0},
    {0.3333333333333333, 1.850371707708594e-17},
    {0.2, -1.1102230246251566e-17},
    {0.14285714285714285, 7.93016446160826e-18},
    {0.1111111111111111, 6.1679056923619804e-18},
    {0.09090909090909091, -2.523234146875356e-18},
    {0.07692307692307693, -4.270088556250602e-18},
    {0.06666666666666667, 9.251858538542971e-19},
    {0.058823529411764705, 8.163404592832033e-19},
    {0.05263157894736842, 2.921639538487254e-18},
    {0.047619047619047616, 2.64338815386942e-18},
    {0.043478260869565216, 1.206764157201257e-18},
};
constexpr double EXP_C[14][2] = {
    {1.0, 0.0},
    {1.0, 0.0},
    {0.5, 0.0},
    {0.16666666666666666, 9.25185853854297e-18},
    {0.041666666666666664, 2.3129646346357427e-18},
    {0.008333333333333333, 1.1564823173178714e-19},
    {0.001388888888888889, -5.300543954373577e-20},
    {0.0001984126984126984, 1.7209558293420705e-22},
    {2.48015873015873e-05, 2.1511947866775882e-23},
    {2.7557319223985893e-06, -1.858393274046472e-22},
    {2.755731922398589e-07, 2.3767714622250297e-23},
    {2.505210838544172e-08, -1.448814070935912e-24},
    {2.08767569878681e-09, -1.20734505911326e-25},
    {1.6059043836821613e-10, 1.2585294588752098e-26},
};
constexpr double ATAN_T[17][2] = {
    {0.0, 0.0},
    {0.06241880999595735, -1.5490756308295046e-18},
    {0.12435499454676144, -3.1253241424539383e-18},
    {0.18534794999569476, 4.180692268843079e-18},
    {0.24497866312686414, 1.0698755618734451e-17},
    {0.3028848683749714, -1.1010827903001369e-17},
    {0.35877067027057225, -2.4623815582638635e-17},
    {0.4124104415973873, -1.587652227770689e-17},
    {0.4636476090008061, 2.2698777452961687e-17},
    {0.5123894603107377, -2.5462781472855804e-17},
    {0.5585993153435624, -5.4556305485916264e-18},
    {0.6022873461349642, 2.950430737228402e-17},
    {0.6435011087932844, 1.5834785051444286e-17},
    {0.6823165548747481, 6.943223671560008e-18},
    {0.7188299996216245, -2.1478388444456983e-17},
    {0.7531512809621944, -2.4256934659182068e-17},
    {0.7853981633974483, 3.061616997868383e-17},
};
constexpr double LOG_T[25][2] = {
    {-0.2876820724517809, -2.607160616442564e-17},
    {-0.24686007793152578, -1.361743371748368e-17},
    {-0.2076393647782445, -1.2053243216686129e-17},
    {-0.16989903679539747, 4.868008764439071e-19},
    {-0.13353139262452263, 3.664457663660085e-18},
    {-0.09844007281325252, 4.439009633675136e-18},
    {-0.06453852113757118, 6.470486661692933e-18},
    {-0.0317486983145803, -3.0382263084680858e-18},
    {0.0, 0.0},
    {0.030771658666753687, 1.0431732029005968e-18},
    {0.06062462181643484, 2.6424025938726934e-18},
    {0.08961215868968714, -5.4268129336647135e-18},
    {0.11778303565638346, -1.1971685747593677e-18},
    {0.1451820098444979, 8.242418783022475e-18},
    {0.17185025692665923, -6.0224538210113705e-18},
    {0.19782574332991987, 1.2821194372980142e-17},
    {0.22314355131420976, -9.091270597324799e-18},
    {0.24783616390458127, -1.2432209578702523e-17},
    {0.27193371548364176, 7.83319637697442e-19},
    {0.2954642128938359, -2.16461086040599e-17},
    {0.3184537311185346, 2.7114779367326236e-17},
    {0.3409265869705932, 1.7467136443544747e-17},
    {0.3629054936893685, -2.1492361455310972e-17},
    {0.38441169891033206, -1.612149700764673e-17},
    {0.4054651081081644, -2.8811380259626426e-18},
};

// ---- double-double arithmetic
struct dd {
  double h, l;
};
HTP_HD inline double fma_(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(a, b, c);
#else
  return std::fma(a, b, c);
#endif
}
HTP_HD inline dd two_sum(double a, double b) {
  const double s = a + b, bp = s - a;
  return {s, (a - (s - bp)) + (b - bp)};
}
HTP_HD inline dd fast_two_sum(double a, double b) {   // |a| >= |b| or a == 0
  const double s = a + b;
  return {s, b - (s - a)};
}
HTP_HD inline dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma_(a, b, -p)};
}
HTP_HD inline dd neg(dd x) { return {-x.h, -x.l}; }
HTP_HD inline dd add(dd x, dd y) {
  dd s = two_sum(x.h, y.h);
  const dd t = two_sum(x.l, y.l);
  s.l += t.h;
  s = fast_two_sum(s.h, s.l);
  s.l += t.l;
  return fast_two_sum(s.h, s.l);
}
HTP_HD inline dd sub(dd x, dd y) { return add(x, neg(y)); }
HTP_HD inline dd add_d(dd x, double d) {
  dd s = two_sum(x.h, d);
  s.l += x.l;
  return fast_two_sum(s.h, s.l);
}
HTP_HD inline dd mul(dd x, dd y) {
  dd p = two_prod(x.h, y.h);
  p.l += x.h * y.l + x.l * y.h;
  return fast_two_sum(p.h, p.l);
}
HTP_HD inline dd mul_d(dd x, double d) {
  dd p = two_prod(x.h, d);
  p.l += x.l * d;
  return fast_two_sum(p.h, p.l);
}
HTP_HD inline dd div(dd x, dd y) {
  const double q1 = x.h / y.h;
  dd r = sub(x, mul_d(y, q1));
  const double q2 = r.h / y.h;
  r = sub(r, mul_d(y, q2));
  const double q3 = r.h / y.h;
  return add_d(fast_two_sum(q1, q2), q3);
}
HTP_HD inline dd div_d(double a, double b) { return div(dd{a, 0.0}, dd{b, 0.0}); }
HTP_HD inline dd sqrt_dd(dd x) {   // x > 0
  const double s = std::sqrt(x.h);
  const dd p = two_prod(s, s);
  const double r = (((x.h - p.h) - p.l) + x.l) / (2.0 * s);
  return fast_two_sum(s, r);
}
HTP_HD inline dd C(const double (&c)[2]) { return {c[0], c[1]}; }
HTP_HD inline double round_dd(dd x) { return x.h + x.l; }

// ---- sin / cos / tan
// x = k pi/2 + r, |r| <~ pi/4, r in double-double; q = k mod 4.  Cody-Waite with a 4-part pi/2 below 2^20
// (k pi/2 to 2^-190), Payne-Hanek above: frac(x 2/pi) from a 256-bit window of 2/pi's bits times the 53-bit
// significand of x (integer arithmetic; the bits before the window add multiples of 4, those after < 2^-200).
HTP_HD inline unsigned two_over_pi_bits32(int p) {   // bits p .. p+31 of 2/pi (bit i weighs 2^-i), 0 for i < 1
  const int o = p - 1;
  if (o + 32 <= 0) return 0u;
  if (o < 0) return TWO_OVER_PI_BITS[0] >> (-o);
  const int j = o >> 5, sh = o & 31;
  const unsigned long long w = ((unsigned long long)TWO_OVER_PI_BITS[j] << 32) |
                               (unsigned long long)(j + 1 < 44 ? TWO_OVER_PI_BITS[j + 1] : 0u);
  return (unsigned)(w >> (32 - sh));
}
HTP_HD inline dd reduce_big(double x, int& q) {
  int ex;
  const double m = std::frexp(std::fabs(x), &ex);
  const unsigned long long M = (unsigned long long)std::ldexp(m, 53);   // |x| = M 2^E
  const int E = ex - 53, s = E - 1;                                     // window bits [s, s + 256)
  const unsigned long long mlo = M & 0xffffffffull, mhi = M >> 32;
  unsigned long long acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < 8; ++k) {                     // limb k (little-endian) of the window integer T
    const unsigned long long t = two_over_pi_bits32(s + 32 * (7 - k));
    const unsigned long long plo = mlo * t, phi = mhi * t;
    acc[k] += plo & 0xffffffffull;
    acc[k + 1] += (plo >> 32) + (phi & 0xffffffffull);
    acc[k + 2] += phi >> 32;
  }
  for (int k = 0; k < 9; ++k) { acc[k + 1] += acc[k] >> 32; acc[k] &= 0xffffffffull; }
  // x 2/pi = M T 2^-254 (mod 4): integer bits 254, 255; fraction = bits 0 .. 253
  q = (int)((acc[7] >> 30) & 3ull);
  dd f{0.0, 0.0};
  for (int k = 0; k < 7; ++k) f = add_d(f, std::ldexp((double)acc[k], 32 * k - 254));
  f = add_d(f, std::ldexp((double)(acc[7] & 0x3fffffffull), 224 - 254));
  if (f.h >= 0.5) { f = add_d(f, -1.0); q = (q + 1) & 3; }
  dd r = mul(f, dd{PIO2_H, PIO2_L});
  if (x < 0) { r = neg(r); q = (4 - q) & 3; }
  return r;
}
HTP_HD inline dd reduce_pio2(double x, int& q) {
  if (std::fabs(x) >= 0x1p20) return reduce_big(x, q);
  const double k = rint(x * TWO_OVER_PI);
  const dd p1 = two_prod(k, PIO2_1);
  dd r = two_sum(x, -p1.h);   // exact: x and k pi/2 agree in their leading bits
  r = add_d(r, -p1.l);
  r = sub(r, two_prod(k, PIO2_2));
  r = sub(r, two_prod(k, PIO2_3));
  r = add_d(r, -(k * PIO2_4));
  const long long ki = (long long)k;
  q = (int)(ki & 3);
  return r;
}
// sin(r) and cos(r) for |r| <= ~0.8 (Taylor; terms below 2^-54 relative in double)
HTP_HD inline dd sin_dd(dd r) {
  const dd r2 = mul(r, r);
  double t = SIN_C[13][0];
  for (int n = 12; n >= 8; --n) t = SIN_C[n][0] + r2.h * t;
  dd p = add(C(SIN_C[7]), mul_d(r2, t));
  for (int n = 6; n >= 0; --n) p = add(C(SIN_C[n]), mul(r2, p));
  return mul(r, p);
}
HTP_HD inline dd cos_dd(dd r) {
  const dd r2 = mul(r, r);
  double t = COS_C[14][0];
  for (int n = 13; n >= 9; --n) t = COS_C[n][0] + r2.h * t;
  dd p = add(C(COS_C[8]), mul_d(r2, t));
  for (int n = 7; n >= 0; --n) p = add(C(COS_C[n]), mul(r2, p));
  return p;
}
HTP_HD inline bool nonfinite(double x) { return !(x - x == 0.0); }

HTP_HD inline double sin(double x) {
  if (nonfinite(x)) return x - x;          // NaN (inf - inf, or the NaN itself)
  if (std::fabs(x) < 0x1p-27) return x;    // |sin x - x| < 2^-55 |x|
  int q;
  const dd r = reduce_pio2(x, q);
  dd v = (q & 1) ? cos_dd(r) : sin_dd(r);
  if (q & 2) v = neg(v);
  return round_dd(v);
}
HTP_HD inline double cos(double x) {
  if (nonfinite(x)) return x - x;
  if (std::fabs(x) < 0x1p-27) return 1.0;
  int q;
  const dd r = reduce_pio2(x, q);
  dd v = (q & 1) ? sin_dd(r) : cos_dd(r);
  if (((q + 1) & 2) != 0) v = neg(v);      // q = 1, 2: negative
  return round_dd(v);
}
HTP_HD inline double tan(double x) {
  if (nonfinite(x)) return x - x;
  if (std::fabs(x) < 0x1p-27) return x;
  int q;
  const dd r = reduce_pio2(x, q);
  const dd s = sin_dd(r), c = cos_dd(r);
  return round_dd((q & 1) ? neg(div(c, s)) : div(s, c));
}

// ---- atan family
// atan(t) for 0 <= t <= 1 (t double-double): atan(i/16) + atan(u), u = (t - i/16) / (1 + t i/16), |u| <= 1/32
HTP_HD inline dd atan_unit(dd t) {
  const int i = (int)rint(t.h * 16.0);
  const double c = (double)i * 0.0625;
  const dd u = div(add_d(t, -c), add_d(mul_d(t, c), 1.0));
  const dd u2 = mul(u, u);
  double s = ATAN_C[11][0];
  for (int n = 10; n >= 6; --n) s = ATAN_C[n][0] + u2.h * s;
  dd p = add(C(ATAN_C[5]), mul_d(u2, s));
  for (int n = 4; n >= 0; --n) p = add(C(ATAN_C[n]), mul(u2, p));
  return add(C(ATAN_T[i]), mul(u, p));
}
// angle of (x, y) for y >= 0, finite, not both zero: in [0, pi]
HTP_HD inline dd angle_dd(dd y, dd x) {
  const double ax = std::fabs(x.h);
  const dd axd = x.h < 0 ? neg(x) : x;
  dd a;
  if (y.h <= ax) a = atan_unit(div(y, axd));
  else a = sub(dd{PIO2_H, PIO2_L}, atan_unit(div(axd, y)));
  if (x.h < 0) a = sub(dd{PI_H, PI_L}, a);
  return a;
}
HTP_HD inline double atan(double x) {
  if (x != x) return x;
  const double ax = std::fabs(x);
  if (ax < 0x1p-27) return x;
  if (ax > 0x1p60) return std::copysign(PIO2_H, x);
  const dd a = ax <= 1.0 ? atan_unit(dd{ax, 0.0}) : sub(dd{PIO2_H, PIO2_L}, atan_unit(div_d(1.0, ax)));
  return std::copysign(round_dd(a), x);
}
HTP_HD inline double atan2(double y, double x) {
  if (x != x || y != y) return x + y;
  const double ay = std::fabs(y);
  const bool xneg = std::signbit(x);
  if (ay == 0.0) return std::copysign(xneg ? PI_H : 0.0, y);
  if (x == 0.0) return std::copysign(PIO2_H, y);
  const bool yinf = nonfinite(y), xinf = nonfinite(x);
  if (yinf && xinf) return std::copysign(xneg ? PI34_H : PIO4_H, y);
  if (yinf) return std::copysign(PIO2_H, y);
  if (xinf) return std::copysign(xneg ? PI_H : 0.0, y);
  const double ax = std::fabs(x);
  if (ay > ax * 0x1p60) return std::copysign(PIO2_H, y);   // |atan2 - pi/2| < 2^-60
  if (ax > ay * 0x1p60 && !xneg) {                         // atan2 ~ y/x
    const double q = ay / ax;
    return std::copysign(q, y);
  }
  return std::copysign(round_dd(angle_dd(dd{ay, 0.0}, dd{x, 0.0})), y);
}
// sqrt(1 - x^2) for |x| < 1, double-double
HTP_HD inline dd cosofsin(double x) { return sqrt_dd(mul(two_sum(1.0, -x), two_sum(1.0, x))); }
HTP_HD inline double asin(double x) {
  if (x != x) return x;
  const double ax = std::fabs(x);
  if (ax > 1.0) return (x - x) / (x - x);
  if (ax == 1.0) return std::copysign(PIO2_H, x);
  if (ax < 0x1p-27) return x;
  return std::copysign(round_dd(angle_dd(dd{ax, 0.0}, cosofsin(ax))), x);
}
HTP_HD inline double acos(double x) {
  if (x != x) return x;
  const double ax = std::fabs(x);
  if (ax > 1.0) return (x - x) / (x - x);
  if (x == 1.0) return 0.0;
  if (x == -1.0) return PI_H;
  if (ax < 0x1p-57) return PIO2_H;
  return round_dd(angle_dd(cosofsin(x), dd{x, 0.0}));
}

// ---- hypot
HTP_HD inline double hypot(double x, double y) {
  double a = std::fabs(x), b = std::fabs(y);
  if (a == __builtin_huge_val() || b == __builtin_huge_val()) return __builtin_huge_val();
  if (a != a || b != b) return a + b;
  if (a < b) { const double t = a; a = b; b = t; }
  if (b == 0.0) return a;
  if (b < a * 0x1p-60) return a;           // sqrt(a^2 + b^2) = a (1 + 2^-121)
  int e;
  std::frexp(a, &e);
  a = std::ldexp(a, -e);                   // a in [0.5, 1), b >= 2^-61: exact scaling, no underflow
  b = std::ldexp(b, -e);
  const dd s = add(two_prod(a, a), two_prod(b, b));
  return std::ldexp(round_dd(sqrt_dd(s)), e);
}

// ---- pow (exp / log in double-double)
HTP_HD inline dd log_dd(double x) {        // x > 0, finite
  int e;
  double m = std::frexp(x, &e);
  if (m < 0.75) { m *= 2.0; --e; }         // m in [0.75, 1.5)
  const int i = (int)rint((m - 1.0) * 32.0);
  const double c = 1.0 + (double)i * 0.03125;
  const dd u = div(dd{m - c, 0.0}, two_sum(m, c));   // m - c exact (Sterbenz)
  const dd u2 = mul(u, u);
  double s = ATANH_C[8][0];
  for (int n = 7; n >= 4; --n) s = ATANH_C[n][0] + u2.h * s;
  dd p = add(C(ATANH_C[3]), mul_d(u2, s));
  for (int n = 2; n >= 0; --n) p = add(C(ATANH_C[n]), mul(u2, p));
  dd r = add(C(LOG_T[i + 8]), mul_d(mul(u, p), 2.0));
  const double ed = (double)e;
  r = add(r, two_prod(ed, LN2_1));
  r = add(r, two_prod(ed, LN2_2));
  return add_d(r, ed * LN2_3);
}
HTP_HD inline double exp_dd(dd a) {        // rounded exp(a); normal results correctly rounded
  if (a.h > 709.79) return __builtin_huge_val();
  if (a.h < -745.2) return 0.0;
  const double k = rint(a.h * INV_LN2);
  dd r = add(a, neg(two_prod(k, LN2_1)));
  r = sub(r, two_prod(k, LN2_2));
  r = add_d(r, -(k * LN2_3));
  r = dd{r.h * 0.03125, r.l * 0.03125};    // r / 32, exact
  double t = EXP_C[11][0];
  for (int n = 10; n >= 8; --n) t = EXP_C[n][0] + r.h * t;
  dd p = add(C(EXP_C[7]), mul_d(r, t));
  for (int n = 6; n >= 1; --n) p = add(C(EXP_C[n]), mul(r, p));
  dd E = mul(r, p);                        // expm1(r / 32)
  for (int j = 0; j < 5; ++j) E = add(mul_d(E, 2.0), mul(E, E));   // expm1(2 z) = 2 E + E^2
  return std::ldexp(round_dd(add_d(E, 1.0)), (int)k);
}
HTP_HD inline double log(double x) {
  if (x != x) return x;
  if (x < 0.0) return (x - x) / (x - x);
  if (x == 0.0) return -__builtin_huge_val();
  if (x == __builtin_huge_val()) return x;
  if (x == 1.0) return 0.0;
  return round_dd(log_dd(x));
}
// sin and cos of one argument, one reduction: the same doubles as sin(x), cos(x)
HTP_HD inline void sincos(double x, double& s, double& c) {
  if (nonfinite(x)) { s = c = x - x; return; }
  if (std::fabs(x) < 0x1p-27) { s = x; c = 1.0; return; }
  int q;
  const dd r = reduce_pio2(x, q);
  const dd sr = sin_dd(r), cr = cos_dd(r);
  dd vs = (q & 1) ? cr : sr, vc = (q & 1) ? sr : cr;
  if (q & 2) vs = neg(vs);
  if (((q + 1) & 2) != 0) vc = neg(vc);
  s = round_dd(vs);
  c = round_dd(vc);
}
HTP_HD inline bool is_int(double y) { return rint(y) == y; }
HTP_HD inline bool is_odd_int(double y) { return is_int(y) && std::fabs(y) < 0x1p53 && std::fmod(y, 2.0) != 0.0; }
HTP_HD inline double pow(double x, double y) {
  if (y == 2.0) return x * x;              // correctly rounded by IEEE multiplication
  if (y == 0.0 || x == 1.0) return 1.0;
  if (x != x || y != y) return x + y;
  if (y == 1.0) return x;
  const double inf = __builtin_huge_val();
  if (x == 0.0) {
    if (y > 0) return is_odd_int(y) ? x : 0.0;
    return is_odd_int(y) ? std::copysign(inf, x) : inf;
  }
  if (nonfinite(y)) {
    const double ax = std::fabs(x);
    if (ax == 1.0) return 1.0;
    return (ax > 1.0) == (y > 0) ? inf : 0.0;
  }
  if (nonfinite(x)) {
    if (x > 0) return y > 0 ? inf : 0.0;
    const double s = is_odd_int(y) ? -1.0 : 1.0;
    return y > 0 ? s * inf : s * 0.0;
  }
  double sign = 1.0;
  if (x < 0) {
    if (!is_int(y)) return (x - x) / (x - x);
    if (is_odd_int(y)) sign = -1.0;
    x = -x;
  }
  if (y == 1.5) {                          // x sqrt(x) (the curvature denominators), scaled by 2^(3e/2)
    int e;
    double f = std::frexp(x, &e);
    if (e & 1) { f *= 2.0; --e; }          // x = f 2^e, e even, f in [0.5, 2)
    const dd s = sqrt_dd(dd{f, 0.0});
    return sign * std::ldexp(round_dd(mul_d(s, f)), (e / 2) * 3);
  }
  if (y == 0.5) return sign * std::sqrt(x);
  return sign * exp_dd(mul_d(log_dd(x), y));
}

#endif  // HTP_LIBM_PLATFORM

}  // namespace hm
}  // namespace htp

#if !defined(__clang__) && defined(__GNUC__)
#pragma GCC pop_options
#endif
