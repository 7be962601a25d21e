// glibc's double exp and pow, restated for the GPU operation by operation.
//
// Why: the reference computes its atmosphere, Fresnel, regularisation and
// sRGB terms with the C library's double exp / pow (path_tracer.hh:483-484,
// 531, 553-560, 91-98, 735-737, 760-764; float arguments promoted to double)
// and keeps using those doubles in double arithmetic before rounding to float.
// ocml's f64 routines are faithful but not glibc's: over all 2^32 float
// arguments they return a different double for 0.33% (exp) to 25% (pow) of
// them (tools/exhaustive_f64.hip, profiles/r03_exhaustive/ocml_vs_glibc.txt),
// and a 1-ulp double difference can change the float a sum or product rounds
// to.  So the hot path calls these restatements instead, and
// tools/exhaustive_f64.hip proves them equal to glibc bit for bit on every
// float argument.
//
// What is restated: glibc 2.35 (Ubuntu 2.35-0ubuntu3.11, the libm the
// reference and the oracle link here and on the GPU boxes), whose exp and pow
// are the table-driven algorithms of sysdeps/ieee754/dbl-64/e_exp.c and
// e_pow.c (N = 128 exp table, 128-entry log table for pow, degree-5 / 7
// polynomials).  On x86-64 hosts with FMA (both hosts here) glibc runs the
// FMA builds of those files, and GCC fused every a * b + c it could; the
// fused-multiply-adds below are exactly the ones in that machine code
// (vfmadd / vfmsub in __exp_fma and __pow_fma), everything else is a plain
// IEEE operation in the same order.  The data (coefficients, tables) comes
// from the same libm, tools/glibc_tables.py -> glibc_tables.h.
//
// Scope: exp on every double; pow on every x for the path's constant
// exponents (a finite y with 2^-65 <= |y| < 2^63: 5, 0.25, 1.5, 1/2.4) -
// glibc's y-special branch (y zero, inf, nan, tiny or huge) is not restated.
//
// Attribution and licence.  The algorithms and constant tables restated here
// are those of the GNU C Library 2.35 (sysdeps/ieee754/dbl-64: e_exp.c,
// e_pow.c, s_sin.c and their data files), which is licensed under the GNU
// Lesser General Public License v2.1 or later.  glibc's exp and pow (and
// their data) derive from Arm's optimized-routines (Szabolcs Nagy, Arm Ltd.,
// MIT / Apache-2.0 WITH LLVM-exception upstream); sin / cos (s_sin.c,
// __sincostab) are IBM Accurate Mathematical Library code contributed to
// glibc.  This file restates those routines for the GPU so that its results
// equal the host libm's bit for bit; the restated parts remain under their
// original terms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "glibc_tables.h"

namespace ptg {
namespace glibc {

#define GL_D __device__ __forceinline__

GL_D double asd(uint64_t u) { return __longlong_as_double((long long)u); }
GL_D uint64_t asu(double d) { return (uint64_t)__double_as_longlong(d); }
GL_D double fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// Where exp reads its 128-entry table (tail, scale bits: one 16-byte entry):
// from global memory, or from an LDS copy a kernel made with
// exp_table_to_lds() (the sky and shade kernels: an LDS read instead of a
// vector-memory gather that queues behind the BVH walks' loads).
typedef uint64_t u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u2v lds_u2v_t;
struct ExpTabGlobal {
    GL_D u2v entry(uint32_t i) const { return reinterpret_cast<const u2v*>(kExpTab)[i]; }
};
struct ExpTabLds {
    const lds_u2v_t* t;
    GL_D u2v entry(uint32_t i) const { return t[i]; }
};
constexpr uint32_t kExpTabEntries = 128;
// the block's threads copy the table to `dst` (kExpTabEntries entries); the
// caller synchronises the block before using it
GL_D void exp_table_to_lds(lds_u2v_t* dst)
{
    for(uint32_t i = threadIdx.x; i < kExpTabEntries; i += blockDim.x) dst[i] = ExpTabGlobal{}.entry(i);
}

// __exp_data scalars (kExpData) and exp_inline's constants
constexpr double kInvLn2N = __builtin_bit_cast(double, kExpData[0]);
constexpr double kShift = __builtin_bit_cast(double, kExpData[1]);
constexpr double kNegLn2hiN = __builtin_bit_cast(double, kExpData[2]);
constexpr double kNegLn2loN = __builtin_bit_cast(double, kExpData[3]);
constexpr double kC2 = __builtin_bit_cast(double, kExpData[4]);
constexpr double kC3 = __builtin_bit_cast(double, kExpData[5]);
constexpr double kC4 = __builtin_bit_cast(double, kExpData[6]);
constexpr double kC5 = __builtin_bit_cast(double, kExpData[7]);
constexpr double kTwoP1009 = __builtin_bit_cast(double, 0x7f00000000000000ull);   // 0x1p1009
constexpr double kTwoM1022 = __builtin_bit_cast(double, 0x0010000000000000ull);   // 0x1p-1022
constexpr double kTwoM767 = __builtin_bit_cast(double, 0x1000000000000000ull);    // 0x1p-767 (__math_uflow)
constexpr double kTwoP769 = __builtin_bit_cast(double, 0x7000000000000000ull);    // 0x1p769  (__math_oflow)
constexpr double kTwoP52 = __builtin_bit_cast(double, 0x4330000000000000ull);
// __pow_log_data scalars (kPowLogData): ln2hi, ln2lo, poly A[0..6]
constexpr double kLn2hi = __builtin_bit_cast(double, kPowLogData[0]);
constexpr double kLn2lo = __builtin_bit_cast(double, kPowLogData[1]);
constexpr double kA0 = __builtin_bit_cast(double, kPowLogData[2]);
constexpr double kA1 = __builtin_bit_cast(double, kPowLogData[3]);
constexpr double kA2 = __builtin_bit_cast(double, kPowLogData[4]);
constexpr double kA3 = __builtin_bit_cast(double, kPowLogData[5]);
constexpr double kA4 = __builtin_bit_cast(double, kPowLogData[6]);
constexpr double kA5 = __builtin_bit_cast(double, kPowLogData[7]);
constexpr double kA6 = __builtin_bit_cast(double, kPowLogData[8]);
constexpr uint64_t kPowOff = 0x3fe6955500000000ull;
constexpr uint32_t kSignBias = 0x800u << 7;          // 0x800 << EXP_TABLE_BITS

// __math_uflow / __math_oflow (math_err.c: xflow(sign, y) = (sign ? -y : y) * y)
GL_D double uflow(uint32_t sign) { return (sign ? -kTwoM767 : kTwoM767) * kTwoM767; }
GL_D double oflow(uint32_t sign) { return (sign ? -kTwoP769 : kTwoP769) * kTwoP769; }

// specialcase of exp / exp_inline (|x| in [512, 1024)): scale's exponent
// out of range, handled around 2^+-1009 / 2^-1022; k < 0 results that fall
// into the subnormal range are rounded once (hi + lo) before scaling.
// `signed_one`: pow's version (the result may be negative: one = -1 when
// y < 0 and |y| is compared); exp's compares y < 1.0 directly.
template<bool POW>
GL_D double specialcase(double tmp, uint64_t sbits, uint64_t ki)
{
    if((ki & 0x80000000u) == 0)
    {   // k > 0: the exponent of scale may have overflowed by <= 460
        sbits -= 1009ull << 52;
        const double scale = asd(sbits);
        return kTwoP1009 * fma(scale, tmp, scale);
    }
    // k < 0: subnormal range needs care (scale * tmp is used twice: no fma)
    sbits += 1022ull << 52;
    const double scale = asd(sbits);
    const double st = scale * tmp;
    double y = scale + st;
    if(POW ? (1.0 > fabs(y)) : (1.0 > y))
    {
        const double one = (POW && y < 0.0) ? -1.0 : 1.0;
        const double lo = (scale - y) + st;
        const double hi = y + one;
        double r = ((one - hi) + y) + lo;
        r = (r + hi) - one;
        if(r == 0) r = asd(sbits & 0x8000000000000000ull);
        y = r;
    }
    return kTwoM1022 * y;
}

// The body of exp after the range check: abstop == 0 marks |x| in [512, 1024).
template<class T>
GL_D double exp_core(double x, uint32_t abstop, const T& tab)
{
    double kd = fma(x, kInvLn2N, kShift);
    const uint64_t ki = asu(kd);
    kd = kd - kShift;
    double r = fma(kd, kNegLn2hiN, x);
    r = fma(kd, kNegLn2loN, r);
    const u2v e = tab.entry(uint32_t(ki & 0x7fu));
    const double tail = asd(e.x);
    const uint64_t sbits = e.y + (ki << 45);
    const double p1 = fma(r, kC3, kC2);
    const double rt = r + tail;
    const double r2 = r * r;
    const double p2 = fma(r, kC5, kC4);
    const double t = fma(p1, r2, rt);
    const double tmp = fma(r2 * r2, p2, t);
    if(abstop == 0) return specialcase<false>(tmp, sbits, ki);
    const double scale = asd(sbits);
    return fma(scale, tmp, scale);
}

// exp outside |x| in [2^-54, 512): tiny, large, huge, inf, nan (rare on the
// path: out of line, so the inlined exp stays small)
template<class T>
inline __device__ __attribute__((noinline)) double exp_special(double x, T tab)
{
    const uint64_t ix = asu(x);
    const uint32_t abstop = uint32_t(ix >> 52) & 0x7ffu;
    if(int32_t(abstop - 0x3c9u) < 0) return x + 1.0;                      // |x| < 2^-54 (and 0)
    if(abstop > 0x408u)
    {   // |x| >= 1024
        if(ix == 0xfff0000000000000ull) return 0.0;                        // -inf
        if(abstop == 0x7ffu) return x + 1.0;                                // +inf, nan
        return (ix >> 63) ? uflow(0) : oflow(0);
    }
    return exp_core(x, 0, tab);                                              // [512, 1024): special case
}

// exp (e_exp.c as in __exp_fma)
template<class T = ExpTabGlobal>
GL_D double exp(double x, const T& tab = T())
{
    const uint32_t abstop = uint32_t(asu(x) >> 52) & 0x7ffu;
    if(abstop - 0x3c9u > 0x3eu) return exp_special(x, tab);
    return exp_core(x, abstop, tab);
}

// checkint (e_pow.c): 0 not an integer, 1 odd integer, 2 even integer
GL_D int checkint(uint64_t iy)
{
    const int e = int(iy >> 52 & 0x7ff);
    if(e < 0x3ff) return 0;
    if(e > 0x3ff + 52) return 2;
    if(iy & ((1ull << (0x3ff + 52 - e)) - 1)) return 0;
    if(iy & (1ull << (0x3ff + 52 - e))) return 1;
    return 2;
}

// log_inline (e_pow.c as in __pow_fma): log(x) as hi + *tail
GL_D double log_inline(uint64_t ix, double& tail)
{
    const uint64_t tmp = ix - kPowOff;
    const uint32_t i = uint32_t(tmp >> 45) & 0x7fu;
    const int32_t k = int32_t(int64_t(tmp) >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double z = asd(iz);
    const double kd = (double)k;
    typedef uint64_t u2 __attribute__((ext_vector_type(2)));
    const u2* e = reinterpret_cast<const u2*>(kPowLogTab) + 2 * i;   // {invc, pad}, {logc, logctail}
    const double invc = asd(e[0].x);
    const u2 lc = e[1];
    const double logc = asd(lc.x), logctail = asd(lc.y);
    const double t1 = fma(kd, kLn2hi, logc);
    const double r = fma(z, invc, -1.0);
    const double ar = r * kA0;
    const double lo1 = fma(kd, kLn2lo, logctail);
    const double q12 = fma(r, kA2, kA1);
    const double q34 = fma(r, kA4, kA3);
    const double t2 = r + t1;
    const double ar2 = r * ar;
    const double lo2 = (t1 - t2) + r;
    const double ar3 = r * ar2;
    const double lo3 = fma(ar, r, -ar2);
    const double q56 = fma(r, kA6, kA5);
    const double hi = t2 + ar2;
    const double lo4 = (t2 - hi) + ar2;
    const double q = fma(ar2, fma(q56, ar2, q34), q12);
    const double lo = fma(ar3, q, ((lo1 + lo2) + lo3) + lo4);
    const double y = hi + lo;
    tail = (hi - y) + lo;
    return y;
}

// exp_inline's body after the range check (abstop == 0: |x| in [512, 1024))
GL_D double exp_inline_core(double x, double xtail, uint32_t sign_bias, uint32_t abstop)
{
    double kd = fma(x, kInvLn2N, kShift);
    const uint64_t ki = asu(kd);
    kd = kd - kShift;
    double r = fma(kd, kNegLn2hiN, x);
    r = fma(kd, kNegLn2loN, r);
    r = xtail + r;
    const u2v e = ExpTabGlobal{}.entry(uint32_t(ki & 0x7fu));
    const double tail = asd(e.x);
    const uint64_t sbits = e.y + ((ki + sign_bias) << 45);
    const double p1 = fma(r, kC3, kC2);
    const double rt = r + tail;
    const double r2 = r * r;
    const double p2 = fma(r, kC5, kC4);
    const double t = fma(p1, r2, rt);
    const double tmp = fma(p2, r2 * r2, t);
    if(abstop == 0) return specialcase<true>(tmp, sbits, ki);
    const double scale = asd(sbits);
    return fma(tmp, scale, scale);
}

inline __device__ __attribute__((noinline)) double exp_inline_special(double x, double xtail, uint32_t sign_bias)
{
    const uint32_t abstop = uint32_t(asu(x) >> 52) & 0x7ffu;
    if(int32_t(abstop - 0x3c9u) < 0)
    {   // tiny
        const double one = x + 1.0;
        return sign_bias ? -one : one;
    }
    if(abstop > 0x408u) return (asu(x) >> 63) ? uflow(sign_bias) : oflow(sign_bias);
    return exp_inline_core(x, xtail, sign_bias, 0);
}

// exp_inline (e_pow.c as in __pow_fma): exp(x + xtail), sign from sign_bias
GL_D double exp_inline(double x, double xtail, uint32_t sign_bias)
{
    const uint32_t abstop = uint32_t(asu(x) >> 52) & 0x7ffu;
    if(abstop - 0x3c9u > 0x3eu) return exp_inline_special(x, xtail, sign_bias);
    return exp_inline_core(x, xtail, sign_bias, abstop);
}

// pow for x <= 0, subnormal x, inf or nan (out of line)
inline __device__ __attribute__((noinline)) double pow_special(double x, double y)
{
    uint64_t ix = asu(x);
    const uint64_t iy = asu(y);
    uint32_t topx = uint32_t(ix >> 52);
    uint32_t sign_bias = 0;
    {   // x <= 0, subnormal, inf or nan
        if(2 * ix - 1 >= 2 * 0x7ff0000000000000ull - 1)
        {   // x zero, inf or nan
            double x2 = x * x;
            if((ix >> 63) && checkint(iy) == 1) x2 = -x2;
            return (iy >> 63) ? 1.0 / x2 : x2;
        }
        if(ix >> 63)
        {   // finite x < 0
            const int yint = checkint(iy);
            if(yint == 0) return (x - x) / (x - x);                        // __math_invalid
            if(yint == 1) sign_bias = kSignBias;
            ix &= 0x7fffffffffffffffull;
            topx &= 0x7ffu;
        }
        if(topx == 0)
        {   // subnormal x: normalise so the exponent becomes negative
            ix = asu(x * kTwoP52) & 0x7fffffffffffffffull;
            ix -= 52ull << 52;
        }
    }
    double lo;
    const double hi = log_inline(ix, lo);
    const double ehi = y * hi;
    const double elo = fma(y, lo, fma(hi, y, -ehi));
    return exp_inline(ehi, elo, sign_bias);
}


// pow (e_pow.c as in __pow_fma) for a finite y with 2^-65 <= |y| < 2^63
GL_D double pow(double x, double y)
{
    uint64_t ix = asu(x);
    const uint32_t topx = uint32_t(ix >> 52);
    if(topx - 1u >= 0x7feu) return pow_special(x, y);                     // x <= 0, subnormal, inf or nan
    double lo;
    const double hi = log_inline(ix, lo);
    const double ehi = y * hi;
    const double elo = fma(y, lo, fma(hi, y, -ehi));
    return exp_inline(ehi, elo, 0);
}

// ---- sin / cos (s_sin.c as in __sin_fma / __cos_fma: IBM Accurate
// Mathematical Library, 440-entry __sincostab), for |x| < 105414350 - the
// range glibc reduces with its 4-part pi/2 (reduce_sincos); larger
// arguments (glibc's __branred) are not restated and never reach this path.
// The hot path needs these only where it keeps the double result
// (sample_ggx_vndf, path_tracer.hh:67-83: phi in [0, 2 pi]); everywhere
// else the float rounding of ocml's sin / cos is already glibc's.
constexpr double kBig = __builtin_bit_cast(double, 0x42c8000000000000ull);
constexpr double kSn3 = __builtin_bit_cast(double, 0xbfc5555555555515ull);
constexpr double kSn5 = __builtin_bit_cast(double, 0x3f811110e829872full);
constexpr double kCs2 = __builtin_bit_cast(double, 0x3fe0000000000000ull);
constexpr double kCs4 = __builtin_bit_cast(double, 0xbfa5555555555535ull);
constexpr double kCs6 = __builtin_bit_cast(double, 0x3f56c16bedd9e239ull);
constexpr double kS1 = __builtin_bit_cast(double, 0xbfc5555555555555ull);
constexpr double kS2 = __builtin_bit_cast(double, 0x3f81111111110eceull);
constexpr double kS3 = __builtin_bit_cast(double, 0xbf2a01a019db08b8ull);
constexpr double kS4 = __builtin_bit_cast(double, 0x3ec71de27b9a7ed9ull);
constexpr double kS5 = __builtin_bit_cast(double, 0xbe5addffc2fcdf59ull);
constexpr double kHp0 = __builtin_bit_cast(double, 0x3ff921fb54442d18ull);
constexpr double kHp1 = __builtin_bit_cast(double, 0x3c91a62633145c07ull);
constexpr double kToInt = __builtin_bit_cast(double, 0x4338000000000000ull);
constexpr double kHpInv = __builtin_bit_cast(double, 0x3fe45f306dc9c883ull);
constexpr double kMp1 = __builtin_bit_cast(double, 0x3ff921fb58000000ull);
constexpr double kMp2 = __builtin_bit_cast(double, 0xbe4dde973c000000ull);
constexpr double kPp3 = __builtin_bit_cast(double, 0xbc8cb3b398000000ull);
constexpr double kPp4 = __builtin_bit_cast(double, 0xbacd747f23e32ed7ull);
constexpr double kTaylorMax = __builtin_bit_cast(double, 0x3fc020c49ba5e354ull);   // 0.126

GL_D double copysign_(double m, double s) { return asd((asu(m) & 0x7fffffffffffffffull) | (asu(s) & 0x8000000000000000ull)); }

// __sincostab entry of x (|x| < 0.855469): sn, ssn, cs, ccs and the reduced x
GL_D void sincos_entry(double ax, double& xr, double& sn, double& ssn, double& cs, double& ccs)
{
    const double u = ax + kBig;
    xr = ax - (u - kBig);
    const uint32_t k = uint32_t(asu(u)) << 2;
    typedef uint64_t u2 __attribute__((ext_vector_type(2)));
    const u2 a = reinterpret_cast<const u2*>(kSinCosTab)[k >> 1], b = reinterpret_cast<const u2*>(kSinCosTab)[(k >> 1) + 1];
    sn = asd(a.x);
    ssn = asd(a.y);
    cs = asd(b.x);
    ccs = asd(b.y);
}

// TAYLOR_SIN(xx, a, da)
GL_D double taylor_sin(double a, double da)
{
    const double xx = a * a;
    double p = fma(xx, kS5, kS4);
    p = fma(xx, p, kS3);
    p = fma(xx, p, kS2);
    p = fma(xx, p, kS1);
    const double t1 = fma(p, a, -(0.5 * da));
    return fma(xx, t1, da) + a;
}

// do_sin(x, dx)
GL_D double do_sin(double x, double dx)
{
    const double ax = fabs(x);
    if(kTaylorMax > ax) return taylor_sin(x, dx);
    if(!(0.0 < x)) dx = -dx;
    double xr, sn, ssn, cs, ccs;
    sincos_entry(ax, xr, sn, ssn, cs, ccs);
    const double xx = xr * xr;
    const double s = xr + fma(xr * xx, fma(xx, kSn5, kSn3), dx);
    const double c = fma(xr, dx, xx * fma(xx, fma(xx, kCs6, kCs4), kCs2));
    const double cor = fma(s, cs, fma(-c, sn, fma(s, ccs, ssn)));
    return copysign_(sn + cor, x);
}

// do_cos(x, dx)
GL_D double do_cos(double x, double dx)
{
    if(x < 0) dx = -dx;
    double xr, sn, ssn, cs, ccs;
    sincos_entry(fabs(x), xr, sn, ssn, cs, ccs);
    xr = xr + dx;
    const double xx = xr * xr;
    const double s = fma(xr * xx, fma(xx, kSn5, kSn3), xr);
    const double c = xx * fma(xx, fma(xx, kCs6, kCs4), kCs2);
    const double cor = fma(-s, sn, fma(-c, cs, fma(-s, ssn, ccs)));
    return cs + cor;
}

// reduce_sincos: x - n pi/2 as a + da, n mod 4
GL_D uint32_t reduce_sincos(double x, double& a, double& da)
{
    const double t = fma(x, kHpInv, kToInt);
    const double xn = t - kToInt;
    const uint32_t n = uint32_t(asu(t)) & 3u;
    double y = fma(-xn, kMp1, x);
    y = fma(-xn, kMp2, y);
    const double t2 = fma(-xn, kPp3, y);
    double db = fma(-kPp3, xn, y - t2);
    const double b = fma(-xn, kPp4, t2);
    db = db + fma(-xn, kPp4, t2 - b);
    a = b;
    da = db;
    return n;
}

GL_D double do_sincos(double a, double da, uint32_t n)
{
    const double r = (n & 1u) ? do_cos(a, da) : do_sin(a, da);
    return (n & 2u) ? -r : r;
}

// sin / cos for |x| < 105414350 (beyond: ocml's, not glibc's)
GL_D double sin(double x)
{
    const uint32_t k = uint32_t(asu(x) >> 32) & 0x7fffffffu;
    if(k < 0x3e500000u) return x;                                           // |x| < 2^-26
    if(k < 0x3feb6000u) return do_sin(x, 0.0);                              // |x| < 0.855469
    if(k < 0x400368fdu) return copysign_(do_cos(kHp0 - fabs(x), kHp1), x);   // |x| < 2.426265
    if(k < 0x419921fbu)
    {
        double a, da;
        const uint32_t n = reduce_sincos(x, a, da);
        return do_sincos(a, da, n);
    }
    return ::sin(x);
}

GL_D double cos(double x)
{
    const uint32_t k = uint32_t(asu(x) >> 32) & 0x7fffffffu;
    if(k < 0x3e400000u) return 1.0;                                         // |x| < 2^-27
    if(k < 0x3feb6000u) return do_cos(x, 0.0);                              // |x| < 0.855469
    if(k < 0x400368fdu)
    {   // |x| < 2.426265
        const double y = kHp0 - fabs(x);
        const double a = y + kHp1;
        const double da = (y - a) + kHp1;
        return do_sin(a, da);
    }
    if(k < 0x419921fbu)
    {
        double a, da;
        const uint32_t n = reduce_sincos(x, a, da);
        return do_sincos(a, da, n + 1u);
    }
    return ::cos(x);
}

} // namespace glibc
} // namespace ptg
