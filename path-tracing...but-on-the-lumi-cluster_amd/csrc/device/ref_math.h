// Device arithmetic with the reference's exact semantics (gfx950).
//
// The hot path must reproduce the reference's float results bit for bit, so
// this header pins down every operation whose result could otherwise differ
// from the reference's C++ on the CPU:
//   * kernels are compiled with -ffp-contract=off (no silent FMA) and
//     without fast-math; f32 division and sqrt are correctly rounded (HIP's
//     default -fhip-fp32-correctly-rounded-divide-sqrt), denormals kept;
//   * the reference's unqualified exp/log/pow/sin/cos/fma on a float run in
//     DOUBLE (math.hh imports only fmin/fmax as float overloads), so do ours:
//     ocml's f64 routines, result rounded to float exactly where the
//     reference assigns to a float;
//   * fminf/fmaxf keep glibc's tie rule (equal operands -> the second one),
//     which decides the sign of a zero; NaN operands are dropped as in C.
// Only the slab test (whose min/max feed comparisons alone) uses the raw
// v_min/v_max instructions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "glibc_math.h"

namespace ptg {
namespace dm {

#define PTG_D __device__ __forceinline__

struct f2 { float x, y; };
struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };
struct m3 { f3 r[3]; };
struct u4 { uint32_t x, y, z, w; };

constexpr double PI_D = 3.14159265358979323846;
constexpr float PI_F = (float)PI_D;

PTG_D f3 V3(float x, float y, float z) { return f3{x, y, z}; }
PTG_D f3 operator+(f3 a, f3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
PTG_D f3 operator-(f3 a, f3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
PTG_D f3 operator*(f3 a, f3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
PTG_D f3 operator*(f3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
PTG_D f3 operator*(float s, f3 a) { return V3(s * a.x, s * a.y, s * a.z); }
PTG_D f3 operator/(f3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
PTG_D f3 operator-(f3 a) { return V3(-a.x, -a.y, -a.z); }
PTG_D float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PTG_D f3 cross(f3 a, f3 b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

// 1.0f / x, correctly rounded, without the full IEEE division sequence
// (v_div_scale / v_div_fmas / v_div_fixup and the denormal-mode switches):
// the hardware reciprocal (about 1 ulp) plus one Newton step with FMA gives the
// correctly rounded reciprocal for every x whose reciprocal is a normal
// number; the rest (zeros, denormals, |x| >= 2^126, inf, NaN) take the
// division.  tools/exhaustive.hip checks all 2^32 inputs against 1.0f / x
// on the GPU, bit for bit.
// rcp_nr(x, ok): the fast path alone; ok is cleared when x is outside its
// range, and the caller then takes the division (one branch for several).
PTG_D float rcp_nr(float x, bool& ok)
{
    ok = ok && ((__float_as_uint(x) >> 23) & 0xFFu) - 1u < 252u;
    const float r = __builtin_amdgcn_rcpf(x);
    const float err = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(err, r, r);
}
PTG_D float rcp_rn(float x)
{
    bool ok = true;
    float r = rcp_nr(x, ok);
    // the IEEE division only in a wave with a lane outside the fast path's
    // range (zeros, denormals, huge values: rare); written as a plain select
    // the compiler computed the division on every lane
    if(!__all(ok)) r = ok ? r : 1.0f / x;
    return r;
}

// x / c for a divisor c known at compile time, with rc = RN(1/c): the
// product q1 = RN(x * rc) is within an ulp of the quotient, its residual
// x - q1 * c is exact by FMA, and one correction step gives the correctly
// rounded quotient (Markstein) as long as nothing underflows.  So zeros,
// denormals and other tiny x (|x| < 2^-100), and NaN, take the IEEE division;
// a zero residual means q1 is exact, and a non-finite one means x is inf,
// where q1 is already the answer.  tools/exhaustive.hip checks every one
// of the 2^32 inputs against x / c on the GPU for each divisor used.
PTG_D float div_by(float x, float c, float rc)
{
    if(!(fabsf(x) >= 0x1p-100f)) return x / c;
    const float q1 = x * rc;
    const float r = __builtin_fmaf(-q1, c, x);
    const float q = __builtin_fmaf(r, rc, q1);
    return __builtin_amdgcn_classf(r, 0x198) ? q : q1;   // finite, non-zero residual
}

// sqrt(x), correctly rounded, without the compiler's sequence (v_sqrt_f32,
// then both ulp neighbours tested by FMA residuals, plus denormal scaling):
// the hardware 1/sqrt (about 1 ulp), a coupled Newton step on g ~ sqrt(x) and
// h ~ 1/(2 sqrt(x)), and a final residual correction with FMA.  x outside
// [2^-100, 2^100] (zeros, denormals, huge values, inf, NaN, negatives) takes
// the IEEE sqrt in a branch.  tools/exhaustive.hip checks all 2^32 inputs
// against sqrtf on the GPU, bit for bit.
PTG_D float sqrt_rn(float x)
{
    if(!(x >= 0x1p-100f && x <= 0x1p100f)) return __builtin_sqrtf(x);
    const float y = __builtin_amdgcn_rsqf(x);
    float g = x * y, h = 0.5f * y;
    const float r = __builtin_fmaf(-g, h, 0.5f);
    g = __builtin_fmaf(g, r, g);
    h = __builtin_fmaf(h, r, h);
    const float d = __builtin_fmaf(-g, g, x);
    return __builtin_fmaf(d, h, g);
}

// f32 sqrt: correctly rounded == the reference's (float)sqrt((double)x)
// (sqrt_rn here measured slower in the sky kernel: frame 0 +1%)
PTG_D float fsqrt(float x) { return __builtin_sqrtf(x); }
PTG_D float length(f3 a) { return fsqrt(dot(a, a)); }
PTG_D f3 normalize(f3 a) { return a / length(a); }

// glibc fminf/fmaxf (x86_64 minss/maxss + NaN fix-up): ties return y.
PTG_D float gmin(float x, float y) { return (x < y || y != y) ? x : y; }
PTG_D float gmax(float x, float y) { return (x > y || y != y) ? x : y; }
PTG_D double gmax_d(double x, double y) { return (x > y || y != y) ? x : y; }
PTG_D float clampf(float v, float lo, float hi) { return gmin(gmax(v, lo), hi); }
PTG_D float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
PTG_D float signf(float v)
{
    if(v < 0) return -1.0f;
    if(v > 0) return 1.0f;
    return v == -0.0f ? -0.0f : +0.0f;
}

// double-precision library calls, as the reference makes them.  exp, pow,
// sin and cos are glibc's own algorithms (glibc_math.h) wherever their
// double feeds further double arithmetic: ocml's differ from glibc's on
// 0.3-25% of float arguments.  log and sqrt, and exp / sin / cos where the
// path rounds the result straight to float (fexp / fsin / fcos), stay ocml's:
// over all 2^32 float arguments that float is glibc's
// (profiles/r03_exhaustive/), and ocml's are table-free and faster.
PTG_D double dexp(double x) { return glibc::exp(x); }
PTG_D double dlog(double x) { return log(x); }
PTG_D double dpow(double x, double y) { return glibc::pow(x, y); }
PTG_D double dsin(double x) { return glibc::sin(x); }
PTG_D double dcos(double x) { return glibc::cos(x); }
PTG_D double dsqrt(double x) { return sqrt(x); }
PTG_D float fcos(float x) { return (float)cos((double)x); }
PTG_D float fsin(float x) { return (float)sin((double)x); }
PTG_D float fexp(float x) { return (float)exp((double)x); }

// ---- glibc's float results: exactly, or through ocml plus a certificate --
// Where the path rounds an expression of a glibc double to float, the two
// hot shading kernels (k_wf_shade, k_wf_sky) evaluate it with ocml's exp /
// pow / sin / cos - table-free, and 30-90 fewer VGPRs per kernel than glibc's
// algorithms inline, which is one more wave per SIMD - and keep that float
// when it is provably the float glibc's double gives.  When the proof fails
// (about 1 evaluation in 4 million) the kernel shades that path again with
// glibc's algorithms (a second, tiny launch over the paths it listed), so
// every float is glibc's.  The policy type says which: MathExact (glibc's
// algorithms, glibc_math.h) everywhere else, MathFast in those two kernels.
//  * D: over every float argument, ocml's double is at most D ulps from
//    glibc's (tools/exhaustive_f64.hip "distance" rows, profiles/r03_exhaustive/:
//    exp, sin, cos, pow(x, 5 / 1.5 / 0.25) all 1); kMaxLibDist = 4 is the
//    largest D the bounds below are sized for.
//  * each wrapper states how far its double v can then be from the double
//    the same expression gives with glibc's value: K ulps of v, K <= 4 (D + 1)
//    (a relative error eps is at most eps 2^53 ulps; two values on either side
//    of a binade edge count twice).  times_one_minus_div_pow sizes its own
//    margin.
//  * float_certain(v): every double within K ulps of v rounds to the same
//    float as v.  |v| >= 2^128 (inf included): float inf, as for every
//    double that close; |v| < 2^-151 (zero included): float +-0 (the
//    wrappers' zero results carry the same sign either way); otherwise v is
//    more than kCertUlps = 32 > K double ulps away from every float rounding
//    boundary - the midpoint of two adjacent floats, where the q bits of v
//    below float's quantum at v equal 2^(q-1) (q = 29 in float's normal
//    range, 30..54 in its subnormal range, where the quantum is 2^-149).
//    Across a binade edge v sits next to a float, not a midpoint.  NaN: no
//    certificate.
constexpr uint32_t kMaxLibDist = 4;
constexpr uint32_t kCertUlps = 32;
// float_certain's rare ranges (float inf / zero / subnormal results), out of
// the inlined fast path
__device__ __noinline__ inline bool float_certain_wide(uint64_t u, uint32_t margin)
{
    const uint32_t e = uint32_t(u >> 52) & 0x7ffu;
    if(e >= 1023u + 128u) return e != 0x7ffu || (u << 12) == 0;             // float inf (not NaN)
    if(e < 1023u - 151u) return true;                                        // float +-0
    const uint32_t q = e >= 1023u - 126u ? 29u : 926u - e;                   // bits below float's quantum
    const uint64_t sig = (u & 0x000fffffffffffffull) | 0x0010000000000000ull;
    const uint64_t low = sig & ((1ull << q) - 1), mid = 1ull << (q - 1);
    return (low > mid ? low - mid : mid - low) > margin;
}
PTG_D bool float_certain(double v, uint32_t margin = kCertUlps)
{
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    // float's normal range, exponent 897..1150: the 29 bits below float
    // precision are in the low word; their distance from 2^28 is > margin
    if(uint32_t(u >> 52 & 0x7ffu) - (1023u - 126u) <= 253u)
        return ((uint32_t(u) - (0x10000000u - margin)) & 0x1fffffffu) > 2u * margin;
    return float_certain_wide(u, margin);
}
// the certificate sites (tools/cert_probe.hip counts failures per site)
enum CertSite { CS_ACC_EXP, CS_EXP_TIMES, CS_ADD_MUL_POW, CS_DIV_MUL_POW, CS_TIMES_COS, CS_TIMES_SIN,
                CS_TIMES_ONE_MINUS_DIV_POW, CS_COUNT };
struct MathExact {   // glibc's algorithms, exp's table in global memory
    static constexpr bool kFast = false;
    static constexpr bool kLdsExp = false;
    static constexpr uint32_t fail_mask = 0;
    PTG_D void check(bool, double, int) {}
    PTG_D double exp(double x) const { return glibc::exp(x); }
};
struct MathExactLds : MathExact {   // the same, exp's table copied to LDS by the kernel (glibc::exp_table_to_lds)
    static constexpr bool kLdsExp = true;
    glibc::ExpTabLds xt;
    PTG_D double exp(double x) const { return glibc::exp(x, xt); }
};
// PTG_CERT_FAIL_ALL=1 (test build libptg_certfail.so only): every certificate
// fails, so every surface path takes the exact redo pass
#ifndef PTG_CERT_FAIL_ALL
#define PTG_CERT_FAIL_ALL 0
#endif
struct MathFast {    // ocml's, certified; fail_mask: bit CS_x when a certificate at site x did not hold
    static constexpr bool kFast = true;
    static constexpr bool kLdsExp = false;
    uint32_t fail_mask = 0;
    PTG_D void check(bool certain, double, int site) { fail_mask |= (certain && !PTG_CERT_FAIL_ALL) ? 0u : 1u << site; }
};

// Arguments where both libraries return the exact value, so the double is
// the same whatever follows: exp(0) = 1, sin(0) = 0, cos(0) = 1, pow(1, y) = 1,
// pow(0, y > 0) = 0 (C99 F.9; the path meets them - pow(1, 0.25) on every
// rejected BSDF sample, whose pdf is 1 - and their results are often exact
// float ties, which no rounding certificate covers).
PTG_D bool pow_exact_arg(double x, double y) { return x == 1.0 || (x == 0.0 && y > 0.0); }

// (float)((double)acc + exp(x)), acc >= 0: the sum is at least exp(x), so
// D ulps of exp(x) plus the two roundings is <= 2 (D + 1) ulps of the sum
// (the factor 2: the two sums may lie in adjacent binades).
template<class MP> PTG_D float acc_exp(float acc, double x, MP& mp)
{
    if constexpr(!MP::kFast) return (float)((double)acc + mp.exp(x));
    const double v = (double)acc + exp(x);
    mp.check(x == 0.0 || (acc >= 0.0f && float_certain(v)), v, CS_ACC_EXP);
    return (float)v;
}
// (float)(exp(x) * (double)s): D ulps of exp(x) times s is <= 2 D ulps of the
// product, plus the two roundings: <= 2 (2 D + 1).
template<class MP> PTG_D float exp_times(double x, float s, MP& mp)
{
    if constexpr(!MP::kFast) return (float)(mp.exp(x) * (double)s);
    const double v = exp(x) * (double)s;
    mp.check(x == 0.0 || float_certain(v), v, CS_EXP_TIMES);
    return (float)v;
}
// (float)((double)a + (double)b * pow(x, y)), a, b >= 0: the product is off by
// <= 2 D + 1 ulps of itself, the sum (>= the product) by one rounding more:
// <= 2 (2 D + 2) ulps of the sum.
template<class MP> PTG_D float add_mul_pow(float a, float b, double x, double y, MP& mp)
{
    if constexpr(!MP::kFast) return (float)((double)a + (double)b * glibc::pow(x, y));
    const double v = (double)a + (double)b * pow(x, y);
    mp.check(pow_exact_arg(x, y) || (a >= 0.0f && b >= 0.0f && float_certain(v)), v, CS_ADD_MUL_POW);
    return (float)v;
}
// (float)(a / (b * pow(x, y))), b * pow > 0: the divisor's relative error is
// (D + 1/2) 2^-52, the quotient's (D + 1) 2^-52: <= 4 (D + 1) ulps.
template<class MP> PTG_D float div_mul_pow(double a, double b, double x, double y, MP& mp)
{
    if constexpr(!MP::kFast) return (float)(a / (b * glibc::pow(x, y)));
    const double v = a / (b * pow(x, y));
    mp.check(pow_exact_arg(x, y) || float_certain(v), v, CS_DIV_MUL_POW);
    return (float)v;
}
// (float)((double)s * cos(phi)), (float)((double)s * sin(phi)): <= 2 (2 D + 1).
template<class MP> PTG_D float times_cos(float s, double phi, MP& mp)
{
    if constexpr(!MP::kFast) return (float)((double)s * glibc::cos(phi));
    const double v = (double)s * cos(phi);
    mp.check(phi == 0.0 || float_certain(v), v, CS_TIMES_COS);
    return (float)v;
}
template<class MP> PTG_D float times_sin(float s, double phi, MP& mp)
{
    if constexpr(!MP::kFast) return (float)((double)s * glibc::sin(phi));
    const double v = (double)s * sin(phi);
    mp.check(phi == 0.0 || float_certain(v), v, CS_TIMES_SIN);
    return (float)v;
}
// (float)((double)r * max(1 - g / pow(x, y), 0)), r >= 0.  q = g / pow is off
// by <= 2 D + 1 ulps of q.  q > 1 + 2^-48: both q exceed 1, the result is
// r * 0.  Otherwise w = 1 - q (exact for q in [0.5, 1], Sterbenz) is off by
// (2 D + 1) 2^s + 1 ulps of w, s = exponent of q minus exponent of w (s <= 0
// when q < 0.5); the product's relative error adds a rounding: the result is
// off by <= 4 ((2 D + 1) 2^max(s, 0) + 1) + 2 ulps, the margin below.
template<class MP> PTG_D float times_one_minus_div_pow(float r, double g, double x, double y, MP& mp)
{
    if constexpr(!MP::kFast) return (float)((double)r * gmax_d(1.0 - g / glibc::pow(x, y), 0.0));
    const double q = g / pow(x, y);
    const double w = gmax_d(1.0 - q, 0.0);
    const double v = (double)r * w;
    const int32_t s = int32_t((uint64_t)__double_as_longlong(q) >> 52 & 0x7ff) -
                      int32_t((uint64_t)__double_as_longlong(w) >> 52 & 0x7ff);
    const bool zero = q > 1.0 + 0x1p-48;
    const bool small = s <= 16 && w > 0.0;
    const uint32_t margin = 4u * (((2u * kMaxLibDist + 1u) << (s > 0 ? s : 0)) + 1u) + 2u;
    mp.check(pow_exact_arg(x, y) || (r >= 0.0f && (zero || (small && float_certain(v, margin)))), v,
             CS_TIMES_ONE_MINUS_DIV_POW);
    return (float)v;
}

PTG_D f3 mul_v3m3(f3 b, const m3& a) { return V3(dot(a.r[0], b), dot(a.r[1], b), dot(a.r[2], b)); }
PTG_D f3 mul_m3v3(const m3& b, f3 a)
{
    m3 t{{V3(b.r[0].x, b.r[1].x, b.r[2].x), V3(b.r[0].y, b.r[1].y, b.r[2].y), V3(b.r[0].z, b.r[1].z, b.r[2].z)}};
    return mul_v3m3(a, t);
}

// create_tangent_space (math.hh:419-435); threshold compared in double
PTG_D m3 tangent_space(f3 n)
{
    f3 major;
    if(fabs((double)n.x) < 0.57735026918962576451) major = V3(1, 0, 0);
    else if(fabs((double)n.y) < 0.57735026918962576451) major = V3(0, 1, 0);
    else major = V3(0, 0, 1);
    f3 t = normalize(cross(n, major));
    f3 b = cross(n, t);
    return m3{{t, b, n}};
}

// pcg4d (math.hh:466-473), simultaneous updates
PTG_D void pcg4d(u4& s)
{
    uint32_t x = s.x * 1664525u + 1013904223u, y = s.y * 1664525u + 1013904223u;
    uint32_t z = s.z * 1664525u + 1013904223u, w = s.w * 1664525u + 1013904223u;
    uint32_t a = x + y * w, b = y + z * x, c = z + x * y, d = w + y * z;
    a ^= a >> 16u; b ^= b >> 16u; c ^= c >> 16u; d ^= d >> 16u;
    s.x = a + b * d; s.y = b + c * a; s.z = c + a * b; s.w = d + b * c;
}
PTG_D f4 uniform4(u4& s)
{
    pcg4d(s);
    const float k = 2.3283064365386963e-10f;
    return f4{(float)s.x * k, (float)s.y * k, (float)s.z * k, (float)s.w * k};
}

} // namespace dm
} // namespace ptg
