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
    const float r = rcp_nr(x, ok);
    return ok ? r : 1.0f / x;
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

// double-precision library calls, as the reference makes them
PTG_D double dexp(double x) { return exp(x); }
PTG_D double dlog(double x) { return log(x); }
PTG_D double dpow(double x, double y) { return pow(x, y); }
PTG_D double dsin(double x) { return sin(x); }
PTG_D double dcos(double x) { return cos(x); }
PTG_D double dsqrt(double x) { return sqrt(x); }
PTG_D float fcos(float x) { return (float)dcos((double)x); }
PTG_D float fsin(float x) { return (float)dsin((double)x); }
PTG_D float fexp(float x) { return (float)dexp((double)x); }

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
