// Host-side vector arithmetic with the reference's exact float semantics.
//
// The scene arrays must come out byte-identical to the reference's
// (scene.cc / bvh.cc / mesh.cc compiled without fast-math), so every helper
// here performs the same IEEE operations in the same order as its reference
// counterpart in math.hh (cited per function).  Two C++ details of the
// reference matter and are reproduced on purpose:
//   * unqualified sqrt/sin/cos/tan/fabs on a float resolve to the C *double*
//     functions (math.hh includes <cmath> but only imports fmin/fmax into the
//     global namespace, math.hh:120-121), so the float argument is promoted,
//     the double result is rounded once on assignment;
//   * fmin/fmax are the float overloads (fminf/fmaxf), whose tie rule
//     (equal operands -> second operand) decides the sign of zero bounds.
// Compile this code with -ffp-contract=off and without -ffast-math.
#pragma once
#include "ptg.h"
#include <cmath>

namespace ptg {
namespace hm {

using f3 = ptg_float3;
using f4 = ptg_float4;
using m3 = ptg_mat3;
using m4 = ptg_mat4;

inline f3 v3(float x, float y, float z) { f3 r{}; r.x = x; r.y = y; r.z = z; return r; }
inline f4 v4(float x, float y, float z, float w) { f4 r{}; r.x = x; r.y = y; r.z = z; r.w = w; return r; }

// math.hh:44-61 element-wise operators
inline f3 operator+(f3 a, f3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 operator-(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 operator*(f3 a, f3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline f3 operator/(f3 a, f3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline f3 operator*(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline f3 operator*(float s, f3 a) { return v3(s * a.x, s * a.y, s * a.z); }
inline f3 operator/(f3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
inline f3 operator-(f3 a, float s) { return v3(a.x - s, a.y - s, a.z - s); }
inline f3 operator-(f3 a) { return v3(-a.x, -a.y, -a.z); }
inline f4 operator+(f4 a, f4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
inline f4 operator-(f4 a, f4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
inline f4 operator*(f4 a, f4 b) { return v4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
inline f4 operator*(f4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }

inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }            // math.hh:94
inline float dot(f4 a, f4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; } // math.hh:95
// math.hh:106 length() = sqrt(dot): double sqrt of the float dot, rounded to float
inline float length(f3 a) { return (float)std::sqrt((double)dot(a, a)); }
inline f3 normalize(f3 a) { return a / length(a); }                                   // math.hh:110
inline f3 cross(f3 a, f3 b)                                                            // math.hh:125
{ return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
// fminf/fmaxf via the float overloads (math.hh:120-123)
inline float fminf_(float a, float b) { return std::fmin(a, b); }
inline float fmaxf_(float a, float b) { return std::fmax(a, b); }
inline f3 vmin(f3 a, f3 b) { return v3(fminf_(a.x, b.x), fminf_(a.y, b.y), fminf_(a.z, b.z)); }
inline f3 vmax(f3 a, f3 b) { return v3(fmaxf_(a.x, b.x), fmaxf_(a.y, b.y), fmaxf_(a.z, b.z)); }
inline float comp(const f3& a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }   // pick, math.hh:117
inline float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }          // math.hh:145
inline f4 mix4(f4 a, f4 b, float t) { return a * (1.0f - t) + b * t; }                   // math.hh:148

// ---- matrices (row vectors; math.hh:151-338) ----
inline m3 mat3_rows(f3 a, f3 b, f3 c) { m3 m; m.r[0] = a; m.r[1] = b; m.r[2] = c; return m; }
inline m4 mat4_rows(f4 a, f4 b, f4 c, f4 d) { m4 m; m.r[0] = a; m.r[1] = b; m.r[2] = c; m.r[3] = d; return m; }

inline m3 transpose(const m3& a)
{ return mat3_rows(v3(a.r[0].x, a.r[1].x, a.r[2].x), v3(a.r[0].y, a.r[1].y, a.r[2].y), v3(a.r[0].z, a.r[1].z, a.r[2].z)); }
inline m4 transpose(const m4& a)
{
    return mat4_rows(v4(a.r[0].x, a.r[1].x, a.r[2].x, a.r[3].x), v4(a.r[0].y, a.r[1].y, a.r[2].y, a.r[3].y),
                     v4(a.r[0].z, a.r[1].z, a.r[2].z, a.r[3].z), v4(a.r[0].w, a.r[1].w, a.r[2].w, a.r[3].w));
}
inline m3 scale(float s, const m3& a) { return mat3_rows(a.r[0] * s, a.r[1] * s, a.r[2] * s); }   // mul_fm3
inline m3 add(const m3& a, const m3& b) { return mat3_rows(a.r[0] + b.r[0], a.r[1] + b.r[1], a.r[2] + b.r[2]); }

// mul_m3v3 / mul_m4v4 / mul_v4m4 (math.hh:224-228): y_k = dot(row k of transpose(b), a)
inline f3 mul_v3m3(f3 b, const m3& a) { return v3(dot(a.r[0], b), dot(a.r[1], b), dot(a.r[2], b)); }
inline f4 mul_v4m4(f4 b, const m4& a) { return v4(dot(a.r[0], b), dot(a.r[1], b), dot(a.r[2], b), dot(a.r[3], b)); }
inline f3 mul_m3v3(const m3& b, f3 a) { return mul_v3m3(a, transpose(b)); }
inline f4 mul_m4v4(const m4& b, f4 a) { return mul_v4m4(a, transpose(b)); }

// mul_m3m3(b, a) / mul_m4m4(b, a) (math.hh:238-256): row i of a times the columns of b
inline m3 mul_m3m3(const m3& b, const m3& a)
{
    m3 bt = transpose(b);
    return mat3_rows(v3(dot(a.r[0], bt.r[0]), dot(a.r[0], bt.r[1]), dot(a.r[0], bt.r[2])),
                     v3(dot(a.r[1], bt.r[0]), dot(a.r[1], bt.r[1]), dot(a.r[1], bt.r[2])),
                     v3(dot(a.r[2], bt.r[0]), dot(a.r[2], bt.r[1]), dot(a.r[2], bt.r[2])));
}
inline m4 mul_m4m4(const m4& b, const m4& a)
{
    m4 bt = transpose(b);
    m4 r;
    for(int i = 0; i < 4; ++i)
        r.r[i] = v4(dot(a.r[i], bt.r[0]), dot(a.r[i], bt.r[1]), dot(a.r[i], bt.r[2]), dot(a.r[i], bt.r[3]));
    return r;
}

inline m4 expand(const m3& m)                                                          // expand_m3m4
{
    return mat4_rows(v4(m.r[0].x, m.r[0].y, m.r[0].z, 0), v4(m.r[1].x, m.r[1].y, m.r[1].z, 0),
                     v4(m.r[2].x, m.r[2].y, m.r[2].z, 0), v4(0, 0, 0, 1));
}
inline m3 extract(const m4& m)                                                         // extract_m4m3
{ return mat3_rows(v3(m.r[0].x, m.r[0].y, m.r[0].z), v3(m.r[1].x, m.r[1].y, m.r[1].z), v3(m.r[2].x, m.r[2].y, m.r[2].z)); }

// inverse4 (math.hh:179-221, GLM cofactor form), same operation order.
inline m4 inverse(const m4& a)
{
    const f4 *r = a.r;
    float c00 = r[2].z * r[3].w - r[3].z * r[2].w;
    float c02 = r[1].z * r[3].w - r[3].z * r[1].w;
    float c03 = r[1].z * r[2].w - r[2].z * r[1].w;
    float c04 = r[2].y * r[3].w - r[3].y * r[2].w;
    float c06 = r[1].y * r[3].w - r[3].y * r[1].w;
    float c07 = r[1].y * r[2].w - r[2].y * r[1].w;
    float c08 = r[2].y * r[3].z - r[3].y * r[2].z;
    float c10 = r[1].y * r[3].z - r[3].y * r[1].z;
    float c11 = r[1].y * r[2].z - r[2].y * r[1].z;
    float c12 = r[2].x * r[3].w - r[3].x * r[2].w;
    float c14 = r[1].x * r[3].w - r[3].x * r[1].w;
    float c15 = r[1].x * r[2].w - r[2].x * r[1].w;
    float c16 = r[2].x * r[3].z - r[3].x * r[2].z;
    float c18 = r[1].x * r[3].z - r[3].x * r[1].z;
    float c19 = r[1].x * r[2].z - r[2].x * r[1].z;
    float c20 = r[2].x * r[3].y - r[3].x * r[2].y;
    float c22 = r[1].x * r[3].y - r[3].x * r[1].y;
    float c23 = r[1].x * r[2].y - r[2].x * r[1].y;
    f4 f0 = v4(c00, c00, c02, c03), f1 = v4(c04, c04, c06, c07), f2 = v4(c08, c08, c10, c11);
    f4 f3_ = v4(c12, c12, c14, c15), f4_ = v4(c16, c16, c18, c19), f5 = v4(c20, c20, c22, c23);
    f4 e0 = v4(r[1].x, r[0].x, r[0].x, r[0].x), e1 = v4(r[1].y, r[0].y, r[0].y, r[0].y);
    f4 e2 = v4(r[1].z, r[0].z, r[0].z, r[0].z), e3 = v4(r[1].w, r[0].w, r[0].w, r[0].w);
    const f4 sa = v4(+1, -1, +1, -1), sb = v4(-1, +1, -1, +1);
    m4 inv = mat4_rows((e1 * f0 - e2 * f1 + e3 * f2) * sa, (e0 * f0 - e2 * f3_ + e3 * f4_) * sb,
                       (e0 * f1 - e1 * f3_ + e3 * f5) * sa, (e0 * f2 - e1 * f4_ + e2 * f5) * sb);
    float det = dot(r[0], v4(inv.r[0].x, inv.r[1].x, inv.r[2].x, inv.r[3].x));
    float k = 1.0f / det;
    return mat4_rows(inv.r[0] * k, inv.r[1] * k, inv.r[2] * k, inv.r[3] * k);
}

inline m4 scaling(f3 s) { return mat4_rows(v4(s.x, 0, 0, 0), v4(0, s.y, 0, 0), v4(0, 0, s.z, 0), v4(0, 0, 0, 1)); }
inline m4 translation(f3 o) { return mat4_rows(v4(1, 0, 0, 0), v4(0, 1, 0, 0), v4(0, 0, 1, 0), v4(o.x, o.y, o.z, 1)); }

// rotation_euler (math.hh:305-318): double sin/cos of each float angle
inline m4 rotation_euler(f3 e)
{
    float sp = (float)std::sin((double)e.x), cp = (float)std::cos((double)e.x);
    float sy = (float)std::sin((double)e.y), cy = (float)std::cos((double)e.y);
    float sr = (float)std::sin((double)e.z), cr = (float)std::cos((double)e.z);
    m3 pitch = mat3_rows(v3(1, 0, 0), v3(0, cp, -sp), v3(0, sp, cp));
    m3 yaw = mat3_rows(v3(cy, 0, sy), v3(0, 1, 0), v3(-sy, 0, cy));
    m3 roll = mat3_rows(v3(cr, -sr, 0), v3(sr, cr, 0), v3(0, 0, 1));
    return expand(mul_m3m3(roll, mul_m3m3(yaw, pitch)));
}

// create_tangent / create_tangent_space (math.hh:419-435); the 1/sqrt(3)
// threshold is compared in double precision, as in the reference.
inline f3 create_tangent(f3 n)
{
    f3 major;
    if(std::fabs((double)n.x) < 0.57735026918962576451) major = v3(1, 0, 0);
    else if(std::fabs((double)n.y) < 0.57735026918962576451) major = v3(0, 1, 0);
    else major = v3(0, 0, 1);
    return normalize(cross(n, major));
}
inline m3 create_tangent_space(f3 n)
{
    f3 t = create_tangent(n);
    f3 b = cross(n, t);
    return mat3_rows(t, b, n);
}

// pcg4d (math.hh:466-473): the two mixing rounds are SIMULTANEOUS updates.
inline ptg_uint4 pcg4d(ptg_uint4* s)
{
    uint32_t x = s->x * 1664525u + 1013904223u, y = s->y * 1664525u + 1013904223u;
    uint32_t z = s->z * 1664525u + 1013904223u, w = s->w * 1664525u + 1013904223u;
    uint32_t nx = x + y * w, ny = y + z * x, nz = z + x * y, nw = w + y * z;
    x = nx ^ (nx >> 16); y = ny ^ (ny >> 16); z = nz ^ (nz >> 16); w = nw ^ (nw >> 16);
    nx = x + y * w; ny = y + z * x; nz = z + x * y; nw = w + y * z;
    s->x = nx; s->y = ny; s->z = nz; s->w = nw;
    return *s;
}
// generate_uniform_random4 (math.hh:475-485)
inline f4 uniform4(ptg_uint4* s)
{
    ptg_uint4 v = pcg4d(s);
    const float k = 2.3283064365386963e-10f;
    return v4((float)v.x * k, (float)v.y * k, (float)v.z * k, (float)v.w * k);
}

} // namespace hm
} // namespace ptg
