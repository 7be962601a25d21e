/* pt_oracle.c - CPU restatement of the reference hot path (TEST ORACLE ONLY).
 *
 * Restates, in plain C11 with strict IEEE arithmetic (no fast-math, no FP
 * contraction; see oracle/Makefile), the per-sample path tracer of
 * Kalache-abdesattar/Path-Tracing...but-on-the-LUMI-cluster @ v1:
 * path_tracer.hh (samplers, BSDF, NEE, Nishita atmosphere,
 * path_trace_pixel, tonemap_pixel), ray_query.hh (two-level stackless BVH
 * traversal) and the math.hh helpers they use.
 *
 * Precision rules reproduced on purpose (the reference is C++ where an
 * unqualified sqrt/exp/log/pow/sin/cos/fabs/fma/floor/round on a float
 * resolves to the C *double* function - only fmin/fmax are imported as float
 * overloads, math.hh:120-121):
 *   - every such call is evaluated in double and, where the reference keeps
 *     computing with the double result (e.g. `f0 + x * pow(..)`,
 *     `acc += exp(..)`, `2*v / (v + sqrt(..))`), so does this code, rounding
 *     to float exactly where the reference assigns to a float;
 *   - literals such as `1.0 - p` are double;
 *   - fminf/fmaxf keep their tie rule (equal operands -> second operand).
 * Pinned against the reference itself built strict (oracle/Makefile
 * REF_MODE=strict): tests/test_oracle.py requires bit-identical
 * per-sample output.  The GPU kernel (csrc/pt_kernels.hip) is checked
 * against this file.
 */
#include "pt_oracle.h"
#include <math.h>
#include <string.h>

#define PI_D 3.14159265358979323846
#define PI_F ((float)PI_D)
#define EARTH_RADIUS 6.3781e6f                 /* config.hh:34 */
#define ATMOSPHERE_HEIGHT 1.0e5f               /* config.hh:37 */
#define RAYLEIGH_SCALE_HEIGHT 7994.0f          /* config.hh:39 */
#define MIE_SCALE_HEIGHT 1200.0f               /* config.hh:42 */
#define MIE_ANISOTROPY 0.80f                   /* config.hh:41 */
#define MIN_RAY_DIST 1e-4f                     /* config.hh:30 */
#define MAX_RAY_DIST 1e9f                      /* config.hh:31 */
#define REGULARIZATION_GAMMA 0.15f             /* config.hh:32 */
#define PRIMARY_ITERATIONS 8                   /* config.hh:35 */
#define SECONDARY_ITERATIONS 4                 /* config.hh:36 */

typedef struct { float x, y; } f2;
typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;
typedef struct { f3 r[3]; } m3;
typedef struct { uint32_t x, y, z, w; } u4;

/* reference-layout records */
typedef struct { float x, y, z, pad; } rf3;
typedef struct { float x, y, z, w; } rf4;
typedef struct { uint32_t node_count, node_offset; } rbvh;
typedef struct { float min_x, min_y, min_z, max_x, max_y, max_z; } rnode;
typedef struct { uint32_t accept, cancel; } rlink;
typedef struct { uint32_t vertex_count, triangle_count, index_offset, base_vertex_offset; } rmesh;
typedef struct { rbvh blas; rmesh m; uint32_t pad[2]; rf4 transform[4]; rf4 inv_transform[4]; } rinstance;
typedef struct {
    rf3 orientation[3]; rf3 position;
    float aspect_ratio, inv_focal_length, focal_distance, aperture_angle;
    int32_t aperture_polygon; float aperture_radius; uint32_t pad[2];
} rcamera;
typedef struct { rf3 direction, color; float cos_solid_angle; uint32_t pad[3]; } rlight;
typedef struct { rbvh tlas; uint32_t pad[2]; rcamera cam; rlight light; } rsubframe;

_Static_assert(sizeof(rinstance) == 160, "tlas_instance layout");
_Static_assert(sizeof(rcamera) == 96, "camera layout");
_Static_assert(sizeof(rlight) == 48, "light layout");
_Static_assert(sizeof(rsubframe) == 160, "subframe layout");

/* ---- math.hh helpers --------------------------------------------------- */
static inline f3 V3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add3(f3 a, f3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub3(f3 a, f3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul3(f3 a, f3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 mul3s(f3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline f3 smul3(float s, f3 a) { return V3(s * a.x, s * a.y, s * a.z); }
static inline f3 div3s(f3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline f3 neg3(f3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }          /* math.hh:94 */
static inline float len3(f3 a) { return (float)sqrt((double)dot3(a, a)); }                  /* math.hh:106 */
static inline f3 norm3(f3 a) { return div3s(a, len3(a)); }                                   /* math.hh:110 */
static inline f3 cross3(f3 a, f3 b)                                                          /* math.hh:125 */
{ return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline float clampf_(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); } /* math.hh:134 */
static inline float mixf_(float a, float b, float t) { return a * (1.0f - t) + b * t; }       /* math.hh:145 */
static inline float signf_(float v)                                                          /* math.hh:127-132 */
{
    if(v < 0) return -1.0f;
    if(v > 0) return 1.0f;
    return v == -0.0f ? -0.0f : +0.0f;
}
static inline f3 ld3(const void* base, size_t i) { const rf3* p = (const rf3*)base + i; return V3(p->x, p->y, p->z); }
static inline f4 ld4(const void* base, size_t i) { const rf4* p = (const rf4*)base + i; f4 r = {p->x, p->y, p->z, p->w}; return r; }
static inline f3 rf3v(rf3 a) { return V3(a.x, a.y, a.z); }

/* mul_v3m3 (math.hh:224): rows dotted with b */
static inline f3 mul_v3m3(f3 b, const m3* a) { return V3(dot3(a->r[0], b), dot3(a->r[1], b), dot3(a->r[2], b)); }
/* mul_m3v3 (math.hh:227) = mul_v3m3(a, transpose(b)) */
static inline f3 mul_m3v3(const m3* b, f3 a)
{
    m3 t = {{V3(b->r[0].x, b->r[1].x, b->r[2].x), V3(b->r[0].y, b->r[1].y, b->r[2].y), V3(b->r[0].z, b->r[1].z, b->r[2].z)}};
    return mul_v3m3(a, &t);
}

/* create_tangent / create_tangent_space (math.hh:419-435) */
static inline m3 tangent_space(f3 n)
{
    f3 major;
    if(fabs((double)n.x) < 0.57735026918962576451) major = V3(1, 0, 0);
    else if(fabs((double)n.y) < 0.57735026918962576451) major = V3(0, 1, 0);
    else major = V3(0, 0, 1);
    f3 t = norm3(cross3(n, major));
    f3 b = cross3(n, t);
    m3 m = {{t, b, n}};
    return m;
}

static inline f3 reflect3(f3 I, f3 N) { return sub3(I, smul3(2.0f * dot3(N, I), N)); }       /* math.hh:442-445 */
static inline f3 refract3(f3 I, f3 N, float eta)                                            /* math.hh:447-453 */
{
    float ndoti = dot3(N, I);
    float k = 1.0f - eta * eta * (1.0f - ndoti * ndoti);
    if(k < 0.0f) return V3(0, 0, 0);
    float s = (float)((double)(eta * ndoti) + sqrt((double)k));
    return sub3(smul3(eta, I), smul3(s, N));
}

/* inv_erf (math.hh:455-463): note the inner sqrt stays double */
static inline float inv_erf(float x)
{
    float ln1x2 = (float)log((double)(1 - x * x));
    const float a = 0.147f;
    const float p = 2.0f / (PI_F * a);
    float k = p + ln1x2 * 0.5f;
    float k2 = k * k;
    double inner = sqrt((double)(k2 - ln1x2 * (1.0f / a)));
    return (float)((double)signf_(x) * sqrt(inner - (double)k));
}

/* pcg4d (math.hh:466-473): simultaneous vector updates */
static inline void pcg4d(u4* s)
{
    uint32_t x = s->x * 1664525u + 1013904223u, y = s->y * 1664525u + 1013904223u;
    uint32_t z = s->z * 1664525u + 1013904223u, w = s->w * 1664525u + 1013904223u;
    uint32_t a = x + y * w, b = y + z * x, c = z + x * y, d = w + y * z;
    a ^= a >> 16u; b ^= b >> 16u; c ^= c >> 16u; d ^= d >> 16u;
    s->x = a + b * d; s->y = b + c * a; s->z = c + a * b; s->w = d + b * c;
}
static inline f4 uniform4(u4* s)                                                              /* math.hh:475-485 */
{
    pcg4d(s);
    const float k = 2.3283064365386963e-10f;
    f4 r = {(float)s->x * k, (float)s->y * k, (float)s->z * k, (float)s->w * k};
    return r;
}

/* ray_sphere_intersection (math.hh:404-417) */
static inline int ray_sphere(f3 o, f3 d, f3 c, float radius, float* tmin, float* tmax)
{
    f3 oc = sub3(o, c);
    float b = dot3(oc, d);
    float cc = dot3(oc, oc) - radius * radius;
    float disc = b * b - cc;
    if(disc < 0) return 0;
    disc = (float)sqrt((double)disc);
    *tmin = -b - disc;
    *tmax = -b + disc;
    return 1;
}

/* ---- ray queries (ray_query.hh) ---------------------------------------- */
typedef struct {
    rbvh as;
    f3 origin, dir, inv_dir;
    uint32_t link_offset, node_index;
} rq_ctx;

typedef struct { f3 bary; float thit; uint32_t instance_id, primitive_id; int back_face; } rq_hit;

typedef struct {
    const orc_scene* s;
    rq_ctx tlas, blas;
    rmesh mesh;
    float tmin, tmax;
    int blas_axis;
    rq_hit candidate, closest;
    uint64_t* cnt;
} rq_state;

static inline float rcp_or_big(float d) { return d == 0 ? (float)1e40 : 1.0f / d; }
static inline uint32_t octant_of(f3 d) { return (d.x > 0 ? 1u : 0u) | (d.y > 0 ? 2u : 0u) | (d.z > 0 ? 4u : 0u); }

/* ray_query_initialize (ray_query.hh:111-151) */
static void rq_init(rq_state* q, const orc_scene* s, rbvh tlas, f3 o, f3 d, float tmin, float tmax, uint64_t* cnt)
{
    q->s = s;
    q->tlas.as = tlas;
    q->tlas.origin = o;
    q->tlas.dir = d;
    q->tlas.inv_dir = V3(rcp_or_big(d.x), rcp_or_big(d.y), rcp_or_big(d.z));
    q->tlas.link_offset = tlas.node_offset * 8 + octant_of(d) * tlas.node_count;
    q->tlas.node_index = 0;
    q->blas.node_index = 0;
    q->tmin = tmin;
    q->tmax = tmax;
    q->blas_axis = -1;
    rq_hit none = {{0, 0, 0}, -1, 0xFFFFFFFFu, 0, 0};
    q->candidate = none;
    q->closest = none;
    q->cnt = cnt;
    if(cnt) cnt[4]++;
}

/* ray_query_traverse (ray_query.hh:184-223) */
static uint32_t rq_traverse(rq_ctx* c, const rnode* nodes, const rlink* links, float tmin, float tmax, uint64_t* cnt)
{
    const f3 inv = c->inv_dir, o = c->origin;
    while(c->node_index < c->as.node_count)
    {
        const rnode* n = nodes + c->as.node_offset + c->node_index;
        const rlink* l = links + c->link_offset + c->node_index;
        if(cnt) cnt[1]++;
        f3 t0 = mul3(sub3(V3(n->min_x, n->min_y, n->min_z), o), inv);
        f3 t1 = mul3(sub3(V3(n->max_x, n->max_y, n->max_z), o), inv);
        f3 lo = V3(fminf(t0.x, t1.x), fminf(t0.y, t1.y), fminf(t0.z, t1.z));
        f3 hi = V3(fmaxf(t0.x, t1.x), fmaxf(t0.y, t1.y), fmaxf(t0.z, t1.z));
        float near_ = fmaxf(lo.x, fmaxf(lo.y, lo.z));
        float far_ = fminf(hi.x, fminf(hi.y, hi.z));
        if(near_ <= far_ && far_ > tmin && near_ < tmax)
        {
            uint32_t accept = l->accept & 0x7FFFFFFFu;
            if(accept != l->accept) { c->node_index = l->cancel; return accept; }
            c->node_index = accept;
        }
        else c->node_index = l->cancel;
    }
    return 0xFFFFFFFFu;
}

/* ray_query_enter_blas (ray_query.hh:153-182) + ray_triangle_intersection_preprocess (math.hh:340-356) */
static void rq_enter_blas(rq_state* q, uint32_t index)
{
    const rinstance* in = (const rinstance*)q->s->instances + index;
    if(q->cnt) q->cnt[3]++;
    q->blas.as = in->blas;
    f3 o = q->tlas.origin;
    const rf4* M = in->inv_transform;
    /* mul_m4v4(inv, (o,1)): component k = M[0].k*o.x + M[1].k*o.y + M[2].k*o.z + M[3].k*1 */
    q->blas.origin = V3(M[0].x * o.x + M[1].x * o.y + M[2].x * o.z + M[3].x * 1.0f,
                        M[0].y * o.x + M[1].y * o.y + M[2].y * o.z + M[3].y * 1.0f,
                        M[0].z * o.x + M[1].z * o.y + M[2].z * o.z + M[3].z * 1.0f);
    f3 d0 = q->tlas.dir;
    f3 d = V3(M[0].x * d0.x + M[1].x * d0.y + M[2].x * d0.z,
              M[0].y * d0.x + M[1].y * d0.y + M[2].y * d0.z,
              M[0].z * d0.x + M[1].z * d0.y + M[2].z * d0.z);
    q->blas.inv_dir = V3(rcp_or_big(d.x), rcp_or_big(d.y), rcp_or_big(d.z));
    q->blas.link_offset = in->blas.node_offset * 8 + octant_of(d) * in->blas.node_count;
    q->blas.node_index = 0;
    q->mesh = in->m;
    f3 ad = V3((float)fabs((double)d.x), (float)fabs((double)d.y), (float)fabs((double)d.z));
    f3 rd = d;
    q->blas_axis = 2;
    if(ad.x > ad.y && ad.x > ad.z) { q->blas_axis = 0; rd = V3(d.z, d.y, d.x); }
    else if(ad.y > ad.z) { q->blas_axis = 1; rd = V3(d.x, d.z, d.y); }
    q->blas.dir = mul3s(V3(rd.x, rd.y, 1.0f), 1.0f / rd.z);
}

/* ray_query_test_triangle (ray_query.hh:225-246) + ray_triangle_intersection (math.hh:358-401) */
static int rq_test_triangle(rq_state* q)
{
    const orc_scene* s = q->s;
    if(q->cnt) q->cnt[2]++;
    uint32_t tri = q->mesh.index_offset + q->candidate.primitive_id * 3;
    uint32_t bv = q->mesh.base_vertex_offset;
    f3 o = q->blas.origin;
    f3 A = sub3(ld3(s->pos, bv + s->indices[tri + 0]), o);
    f3 B = sub3(ld3(s->pos, bv + s->indices[tri + 1]), o);
    f3 C = sub3(ld3(s->pos, bv + s->indices[tri + 2]), o);
    f3 x = V3(A.x, B.x, C.x), y = V3(A.y, B.y, C.y), z = V3(A.z, B.z, C.z);
    int axis = q->blas_axis;
    if(axis == 0) { x = z; z = V3(A.x, B.x, C.x); }
    else if(axis == 1) { y = z; z = V3(A.y, B.y, C.y); }
    f3 S = q->blas.dir;
    x = sub3(x, smul3(S.x, z));
    y = sub3(y, smul3(S.y, z));
    f3 uvw = cross3(y, x);
    float det = uvw.x + uvw.y + uvw.z;
    f3 uvt = mul3s(V3(uvw.x, uvw.y, dot3(uvw, smul3(S.z, z))), 1.0f / det);
    int back = det < 0;
    if(S.z < 0) back = !back;
    if(axis != 2) back = !back;
    int hit = det != 0.0f && uvt.z >= 0.0f &&
              ((uvw.x >= 0.0f && uvw.y >= 0.0f && uvw.z >= 0.0f) || (uvw.x <= 0.0f && uvw.y <= 0.0f && uvw.z <= 0.0f));
    q->candidate.thit = uvt.z;
    q->candidate.bary = V3(uvt.x, uvt.y, 1.0f - uvt.x - uvt.y);
    q->candidate.back_face = back;
    return hit && q->candidate.thit < q->tmax && q->candidate.thit > q->tmin;
}

/* ray_query_proceed (ray_query.hh:248-278) */
static int rq_proceed(rq_state* q)
{
    const rnode* nodes = (const rnode*)q->s->nodes;
    const rlink* links = (const rlink*)q->s->links;
    for(;;)
    {
        uint32_t leaf = rq_traverse(q->blas_axis < 0 ? &q->tlas : &q->blas, nodes, links, q->tmin, q->tmax, q->cnt);
        if(leaf != 0xFFFFFFFFu)
        {
            if(q->blas_axis < 0) { q->candidate.instance_id = leaf; rq_enter_blas(q, leaf); }
            else
            {
                q->candidate.primitive_id = leaf;
                if(rq_test_triangle(q)) return 1;
            }
        }
        else
        {
            if(q->blas_axis < 0) return 0;
            q->blas_axis = -1;
        }
    }
}

/* ray_query_confirm (ray_query.hh:280-290) */
static inline void rq_confirm(rq_state* q)
{
    q->closest = q->candidate;
    q->tmax = q->candidate.thit;
}

/* ---- path_tracer.hh ----------------------------------------------------- */
typedef struct {
    const orc_scene* s;
    rbvh tlas;
    f3 light_dir, light_color;
    float light_cos;
    uint64_t* cnt;
} pt_ctx;

typedef struct {
    float thit;
    f3 pos;
    m3 tbn;
    f3 albedo;
    float alpha, roughness, metallic, emission, transmission, eta, nee_pdf;
} hit_info;

/* sample_gaussian (:12-17) */
static inline float sample_gaussian(float u, float sigma, float eps)
{
    float k = u * 2.0f - 1.0f;
    k = clampf_(k, -(1.0f - eps), 1.0f - eps);
    return sigma * 1.41421356f * inv_erf(k);
}
/* sample_gaussian_weighted_disk (:19-25) */
static inline f2 gaussian_disk(f2 u, float sigma)
{
    float r = (float)sqrt((double)u.x);
    float theta = 2.0f * PI_F * u.y;
    r = sample_gaussian(r, sigma, 1e-6f);
    f2 o = {r * (float)cos((double)theta), r * (float)sin((double)theta)};
    return o;
}
/* sample_cosine_hemisphere (:27-33) */
static inline f3 cosine_hemisphere(f2 u)
{
    float r = (float)sqrt((double)u.x);
    float theta = 2.0f * PI_F * u.y;
    f2 d = {r * (float)cos((double)theta), r * (float)sin((double)theta)};
    return V3(d.x, d.y, (float)sqrt((double)fmaxf(0.0f, 1.0f - (d.x * d.x + d.y * d.y))));
}
/* cosine_hemisphere_pdf (:35-38) */
static inline float cosine_pdf(f3 d) { return fmaxf(d.z * (1.0f / PI_F), 0.0f); }
/* sample_cone (:40-48) */
static inline f3 sample_cone(f3 dir, float cos_min, f2 u)
{
    float ct = mixf_(1.0f, cos_min, u.x);
    float st = (float)sqrt((double)(1.0f - ct * ct));
    float phi = u.y * 2.0f * PI_F;
    m3 ts = tangent_space(dir);
    return mul_m3v3(&ts, V3((float)cos((double)phi) * st, (float)sin((double)phi) * st, ct));
}
/* sample_regular_polygon (:50-62) */
static inline f2 regular_polygon(f2 u, float angle, uint32_t sides)
{
    float side = (float)floor((double)(u.x * (float)sides));
    u.x *= (float)sides;
    u.x = (float)((double)u.x - floor((double)u.x));
    float side_radians = (2.0f * PI_F) / (float)sides;
    float a1 = side_radians * side + angle;
    float a2 = side_radians * (side + 1.0f) + angle;
    f2 b = {(float)sin((double)a1), (float)cos((double)a1)};
    f2 c = {(float)sin((double)a2), (float)cos((double)a2)};
    if(u.x + u.y > 1.0f) { u.x = 1.0f - u.x; u.y = 1.0f - u.y; }
    f2 r = {b.x * u.x + c.x * u.y, b.y * u.x + c.y * u.y};
    return r;
}
/* sample_ggx_vndf (:67-83) */
static inline f3 ggx_vndf(f3 view, float roughness, f2 u)
{
    if(roughness < 1e-3f) return V3(0, 0, 1);
    f3 v = norm3(V3(roughness * view.x, roughness * view.y, view.z));
    float phi = 2.0f * PI_F * u.x;
    float z = (float)fma((double)(1.0f - u.y), (double)(1.0f + v.z), (double)(-v.z));
    float sin_theta = (float)sqrt((double)clampf_(1.0f - z * z, 0.0f, 1.0f));
    float x = (float)((double)sin_theta * cos((double)phi));
    float y = (float)((double)sin_theta * sin((double)phi));
    f3 h = add3(V3(x, y, z), v);
    return norm3(V3(roughness * h.x, roughness * h.y, fmaxf(0.0f, h.z)));
}
/* fresnel_schlick_bidir_attenuated (:89-98) */
static inline float fresnel_att(float vdh, float f0, float eta, float roughness)
{
    if(eta > 1.0f)
    {
        float s2 = eta * eta * (1.0f - vdh * vdh);
        if(s2 >= 1.0f) return 1.0f;
        vdh = (float)sqrt((double)(1.0f - s2));
    }
    return (float)((double)f0 + (double)(fmaxf(1.0f - roughness, f0) - f0) * pow((double)fmaxf(1.0f - vdh, 0.0f), 5.0));
}
/* trowbridge_reitz_distribution (:105-110) */
static inline float tr_distribution(float hdotn, float a)
{
    float a2 = a * a;
    float denom = hdotn * hdotn * (a2 - 1.0f) + 1.0f;
    return a2 / fmaxf(PI_F * denom * denom, 1e-10f);
}
/* trowbridge_reitz_masking_shadowing (:112-123) */
static inline float tr_masking_shadowing(float ldotn, float ldoth, float vdotn, float vdoth, float a)
{
    if(vdotn * vdoth < 0) return 0;
    if(ldotn * ldoth < 0) return 0;
    double l = fabs((double)vdotn) * sqrt((double)(ldotn * ldotn - a * a * ldotn * ldotn + a * a));
    double v = fabs((double)ldotn) * sqrt((double)(vdotn * vdotn - a * a * vdotn * vdotn + a * a));
    return (float)(0.5 / (l + v));
}
/* trowbridge_reitz_masking (:125-129) */
static inline float tr_masking(float vdotn, float vdoth, float a)
{
    if(vdotn * vdoth < 0) return 0;
    return (float)((double)(2.0f * vdotn) / ((double)vdotn + sqrt((double)(vdotn * vdotn * (1.0f - a * a) + a * a))));
}

/* bsdf_core (:131-181) */
static f3 bsdf_core(f3 light, f3 h, f3 view, f3 albedo, float roughness, float metallic, float transmission,
                    float eta, float f0, float distribution, float* rpdf, float* dpdf, float* tpdf)
{
    const int brdf = light.z > 0;
    const float ldotn = light.z, vdotn = view.z;
    const float vdoth = dot3(view, h), ldoth = dot3(light, h);
    float fresnel = fresnel_att(vdoth, f0, eta, 0);
    float geometry = tr_masking_shadowing(ldotn, ldoth, vdotn, vdoth, roughness);
    float G1 = tr_masking(vdotn, vdoth, roughness);
    f3 color;
    if(brdf)
    {
        float spec = fresnel * (1.0f - metallic);
        color = V3((albedo.x * metallic + spec) * geometry * distribution,
                   (albedo.y * metallic + spec) * geometry * distribution,
                   (albedo.z * metallic + spec) * geometry * distribution);
        float diffuse = (1.0f - fresnel) * (1.0f - metallic) * (1.0f - transmission) / PI_F;
        color = add3(color, smul3(diffuse, albedo));
        *rpdf = G1 * distribution / (4.0f * view.z);
        *dpdf = cosine_pdf(light);
        *tpdf = 0;
    }
    else
    {
        float denom = eta * vdoth + ldoth;
        double k = (double)transmission * fabs((double)(vdoth * ldoth)) * (double)(1.0f - fresnel) * 4.0 *
                   (double)geometry * (double)distribution / (double)(denom * denom);
        color = mul3s(albedo, (float)k);
        *rpdf = 0;
        *dpdf = 0;
        *tpdf = (float)(fabs((double)(vdoth * ldoth)) * (double)G1 * (double)distribution /
                        (fabs((double)view.z) * (double)denom * (double)denom));
    }
    return mul3s(color, (float)fabs((double)ldotn));
}

static inline float luminance(f3 c) { return dot3(c, V3(0.2126f, 0.7152f, 0.0722f)); }        /* math.hh:437-440 */

/* the three lobe probabilities shared by bsdf (:199-207) and sample_bsdf (:238-246) */
static inline void lobe_probs(f3 view, f3 albedo, float roughness, float metallic, float transmission, float eta,
                              float* f0, float* rp, float* tp, float* dp)
{
    float f = (1.0f - eta) / (1.0f + eta);
    f *= f;
    *f0 = f;
    *rp = mixf_(1.0f, fresnel_att(view.z, f, eta, roughness), luminance(albedo) * (1.0f - metallic));
    *tp = (float)((1.0 - (double)*rp) * (double)transmission);
    *dp = (float)((1.0 - (double)*rp) * (double)(1.0f - transmission));
}

/* bsdf (:184-222) */
static f3 bsdf_eval(f3 light, f3 view, f3 albedo, float roughness, float metallic, float transmission, float eta,
                    float* out_pdf)
{
    f3 h;
    if(light.z > 0) h = norm3(add3(view, light));
    else h = smul3(signf_(eta - 1.0f), norm3(add3(light, smul3(eta, view))));
    float distribution = tr_distribution(h.z, roughness);
    float f0, rp, tp, dp;
    lobe_probs(view, albedo, roughness, metallic, transmission, eta, &f0, &rp, &tp, &dp);
    float r, d, t;
    f3 att = bsdf_core(light, h, view, albedo, roughness, metallic, transmission, eta, f0,
                       roughness < 1e-3f ? 0.0f : distribution, &r, &d, &t);
    *out_pdf = r * rp + d * dp + t * tp;
    return att;
}

/* sample_bsdf (:224-296) */
static void bsdf_sample(f3 u, f3 view, f3 albedo, float roughness, float metallic, float transmission, float eta,
                        f3* out_dir, f3* out_att, float* out_pdf)
{
    f2 uxy = {u.x, u.y};
    f3 h = ggx_vndf(view, roughness, uxy);
    float f0, rp, tp, dp;
    lobe_probs(view, albedo, roughness, metallic, transmission, eta, &f0, &rp, &tp, &dp);
    int diffuse = 0, bad;
    if((u.z -= rp) <= 0) { *out_dir = reflect3(neg3(view), h); bad = out_dir->z <= 0; }
    else if((u.z -= tp) <= 0) { *out_dir = refract3(neg3(view), h, eta); bad = out_dir->z >= 0; }
    else
    {
        *out_dir = cosine_hemisphere(uxy);
        h = norm3(add3(*out_dir, view));
        diffuse = 1;
        bad = out_dir->z == 0;
    }
    if(bad)
    {
        *out_dir = V3(0, 0, 1);
        *out_att = V3(0, 0, 0);
        *out_pdf = 1;
        return;
    }
    float distribution = tr_distribution(h.z, roughness);
    if(roughness < 1e-3f) distribution = diffuse ? 0 : (float)fabs((double)(4.0f * out_dir->z * view.z));
    float r, d, t;
    *out_att = bsdf_core(*out_dir, h, view, albedo, roughness, metallic, transmission, eta, f0, distribution, &r, &d, &t);
    *out_pdf = r * rp + t * tp;
    if(roughness < 1e-3f && !diffuse) *out_pdf = -*out_pdf;
    else *out_pdf += d * dp;
}

/* trace_ray (:340-412) */
static hit_info trace_ray(const pt_ctx* c, f3 origin, f3 dir, float tmin)
{
    rq_state q;
    rq_init(&q, c->s, c->tlas, origin, dir, tmin, 1e9f, c->cnt);
    while(rq_proceed(&q)) rq_confirm(&q);
    hit_info hi;
    memset(&hi, 0, sizeof(hi));
    hi.thit = q.closest.thit;
    hi.nee_pdf = 0;
    if(hi.thit < 0)
    {   /* sky: only the sun disk is explicit (the sky itself is the atmosphere pass) */
        float visible = dot3(c->light_dir, dir) > c->light_cos;
        hi.nee_pdf = visible / (2.0f * PI_F * (1.0f - c->light_cos));
        float w = hi.nee_pdf == 0.0f ? 1.0f : hi.nee_pdf;
        hi.albedo = add3(V3(0.0f, 0.0f, 0.0f), mul3s(smul3(visible, c->light_color), w));
        hi.emission = 1.0f;
        return hi;
    }
    if(c->cnt) c->cnt[5]++;
    const orc_scene* s = c->s;
    const rinstance* in = (const rinstance*)s->instances + q.closest.instance_id;
    hi.pos = add3(origin, mul3s(dir, q.closest.thit));
    m3 rot = {{rf3v(*(const rf3*)&in->transform[0]), rf3v(*(const rf3*)&in->transform[1]), rf3v(*(const rf3*)&in->transform[2])}};
    uint32_t tri = in->m.index_offset + q.closest.primitive_id * 3;
    uint32_t bv = in->m.base_vertex_offset;
    uint32_t i0 = s->indices[tri], i1 = s->indices[tri + 1], i2 = s->indices[tri + 2];
    f3 n0 = ld3(s->normal, bv + i0), n1 = ld3(s->normal, bv + i1), n2 = ld3(s->normal, bv + i2);
    f4 a0 = ld4(s->albedo, bv + i0), a1 = ld4(s->albedo, bv + i1), a2 = ld4(s->albedo, bv + i2);
    f4 m0 = ld4(s->material, bv + i0), m1 = ld4(s->material, bv + i1), m2 = ld4(s->material, bv + i2);
    f3 b = q.closest.bary;
    f4 alb = {a0.x * b.x + a1.x * b.y + a2.x * b.z, a0.y * b.x + a1.y * b.y + a2.y * b.z,
              a0.z * b.x + a1.z * b.y + a2.z * b.z, a0.w * b.x + a1.w * b.y + a2.w * b.z};
    f4 mat = {m0.x * b.x + m1.x * b.y + m2.x * b.z, m0.y * b.x + m1.y * b.y + m2.y * b.z,
              m0.z * b.x + m1.z * b.y + m2.z * b.z, m0.w * b.x + m1.w * b.y + m2.w * b.z};
    f3 n = add3(add3(mul3s(n0, b.x), mul3s(n1, b.y)), mul3s(n2, b.z));
    n = norm3(mul_m3v3(&rot, n));
    const float ior = 1.5f;
    if(q.closest.back_face) { hi.eta = ior; n = neg3(n); }
    else hi.eta = 1.0f / ior;
    hi.tbn = tangent_space(n);
    hi.albedo = V3(alb.x, alb.y, alb.z);
    hi.alpha = alb.w;
    hi.roughness = mat.x * mat.x;
    hi.metallic = mat.y;
    hi.transmission = mat.z;
    hi.emission = mat.w;
    return hi;
}

/* trace_shadow_ray (:415-427): any hit */
static int trace_shadow(const pt_ctx* c, f3 o, f3 d, float tmin, float tmax)
{
    rq_state q;
    rq_init(&q, c->s, c->tlas, o, d, tmin, tmax, c->cnt);
    return rq_proceed(&q);
}

/* get_camera_ray (:429-450) */
static void camera_ray(const rcamera* cam, const orc_config* cfg, f2 u, f2 coord, f3* dir, f3* origin)
{
    f2 uv = {coord.x / (float)cfg->width * 2.0f - 1.0f, coord.y / (float)cfg->height * 2.0f - 1.0f};
    uv.x *= cam->aspect_ratio;
    uv.y = -uv.y;
    f2 ap = {0, 0};
    if(cam->aperture_polygon > 3)
    {
        f2 p = regular_polygon(u, cam->aperture_angle, (uint32_t)cam->aperture_polygon);
        ap.x = p.x * cam->aperture_radius;
        ap.y = p.y * cam->aperture_radius;
    }
    *origin = V3(ap.x, ap.y, 0.0f);
    f3 d = mul3s(V3(uv.x * cam->inv_focal_length, uv.y * cam->inv_focal_length, -1), cam->focal_distance);
    d = norm3(sub3(d, *origin));
    m3 o = {{rf3v(cam->orientation[0]), rf3v(cam->orientation[1]), rf3v(cam->orientation[2])}};
    *dir = mul_m3v3(&o, d);
    *origin = add3(mul_m3v3(&o, *origin), rf3v(cam->position));
}

static const f3 RAYLEIGH = {5.8e-6f, 13.6e-6f, 33.1e-6f};   /* config.hh:38 */
static const f3 MIE = {4.0e-6f, 4.0e-6f, 4.0e-6f};         /* config.hh:40 */

/* nishita_atmosphere_attenuation (:456-497) */
static f3 atmosphere_attenuation(float jitter, int iterations, f3 pos, f3 view, float tmax)
{
    const f3 earth = V3(0, -EARTH_RADIUS, 0);
    f3 att = V3(1.0f, 1.0f, 1.0f);
    float tmin = 0, atmax = 0;
    int hit = ray_sphere(pos, view, earth, EARTH_RADIUS + ATMOSPHERE_HEIGHT, &tmin, &atmax);
    if(!hit) return att;
    tmin = (float)fmax((double)tmin, 0.0);
    tmax = fminf(atmax, tmax < 0 ? MAX_RAY_DIST : tmax);
    float segment = (tmax - tmin) / (float)iterations;
    float ray_depth = 0, mie_depth = 0;
    int shadowed = 0;
    for(int i = 0; i < iterations; ++i)
    {
        float t = segment * (jitter + (float)i);
        float height = len3(sub3(add3(pos, smul3(t, view)), earth)) - EARTH_RADIUS;
        ray_depth = (float)((double)ray_depth + exp((double)(-height / RAYLEIGH_SCALE_HEIGHT)));
        mie_depth = (float)((double)mie_depth + exp((double)(-height / MIE_SCALE_HEIGHT)));
        if(height < 0) shadowed = 1;
    }
    f3 tau = mul3s(add3(mul3s(RAYLEIGH, ray_depth), mul3s(MIE, mie_depth)), segment);
    att.x = (float)exp((double)-tau.x);
    att.y = (float)exp((double)-tau.y);
    att.z = (float)exp((double)-tau.z);
    if(shadowed) att = V3(0.0f, 0.0f, 0.0f);
    return att;
}

/* nishita_atmosphere_scattering (:499-588) */
static void atmosphere_scattering(u4* seed, const pt_ctx* c, f3 pos, f3 view, float tmax, f3* attenuation, f3* in_scatter)
{
    const f3 earth = V3(0, -EARTH_RADIUS, 0);
    *attenuation = V3(1.0f, 1.0f, 1.0f);
    *in_scatter = V3(0.0f, 0.0f, 0.0f);
    if(tmax > 0 && tmax < 1e3f) return;
    float tmin = 0, atmax = 0;
    int hit = ray_sphere(pos, view, earth, EARTH_RADIUS + ATMOSPHERE_HEIGHT, &tmin, &atmax);
    if(!hit) return;
    tmin = (float)fmax((double)tmin, 0.0);
    tmax = fminf(atmax, tmax < 0 ? MAX_RAY_DIST : tmax);
    float segment = (tmax - tmin) / (float)PRIMARY_ITERATIONS;
    f4 jitter = uniform4(seed);
    float mu = dot3(view, c->light_dir);
    float rayleigh_phase = 3.0f / (16.0f * PI_F) * (1.0f + mu * mu);
    const float g = MIE_ANISOTROPY;
    float mie_phase = (float)((double)(3.0f / (8.0f * PI_F) * (1.0f - g * g) * (1.0f + mu * mu)) /
                              ((double)(2.0f + g * g) * pow((double)(1.0f + g * g - 2.0f * g * mu), 1.5)));
    float ray_depth = 0, mie_depth = 0;
    f3 ray_sum = V3(0, 0, 0), mie_sum = V3(0, 0, 0);
    for(int i = 0; i < PRIMARY_ITERATIONS; ++i)
    {
        float t = segment * (jitter.x + (float)i);
        f3 p = add3(pos, smul3(t, view));
        ray_sphere(p, c->light_dir, earth, EARTH_RADIUS + ATMOSPHERE_HEIGHT, &tmin, &tmax);   /* keeps old values on a miss */
        float light_segment = (tmax - tmin) / (float)SECONDARY_ITERATIONS;
        float lray = 0, lmie = 0;
        int shadowed = 0;
        for(int j = 0; j < SECONDARY_ITERATIONS; ++j)
        {
            float tt = light_segment * (jitter.y + (float)j);
            float height = len3(sub3(add3(p, smul3(tt, c->light_dir)), earth)) - EARTH_RADIUS;
            lray = (float)((double)lray + exp((double)(-height / RAYLEIGH_SCALE_HEIGHT)));
            lmie = (float)((double)lmie + exp((double)(-height / MIE_SCALE_HEIGHT)));
            if(height < 0) shadowed = 1;
        }
        float height = fmaxf(len3(sub3(p, earth)) - EARTH_RADIUS, 0.0f);
        float ray_density = (float)(exp((double)(-height / RAYLEIGH_SCALE_HEIGHT)) * (double)segment);
        float mie_density = (float)(exp((double)(-height / MIE_SCALE_HEIGHT)) * (double)segment);
        ray_depth += ray_density;
        mie_depth += mie_density;
        float kr = lray * light_segment + ray_depth, km = lmie * light_segment + mie_depth;
        f3 tau = add3(mul3s(RAYLEIGH, kr), mul3s(MIE, km));
        f3 local = V3((float)exp((double)-tau.x), (float)exp((double)-tau.y), (float)exp((double)-tau.z));
        if(shadowed) local = V3(0.0f, 0.0f, 0.0f);
        ray_sum = add3(ray_sum, mul3s(local, ray_density));
        mie_sum = add3(mie_sum, mul3s(local, mie_density));
    }
    f3 tau = add3(mul3s(RAYLEIGH, ray_depth), mul3s(MIE, mie_depth));
    attenuation->x = (float)exp((double)-tau.x);
    attenuation->y = (float)exp((double)-tau.y);
    attenuation->z = (float)exp((double)-tau.z);
    *in_scatter = mul3s(mul3(add3(mul3s(mul3(ray_sum, RAYLEIGH), rayleigh_phase), mul3s(mul3(mie_sum, MIE), mie_phase)),
                             c->light_color), 4.0f);
}

/* nee_branch (:594-620) */
static f3 nee_branch(u4* seed, const pt_ctx* c, const hit_info* info, f3 tview)
{
    f4 u = uniform4(seed);
    f2 uxy = {u.x, u.y};
    f3 light_dir = sample_cone(c->light_dir, c->light_cos, uxy);
    float nee_pdf = 1.0f / (2.0f * PI_F * (1.0f - c->light_cos));
    float bsdf_pdf = 0;
    f3 b = bsdf_eval(mul_v3m3(light_dir, &info->tbn), tview, info->albedo, info->roughness, info->metallic,
                     info->transmission, info->eta, &bsdf_pdf);
    f3 color = mul3(mul3s(b, nee_pdf), c->light_color);
    if((color.x == 0 && color.y == 0 && color.z == 0) || trace_shadow(c, info->pos, light_dir, MIN_RAY_DIST, MAX_RAY_DIST))
        return V3(0, 0, 0);
    float mis_pdf = 1.0f;
    if(c->light_cos < 1.0f) mis_pdf = (nee_pdf * nee_pdf + bsdf_pdf * bsdf_pdf) / nee_pdf;
    color = mul3(color, atmosphere_attenuation(u.w, PRIMARY_ITERATIONS, info->pos, light_dir, MAX_RAY_DIST));
    return div3s(color, mis_pdf);
}

/* path_trace_pixel (:637-741) */
void orc_path_trace_pixel(const orc_scene* s, const orc_config* cfg, uint32_t x, uint32_t y, int32_t sample_index,
                          float out[4], uint64_t* counters)
{
    uint32_t sub = sample_index < 0 ? 0 : (uint32_t)sample_index / cfg->samples_per_motion_blur_step;
    const rsubframe* sf = (const rsubframe*)s->subframes + sub;
    u4 seed = {x, y, (uint32_t)sample_index, cfg->student_id};
    pcg4d(&seed);
    f4 u = uniform4(&seed);
    f2 uxy = {u.x, u.y}, uzw = {u.z, u.w};
    f2 film = gaussian_disk(uxy, 0.4f);
    film.x = film.x + 0.5f;
    film.y = film.y + 0.5f;
    f2 coord = {(float)x + film.x, (float)y + film.y};
    f3 ray_dir, ray_o;
    camera_ray(&sf->cam, cfg, uzw, coord, &ray_dir, &ray_o);

    pt_ctx c;
    c.s = s;
    c.tlas = sf->tlas;
    c.light_dir = rf3v(sf->light.direction);
    c.light_color = rf3v(sf->light.color);
    c.light_cos = sf->light.cos_solid_angle;
    c.cnt = counters;
    if(counters) counters[0]++;

    hit_info info = trace_ray(&c, ray_o, ray_dir, 0.0f);
    f3 attenuation = V3(1, 1, 1);
    f3 contribution = V3(0, 0, 0);
    f3 in_scatter;
    atmosphere_scattering(&seed, &c, ray_o, ray_dir, info.thit, &attenuation, &in_scatter);
    contribution = add3(contribution, add3(in_scatter, mul3s(mul3(attenuation, info.albedo), info.emission)));

    float regularization = 1.0f;
    for(uint32_t bounce = 0; bounce < cfg->max_bounces && info.thit > 0; ++bounce)
    {
        f3 view = mul_v3m3(neg3(ray_dir), &info.tbn);
        if(view.z < 1e-7f) view.z = fmaxf(view.z, 1e-7f);
        view = norm3(view);

        contribution = add3(contribution, mul3(attenuation, nee_branch(&seed, &c, &info, view)));

        f4 ub = uniform4(&seed);
        f3 tdir, batt;
        float bpdf;
        bsdf_sample(V3(ub.x, ub.y, ub.z), view, info.albedo, info.roughness, info.metallic, info.transmission,
                    info.eta, &tdir, &batt, &bpdf);
        ray_dir = norm3(mul_m3v3(&info.tbn, tdir));
        ray_o = info.pos;
        info = trace_ray(&c, ray_o, ray_dir, MIN_RAY_DIST);

        float mis_pdf = bpdf < 0 ? -bpdf : (info.nee_pdf * info.nee_pdf + bpdf * bpdf) / bpdf;
        attenuation = mul3(attenuation, batt);
        f3 aatt, insc;
        atmosphere_scattering(&seed, &c, ray_o, ray_dir, info.thit, &aatt, &insc);
        f3 term = mul3(attenuation, add3(insc, mul3s(mul3(aatt, info.albedo), info.emission)));
        contribution = add3(contribution, div3s(term, mis_pdf));
        attenuation = mul3(attenuation, div3s(aatt, (float)fabs((double)bpdf)));
        if(bpdf > 0.0f)
            regularization = (float)((double)regularization *
                                     fmax(1 - (double)REGULARIZATION_GAMMA / pow((double)bpdf, 0.25), 0.0));
        info.roughness = 1.0f - (1.0f - info.roughness) * regularization;
    }
    out[0] = contribution.x;
    out[1] = contribution.y;
    out[2] = contribution.z;
    out[3] = 0.0f;
}

/* tonemap_pixel (:753-771) */
static inline float srgb(float c)
{
    return c < 0.0031308f ? c * 12.92f : (float)(pow((double)c, (double)(1.0f / 2.4f)) * (double)1.055f - (double)0.055f);
}
static inline float aces(float c) { return (c * (2.51f * c + 0.03f)) / (c * (2.43f * c + 0.59f) + 0.14f); }

void orc_tonemap_pixel(const float color[3], uint8_t out[4])
{
    float r = clampf_(srgb(aces(color[0])), 0.0f, 1.0f);
    float g = clampf_(srgb(aces(color[1])), 0.0f, 1.0f);
    float b = clampf_(srgb(aces(color[2])), 0.0f, 1.0f);
    out[0] = (uint8_t)round((double)(b * 255.0f));
    out[1] = (uint8_t)round((double)(g * 255.0f));
    out[2] = (uint8_t)round((double)(r * 255.0f));
    out[3] = 255;
}

void orc_pcg4d(uint32_t seed[4])
{
    u4 s = {seed[0], seed[1], seed[2], seed[3]};
    pcg4d(&s);
    seed[0] = s.x; seed[1] = s.y; seed[2] = s.z; seed[3] = s.w;
}

void orc_uniform4(uint32_t seed[4], float out[4])
{
    u4 s = {seed[0], seed[1], seed[2], seed[3]};
    f4 u = uniform4(&s);
    seed[0] = s.x; seed[1] = s.y; seed[2] = s.z; seed[3] = s.w;
    out[0] = u.x; out[1] = u.y; out[2] = u.z; out[3] = u.w;
}

void orc_trace_ray(const orc_scene* s, uint32_t subframe, const float ray[8], uint32_t out[8])
{
    const rsubframe* sf = (const rsubframe*)s->subframes + subframe;
    f3 o = V3(ray[0], ray[1], ray[2]), d = V3(ray[3], ray[4], ray[5]);
    rq_state q;
    rq_init(&q, s, sf->tlas, o, d, ray[6], ray[7], 0);
    while(rq_proceed(&q)) rq_confirm(&q);
    rq_state sq;
    rq_init(&sq, s, sf->tlas, o, d, ray[6], ray[7], 0);
    int shadow = rq_proceed(&sq);
    memcpy(&out[0], &q.closest.bary.x, 4);
    memcpy(&out[1], &q.closest.bary.y, 4);
    memcpy(&out[2], &q.closest.bary.z, 4);
    memcpy(&out[3], &q.closest.thit, 4);
    out[4] = q.closest.instance_id;
    out[5] = q.closest.primitive_id;
    out[6] = q.closest.back_face ? 1u : 0u;
    out[7] = shadow ? 1u : 0u;
}

/* baseline_render (main.cc:12-46): j-ordered float sum, / SPP, tonemap */
void orc_render_rect(const orc_scene* s, const orc_config* c, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                     uint32_t j0, uint32_t j1, float* accum, uint8_t* bgra, uint64_t* counters)
{
    for(uint32_t r = 0; r < h; ++r)
        for(uint32_t q = 0; q < w; ++q)
        {
            float acc[3] = {0, 0, 0};
            for(uint32_t j = j0; j < j1; ++j)
            {
                float v[4];
                orc_path_trace_pixel(s, c, x0 + q, y0 + r, (int32_t)j, v, counters);
                acc[0] += v[0];
                acc[1] += v[1];
                acc[2] += v[2];
            }
            const float n = (float)c->samples_per_pixel;
            acc[0] /= n; acc[1] /= n; acc[2] /= n;
            size_t i = (size_t)r * w + q;
            if(accum) { accum[i * 4 + 0] = acc[0]; accum[i * 4 + 1] = acc[1]; accum[i * 4 + 2] = acc[2]; accum[i * 4 + 3] = 0; }
            if(bgra) orc_tonemap_pixel(acc, bgra + i * 4);
        }
}
