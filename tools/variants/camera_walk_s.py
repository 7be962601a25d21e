# variant: camera_walk112.py (camera rays in the round-0 walk, its own kernel
# capped at PTG_CAM_VGPRS x 2 registers) with the camera's constants in scalar
# registers: the refilling lanes are served one subframe at a time (waterfall
# over the distinct subframes of the refill, usually one), the subframe's
# camera record read through the constant address space (s_load), so the
# per-lane registers hold only the sample's own values.  Same operations in
# the same order as camera_ray (path_tracer.h).
import os
import runpy
import sys
os.environ.setdefault("PTG_CAM_VGPRS", "56")
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "camera_walk112.py"), run_name="__main__")
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (old, s.count(old))
    s = s.replace(old, new)


# the uniform-subframe camera ray
sub("""struct CamArgs {""", """typedef const __attribute__((address_space(4))) uint8_t* cbytes;
__device__ __forceinline__ float rc_f(cbytes p, uint32_t off) { return *reinterpret_cast<const __attribute__((address_space(4))) float*>(p + off); }
__device__ __forceinline__ uint32_t rc_u(cbytes p, uint32_t off) { return *reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(p + off); }
__device__ __forceinline__ f3 rc_f3(cbytes p, uint32_t off) { return V3(rc_f(p, off), rc_f(p, off + 4), rc_f(p, off + 8)); }
// camera_ray (path_tracer.h) for a wave-uniform subframe s0
template<class SC>
__device__ __forceinline__ void camera_ray_u(const SC& sc, uint32_t s0, uint32_t px, uint32_t py, int32_t sample_index,
                                             u4& seed, f3& ray_o, f3& ray_dir)
{
    seed = u4{px, py, (uint32_t)sample_index, sc.student_id};
    pcg4d(seed);
    const f4 u = uniform4(seed);
    f2 film = gaussian_disk(f2{u.x, u.y}, 0.4f);
    film.x = film.x + 0.5f;
    film.y = film.y + 0.5f;
    const cbytes cam = (cbytes)(sc.subframes + size_t(s0) * SF_STRIDE + SF_CAM);
    float uvx = ((float)px + film.x) / (float)sc.width * 2.0f - 1.0f;
    float uvy = ((float)py + film.y) / (float)sc.height * 2.0f - 1.0f;
    uvx *= rc_f(cam, 64);
    uvy = -uvy;
    f2 ap{0, 0};
    const int32_t polygon = (int32_t)rc_u(cam, 80);
    if(polygon > 3)
    {
        const float2* table = (sc.polygon && (uint32_t)polygon <= kPolyMaxSides) ? sc.polygon + size_t(s0) * kPolyStride
                                                                                 : nullptr;
        const f2 p = regular_polygon(f2{u.z, u.w}, rc_f(cam, 76), (uint32_t)polygon, table);
        const float rad = rc_f(cam, 84);
        ap = f2{p.x * rad, p.y * rad};
    }
    const f3 origin = V3(ap.x, ap.y, 0.0f);
    const float ifl = rc_f(cam, 68), fd = rc_f(cam, 72);
    f3 d = V3(uvx * ifl * fd, uvy * ifl * fd, -1.0f * fd);
    d = normalize(d - origin);
    const m3 ori{{rc_f3(cam, 0), rc_f3(cam, 16), rc_f3(cam, 32)}};
    ray_dir = mul_m3v3(ori, d);
    ray_o = mul_m3v3(ori, origin) + rc_f3(cam, 48);
}

struct CamArgs {""")
sub("""                                    const int32_t j = (int32_t)(cam.j0 + jj);
                                    const uint8_t* sf = subframe_of(sc, j);
                                    u4 seed;
                                    camera_ray(sc, sf, x, y, j, seed, o, d);
                                    const uint32_t sb = (uint32_t)(sf - sc.subframes) / SF_STRIDE;""",
    """                                    const int32_t j = (int32_t)(cam.j0 + jj);
                                    const uint32_t sb = (uint32_t)j / sc.blur_step;   // subframe_of (j >= 0)
                                    u4 seed;
                                    for(bool todo = true; todo;)
                                    {   // one subframe per pass, its constants in scalar registers
                                        const int l = __ffsll((long long)__ballot(true)) - 1;
                                        const uint32_t s0 = __builtin_amdgcn_readlane(sb, l);
                                        if(sb == s0)
                                        {
                                            camera_ray_u(sc, s0, x, y, j, seed, o, d);
                                            todo = false;
                                        }
                                    }""")
open(p, "w").write(s)
