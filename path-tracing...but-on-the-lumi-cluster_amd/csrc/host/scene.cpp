// Scene construction and animation - restatement of scene.cc
// (load_scene :135-269, setup_animation_frame :271-718) behind the C ABI.
//
// The output arrays (meshes, BLAS/TLAS nodes + links, instances, subframes)
// are the inputs of the accelerated hot path; they are reproduced
// bit-for-bit (tests/test_scene_parity.py checks them against the reference
// built in strict IEEE mode).  The keyframe table is data lifted from
// scene.cc:319-627 into data/animation_track.csv (tools/extract_animation.py).
#include "scene_internal.h"
#include "hmath.h"
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <sched.h>

namespace ptg {

static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }

static std::atomic<unsigned> g_host_threads{0};   // ptg_set_host_threads; 0 = automatic

unsigned host_threads()
{
    if(const unsigned n = g_host_threads.load()) return n;
    static const unsigned automatic = [] {
        unsigned cpus = std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t set;
        if(sched_getaffinity(0, sizeof(set), &set) == 0) cpus = std::max(1, CPU_COUNT(&set));
        // cgroup v2 quota "max 100000" or "<quota> <period>" (a job limited to
        // N CPUs of time runs N-ish threads at full speed, not more)
        if(FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r"))
        {
            char q[32] = {0};
            long period = 0;
            if(fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
                cpus = std::min(cpus, unsigned(std::max(1L, (atol(q) + period - 1) / period)));
            fclose(f);
        }
        // ranks of one node share the host (torch.distributed.run sets it)
        if(const char* lw = getenv("LOCAL_WORLD_SIZE"))
            if(const int ranks = atoi(lw); ranks > 1) cpus = std::max(1u, cpus / unsigned(ranks));
        return cpus;
    }();
    return automatic;
}

namespace {

using namespace hm;

const double PI = 3.14159265358979323846;   // M_PI
const float PI_F = (float)PI;
const int FRAMERATE = 30;                   // config.hh:17
const int OBJECT_COUNT = 1024;              // scene.cc:4

const char* kAnimationTrack =
#include "animation_track.inc"
;

struct GradientStop { float t; f4 value; };   // scene.cc:6-10

// get_gradient_value (scene.cc:12-22)
f4 gradient(const std::vector<GradientStop>& g, float t)
{
    auto it = std::lower_bound(g.begin(), g.end(), t, [](const GradientStop& s, float v) { return s.t < v; });
    if(it == g.begin()) return g.front().value;
    if(it == g.end()) return g.back().value;
    return mix4((it - 1)->value, it->value, (t - (it - 1)->t) / (it->t - (it - 1)->t));
}

// The animated variables of setup_animation_frame (scene.cc:282-316).
struct AnimState {
    ptg_camera cam{};
    float fov = 80.0f;
    f3 cam_orientation{};
    float logo_visible = 0, armadillo_visible = 0, dragon_visible = 0, bunny_visible = 0, end_visible = 0;
    f3 teapot_pos{}, teapot_ori{}, armadillo_pos{}, armadillo_ori{}, dragon_pos{}, dragon_ori{};
    f3 bunny_pos{}, bunny_ori{}, end_pos{}, end_ori{};
};

const f3 kCamStartPos = v3((float)-81.4, (float)65, (float)-113.6);   // scene.cc:279
const f3 kCamStartOri = v3((float)30.6, (float)146.6, (float)0);      // scene.cc:280

struct Keyframe {                    // animation_stop (scene.cc:24-31)
    float start, duration, from, to;
    size_t var;                      // offset of the animated float in AnimState
};

// C++ literal conversion rules of the table entries: "1.5f" is a float
// literal; "-90.6" a double literal narrowed to float; identifiers are the
// constants the table refers to.
float literal(const std::string& s)
{
    if(s == "camera_start_pos.x") return kCamStartPos.x;
    if(s == "camera_start_pos.y") return kCamStartPos.y;
    if(s == "camera_start_pos.z") return kCamStartPos.z;
    if(s == "camera_start_ori.x") return kCamStartOri.x;
    if(s == "camera_start_ori.y") return kCamStartOri.y;
    if(s == "camera_start_ori.z") return kCamStartOri.z;
    if(!s.empty() && (s.back() == 'f' || s.back() == 'F'))
        return strtof(s.substr(0, s.size() - 1).c_str(), nullptr);
    char* end = nullptr;
    double d = strtod(s.c_str(), &end);
    if(end == s.c_str() || *end) throw std::runtime_error("bad keyframe literal '" + s + "'");
    return (float)d;
}

size_t variable_offset(const std::string& name)
{
    static const std::map<std::string, size_t> table = {
        {"logo_visible", offsetof(AnimState, logo_visible)},
        {"armadillo_visible", offsetof(AnimState, armadillo_visible)},
        {"dragon_visible", offsetof(AnimState, dragon_visible)},
        {"bunny_visible", offsetof(AnimState, bunny_visible)},
        {"end_visible", offsetof(AnimState, end_visible)},
        {"fov", offsetof(AnimState, fov)},
        {"cam.position.x", offsetof(AnimState, cam) + offsetof(ptg_camera, position) + 0},
        {"cam.position.y", offsetof(AnimState, cam) + offsetof(ptg_camera, position) + 4},
        {"cam.position.z", offsetof(AnimState, cam) + offsetof(ptg_camera, position) + 8},
        {"cam.focal_distance", offsetof(AnimState, cam) + offsetof(ptg_camera, focal_distance)},
        {"cam.aperture_radius", offsetof(AnimState, cam) + offsetof(ptg_camera, aperture_radius)},
        {"cam_orientation.x", offsetof(AnimState, cam_orientation) + 0},
        {"cam_orientation.y", offsetof(AnimState, cam_orientation) + 4},
        {"cam_orientation.z", offsetof(AnimState, cam_orientation) + 8},
#define PTG_VEC(n) {#n ".x", offsetof(AnimState, n) + 0}, {#n ".y", offsetof(AnimState, n) + 4}, \
                   {#n ".z", offsetof(AnimState, n) + 8}
        PTG_VEC(teapot_pos), PTG_VEC(teapot_ori), PTG_VEC(armadillo_pos), PTG_VEC(armadillo_ori),
        PTG_VEC(dragon_pos), PTG_VEC(dragon_ori), PTG_VEC(bunny_pos), PTG_VEC(bunny_ori),
        PTG_VEC(end_pos), PTG_VEC(end_ori),
#undef PTG_VEC
    };
    auto it = table.find(name);
    if(it == table.end()) throw std::runtime_error("unknown animated variable '" + name + "'");
    return it->second;
}

const std::vector<Keyframe>& keyframes()
{
    static const std::vector<Keyframe> track = [] {
        std::vector<Keyframe> out;
        std::istringstream in(kAnimationTrack);
        std::string line;
        while(std::getline(in, line))
        {
            if(line.empty() || line[0] == '#') continue;
            std::string f[5];
            std::istringstream ls(line);
            for(int i = 0; i < 5; ++i)
                if(!std::getline(ls, f[i], ',')) throw std::runtime_error("bad keyframe row: " + line);
            out.push_back(Keyframe{literal(f[0]), literal(f[1]), literal(f[2]), literal(f[3]), variable_offset(f[4])});
        }
        return out;
    }();
    return track;
}

// play_animation_track (scene.cc:33-42): every keyframe that has started is
// applied in table order, later ones overriding earlier ones.
void play(AnimState& st, float t)
{
    for(const Keyframe& k: keyframes())
    {
        if(!(k.start <= t)) break;
        float lt = k.duration == 0 ? 1.0f : std::clamp((t - k.start) / k.duration, 0.0f, 1.0f);
        *(float*)((char*)&st + k.var) = mixf(k.from, k.to, lt);
    }
}

void add_instance(ptg_scene& s, const char* name, const m4& transform)       // scene.cc:51-60
{
    const auto& p = s.meshes.at(name);
    ptg_tlas_instance in{};
    in.blas = p.second;
    in.m = p.first;
    in.transform = transform;
    in.inv_transform = inverse(transform);
    s.instances.push_back(in);
}

void add_instance(ptg_scene& s, const char* name, f3 pos, f3 pyr, f3 scl = v3(1, 1, 1))   // scene.cc:62-73
{
    m4 t = scaling(scl);
    t = mul_m4m4(rotation_euler(pyr * PI_F / 180.0f), t);
    t = mul_m4m4(translation(pos), t);
    add_instance(s, name, t);
}

// terrain_trace (scene.cc:93-133)
bool terrain_trace(ptg_scene& s, const ptg_bvh& tlas, f3 origin, f3 dir, f3* hit_pos, f3* hit_normal)
{
    HostHit h = host_closest_hit(tlas, s.instances.data(), s.bvh_buf.nodes.data(), s.bvh_buf.links.data(),
                                 s.mesh_buf.indices.data(), s.mesh_buf.pos.data(), origin, dir, 0.0f, 1e9f);
    if(h.thit < 0) return false;
    const ptg_mesh m = s.instances[h.instance_id].m;
    const uint32_t* tri = &s.mesh_buf.indices[m.index_offset + size_t(h.primitive_id) * 3];
    if(s.mesh_buf.material[m.base_vertex_offset + tri[0]].z != 0) return false;   // water
    f3 n0 = s.mesh_buf.normal[m.base_vertex_offset + tri[0]];
    f3 n1 = s.mesh_buf.normal[m.base_vertex_offset + tri[1]];
    f3 n2 = s.mesh_buf.normal[m.base_vertex_offset + tri[2]];
    *hit_normal = normalize(n0 * h.bary.x + n1 * h.bary.y + n2 * h.bary.z);
    *hit_pos = origin + dir * h.thit;
    return true;
}

// The meshes of load_scene (scene.cc:139-183), in load order.
const char* const kMeshNames[] = {"terrain", "leaf_tree", "maple_tree", "pine_tree", "tropical_tree", "willow_tree",
                                  "rock0", "rock1", "rock2", "rock3", "rock4", "armadillo", "buddha", "bunny",
                                  "dragon", "teapot", "end", "logo"};

// Parse + BLAS build of every mesh on worker threads, each into buffers of
// its own, then appended in load order.  A mesh's arrays and its BVH (links
// and leaf payloads are BVH-local indices) do not depend on what was loaded
// before it, so appending with rebased offsets gives the very bytes of the
// sequential load (tests/test_scene_parity.py).
void load_meshes_parallel(ptg_scene& s, const std::string& assets)
{
    constexpr size_t kCount = sizeof(kMeshNames) / sizeof(kMeshNames[0]);
    struct Part {
        MeshBuffers mb;
        BvhBuffers bb;
        ptg_mesh m{};
        ptg_bvh b{};
        std::string error;
    };
    std::vector<Part> parts(kCount);
    const size_t threads = std::max<size_t>(1, std::min<size_t>(host_threads(), std::min<size_t>(kCount, 16)));
    std::atomic<size_t> next{0};
    auto worker = [&] {
        // biggest meshes are not first in the list; a shared counter balances them
        for(size_t i; (i = next.fetch_add(1)) < kCount;)
        {
            Part& p = parts[i];
            try
            {
                p.m = load_obj_mesh(p.mb, assets + "/data/" + kMeshNames[i] + ".obj");
                p.b = build_blas(p.m, p.mb, p.bb);
            }
            catch(const std::exception& ex)
            {
                p.error = ex.what();
            }
        }
    };
    std::vector<std::thread> pool;
    for(size_t t = 1; t < threads; ++t) pool.emplace_back(worker);
    worker();
    for(std::thread& t: pool) t.join();
    for(Part& p: parts)
        if(!p.error.empty()) throw std::runtime_error(p.error);
    for(size_t i = 0; i < kCount; ++i)
    {
        Part& p = parts[i];
        MeshBuffers& mb = s.mesh_buf;
        p.m.index_offset += uint32_t(mb.indices.size());
        p.m.base_vertex_offset += uint32_t(mb.pos.size());
        mb.indices.insert(mb.indices.end(), p.mb.indices.begin(), p.mb.indices.end());
        mb.pos.insert(mb.pos.end(), p.mb.pos.begin(), p.mb.pos.end());
        mb.normal.insert(mb.normal.end(), p.mb.normal.begin(), p.mb.normal.end());
        mb.albedo.insert(mb.albedo.end(), p.mb.albedo.begin(), p.mb.albedo.end());
        mb.material.insert(mb.material.end(), p.mb.material.begin(), p.mb.material.end());
        BvhBuffers& bb = s.bvh_buf;
        p.b.node_offset += uint32_t(bb.nodes.size());
        bb.nodes.insert(bb.nodes.end(), p.bb.nodes.begin(), p.bb.nodes.end());
        bb.links.insert(bb.links.end(), p.bb.links.begin(), p.bb.links.end());
        s.meshes[kMeshNames[i]] = {p.m, p.b};
        p = Part{};   // release the part's memory early
    }
}

void load(ptg_scene& s, const std::string& assets)
{
    load_meshes_parallel(s, assets);
    const auto terrain = s.meshes.at("terrain");
    const std::vector<GradientStop> albedo_gradient = {
        {-10, v4((float)0.25, (float)0.2, (float)0.1, 1)},
        {5, v4((float)0.2, (float)0.3, (float)0.02, 1)},
        {10, v4((float)0.2, (float)0.3, (float)0.02, 1)},
        {25, v4((float)0.3, (float)0.2, (float)0.1, 1)},
        {28, v4((float)0.95, (float)0.95, (float)0.95, 1)}};
    const std::vector<GradientStop> material_gradient = {
        {5, v4((float)1.0, 0, 0, 0)}, {25, v4((float)0.5, 0, 0, 0)}, {28, v4((float)0.2, 0, 0, 0)}};
    // height-based terrain recolouring, water excluded (scene.cc:155-163)
    for(uint32_t i = 0; i < terrain.first.vertex_count; ++i)
    {
        if(s.mesh_buf.material[i].z != 0) continue;
        float h = s.mesh_buf.pos[i].y;
        s.mesh_buf.albedo[i] = gradient(albedo_gradient, h);
        s.mesh_buf.material[i] = gradient(material_gradient, h);
    }
    add_instance(s, "terrain", v3(0, 0, 0), v3(0, 0, 0));

    // throwaway terrain-only TLAS for object placement (scene.cc:186-189)
    const ptg_tlas_instance* first = &s.instances[0];
    const uint32_t first_id = 0;
    ptg_bvh terrain_tlas = build_tlas(1, &first, &first_id, s.bvh_buf, s.bvh_buf);

    // 1024 random placements (scene.cc:191-263)
    ptg_uint4 seed{1, 2, 3, 4};
    for(int i = 0; i < OBJECT_COUNT; ++i)
    {
        f3 hit_pos, hit_normal;
        f4 u = uniform4(&seed);
        bool hit = terrain_trace(s, terrain_tlas, v3(u.x * 200 - 100, 200, u.y * 200 - 100), v3(0, -1, 0),
                                 &hit_pos, &hit_normal);
        if(!hit) continue;
        const bool tree_ok = (double)hit_normal.y > 0.7;
        const bool rock_ok = (double)hit_normal.y > 0.9;
        if(!tree_ok && !rock_ok) continue;
        const float tree_probability = 0.3f;
        int kind;
        if(rock_ok && !tree_ok) kind = 1;
        else if(!rock_ok && tree_ok) kind = 0;
        else kind = u.z < tree_probability ? 0 : 1;
        if(kind == 0)
        {
            u.z /= tree_probability;
            m4 t = rotation_euler(v3(0, (float)(2.0f * PI * u.w), 0));
            t = mul_m4m4(translation(hit_pos), t);
            if(hit_pos.y < 10) add_instance(s, "tropical_tree", t);
            else if(hit_pos.y < 20)
            {
                if((double)u.z < 0.3) add_instance(s, "maple_tree", t);
                else add_instance(s, "willow_tree", t);   // the leaf_tree branch repeats the test (dead)
            }
            else add_instance(s, "pine_tree", t);
        }
        else
        {
            u.z = (u.z - tree_probability) / (1 - tree_probability);
            m4 t = expand(create_tangent_space(hit_normal));
            std::swap(t.r[2], t.r[1]);
            t = mul_m4m4(translation(hit_pos), t);
            if(!tree_ok)
            {
                if((double)u.z < 0.6) add_instance(s, "rock3", t);
                else add_instance(s, "rock4", t);
            }
            else
            {
                if((double)u.z < 0.3) add_instance(s, "rock0", t);
                else add_instance(s, "rock2", t);           // the rock1 branch repeats the test (dead)
            }
        }
    }
    pop_bvh(s.bvh_buf, terrain_tlas);
    s.static_instance_count = uint32_t(s.instances.size());
    s.static_node_count = s.bvh_buf.nodes.size();
}

void setup_frame(ptg_scene& s, uint32_t frame_index)
{
    if(!s.subframes.empty()) pop_bvh(s.bvh_buf, s.subframes[0].tlas);
    s.instances.resize(s.static_instance_count);
    s.subframes.clear();

    AnimState st;
    st.cam.position = kCamStartPos;
    st.cam.aspect_ratio = float(s.cfg.width) / float(s.cfg.height);
    st.cam_orientation = kCamStartOri;
    st.cam.focal_distance = 2.0f;
    st.cam.aperture_angle = (float)(PI / 16.0f);
    st.cam.aperture_polygon = 6;
    st.cam.aperture_radius = 0.0f;
    ptg_directional_light light{};
    light.color = v3(4, 4, 4);
    light.cos_solid_angle = (float)std::cos(4.0f * PI / 180.0f);
    light.direction = normalize(v3(0, 1, 1));
    f3 logo_pos = kCamStartPos;
    st.teapot_pos = v3((float)40.1, (float)13.95, (float)13.611633);

    float anim_t = float(frame_index) / FRAMERATE * 30.0f;
    play(st, anim_t);

    if(st.logo_visible != 0)
    {   // scene.cc:634-642
        m4 t = rotation_euler(kCamStartOri * PI_F / 180.0f);
        logo_pos = logo_pos - v3((float)-1.3, 2, -2);
        t = mul_m4m4(translation(logo_pos), t);
        add_instance(s, "logo", t);
    }
    add_instance(s, "buddha", v3((float)-39.255131, (float)30.395447, (float)40.472446), v3(0, 0, 0));
    const uint32_t static_end = uint32_t(s.instances.size());

    const uint32_t step = s.cfg.samples_per_motion_blur_step;
    const uint32_t count = (s.cfg.samples_per_pixel + step - 1) / step;
    std::vector<std::pair<uint32_t, uint32_t>> dynamic;
    for(uint32_t i = 0; i < count; ++i)
    {
        float t = float(frame_index + float(i) / count) / FRAMERATE * 30.0f;
        play(st, t);
        uint32_t begin = uint32_t(s.instances.size());
        add_instance(s, "teapot", st.teapot_pos, st.teapot_ori);
        if(st.armadillo_visible != 0) add_instance(s, "armadillo", st.armadillo_pos, st.armadillo_ori);
        if(st.dragon_visible != 0) add_instance(s, "dragon", st.dragon_pos, st.dragon_ori);
        if(st.bunny_visible != 0) add_instance(s, "bunny", st.bunny_pos, st.bunny_ori);
        if(st.end_visible != 0) add_instance(s, "end", st.end_pos, st.end_ori);
        dynamic.push_back({begin, uint32_t(s.instances.size())});

        ptg_subframe sf{};
        sf.cam = st.cam;
        sf.cam.orientation = extract(rotation_euler(st.cam_orientation * PI_F / 180.0f));
        sf.cam.inv_focal_length = (float)std::tan(st.fov * PI / 360.0f);
        float sunset_t = t / (30.0f * 60.0f) * 1.1f - 0.05f;
        light.direction = v3(0, sinf((float)(sunset_t * PI)), cosf((float)(sunset_t * PI)));
        sf.light = light;
        s.subframes.push_back(sf);
    }

    // per-subframe TLAS over static + that subframe's dynamic instances
    // (scene.cc:698-717); built in parallel into private buffers, then
    // appended in subframe order.
    std::vector<BvhBuffers> local(count);
    auto build_one = [&](uint32_t i) {
        std::vector<const ptg_tlas_instance*> list;
        std::vector<uint32_t> ids;
        for(uint32_t k = 0; k < static_end; ++k) { list.push_back(&s.instances[k]); ids.push_back(k); }
        for(uint32_t k = dynamic[i].first; k < dynamic[i].second; ++k) { list.push_back(&s.instances[k]); ids.push_back(k); }
        s.subframes[i].tlas = build_tlas(list.size(), list.data(), ids.data(), s.bvh_buf, local[i]);
    };
    const unsigned nt = std::max(1u, std::min(std::min(count, host_threads()), 16u));
    std::vector<std::thread> pool;
    for(unsigned w = 0; w < nt; ++w)
        pool.emplace_back([&, w] { for(uint32_t i = w; i < count; i += nt) build_one(i); });
    for(auto& th: pool) th.join();
    for(uint32_t i = 0; i < count; ++i)
    {
        s.subframes[i].tlas.node_offset = uint32_t(s.bvh_buf.nodes.size());
        s.bvh_buf.nodes.insert(s.bvh_buf.nodes.end(), local[i].nodes.begin(), local[i].nodes.end());
        s.bvh_buf.links.insert(s.bvh_buf.links.end(), local[i].links.begin(), local[i].links.end());
    }
}

bool valid_cfg(const ptg_render_config* c)
{
    return c && c->width > 0 && c->height > 0 && c->samples_per_pixel > 0 && c->samples_per_motion_blur_step > 0;
}

} // namespace
} // namespace ptg

extern "C" {

void ptg_render_config_default(ptg_render_config* cfg)
{
    cfg->width = 640;
    cfg->height = 360;
    cfg->samples_per_pixel = 256;
    cfg->max_bounces = 4;
    cfg->student_id = 152121358u;
    cfg->samples_per_motion_blur_step = 8;
}

int ptg_abi_version(void) { return PTG_ABI_VERSION; }
const char* ptg_last_error(void) { return ptg::g_last_error.c_str(); }

int ptg_set_host_threads(int threads)
{
    if(threads < 0) { ptg::set_last_error("ptg_set_host_threads: negative"); return PTG_E_INVALID; }
    ptg::g_host_threads.store(unsigned(threads));
    return int(ptg::host_threads());
}

int ptg_scene_load(const char* assets_dir, const ptg_render_config* cfg, ptg_scene** out)
{
    if(!assets_dir || !out || !ptg::valid_cfg(cfg)) { ptg::set_last_error("ptg_scene_load: bad argument"); return PTG_E_INVALID; }
    *out = nullptr;
    try
    {
        std::unique_ptr<ptg_scene> s(new ptg_scene());
        s->cfg = *cfg;
        ptg::load(*s, assets_dir);
        *out = s.release();
        return PTG_OK;
    }
    catch(const std::bad_alloc&) { ptg::set_last_error("ptg_scene_load: out of memory"); return PTG_E_NOMEM; }
    catch(const std::exception& e) { ptg::set_last_error(std::string("ptg_scene_load: ") + e.what()); return PTG_E_IO; }
}

int ptg_scene_setup_frame(ptg_scene* s, uint32_t frame_index)
{
    if(!s) { ptg::set_last_error("ptg_scene_setup_frame: null scene"); return PTG_E_INVALID; }
    try { ptg::setup_frame(*s, frame_index); return PTG_OK; }
    catch(const std::bad_alloc&) { ptg::set_last_error("ptg_scene_setup_frame: out of memory"); return PTG_E_NOMEM; }
    catch(const std::exception& e) { ptg::set_last_error(std::string("ptg_scene_setup_frame: ") + e.what()); return PTG_E_INVALID; }
}

int ptg_scene_view_get(const ptg_scene* s, ptg_scene_view* v)
{
    if(!s || !v) { ptg::set_last_error("ptg_scene_view_get: bad argument"); return PTG_E_INVALID; }
    v->nodes = s->bvh_buf.nodes.data();
    v->node_count = s->bvh_buf.nodes.size();
    v->links = s->bvh_buf.links.data();
    v->static_node_count = s->static_node_count;
    v->indices = s->mesh_buf.indices.data();
    v->index_count = s->mesh_buf.indices.size();
    v->pos = s->mesh_buf.pos.data();
    v->normal = s->mesh_buf.normal.data();
    v->albedo = s->mesh_buf.albedo.data();
    v->material = s->mesh_buf.material.data();
    v->vertex_count = s->mesh_buf.pos.size();
    v->instances = s->instances.data();
    v->instance_count = s->instances.size();
    v->static_instance_count = s->static_instance_count;
    v->subframes = s->subframes.data();
    v->subframe_count = s->subframes.size();
    return PTG_OK;
}

uint32_t ptg_scene_frame_count(const ptg_scene*) { return 60 * ptg::FRAMERATE; }

int ptg_scene_mesh(const ptg_scene* s, const char* name, ptg_mesh* mesh, ptg_bvh* blas)
{
    if(!s || !name) return PTG_E_INVALID;
    auto it = s->meshes.find(name);
    if(it == s->meshes.end()) return PTG_E_INVALID;
    if(mesh) *mesh = it->second.first;
    if(blas) *blas = it->second.second;
    return PTG_OK;
}

void ptg_scene_destroy(ptg_scene* s) { delete s; }

// write_bmp (bmp.cc:7-63)
int ptg_write_bmp(const char* path, uint32_t w, uint32_t h, uint32_t stride, uint32_t pitch, const uint8_t* px)
{
    if(!path || !px) { ptg::set_last_error("ptg_write_bmp: bad argument"); return PTG_E_INVALID; }
    const uint32_t row = (w * 3 + 3) / 4 * 4;
    const uint32_t size = 54 + row * h;
    std::vector<uint8_t> file(size, 0);
    auto put32 = [&](size_t at, uint32_t v) { memcpy(&file[at], &v, 4); };
    auto put16 = [&](size_t at, uint16_t v) { memcpy(&file[at], &v, 2); };
    file[0] = 'B'; file[1] = 'M';
    put32(0x02, size);
    put32(0x0A, 54);
    put32(0x0E, 40);
    put32(0x12, w);
    put32(0x16, h);
    put16(0x1A, 1);
    put16(0x1C, 24);
    put32(0x1E, 0);
    put32(0x22, row * h);
    put32(0x26, 2835);
    put32(0x2A, 2835);
    put32(0x2E, 0);
    put32(0x32, 0);
    for(uint32_t y = 0; y < h; ++y)          // bottom-up rows, first 3 bytes of each pixel
        for(uint32_t x = 0; x < w; ++x)
            memcpy(&file[54 + size_t(y) * row + size_t(x) * 3], px + size_t(h - 1 - y) * pitch + size_t(x) * stride, 3);
    FILE* f = fopen(path, "wb");
    if(!f) { ptg::set_last_error(std::string("Failed to write ") + path); return PTG_E_IO; }
    size_t n = fwrite(file.data(), 1, size, f);
    fclose(f);
    if(n != size) { ptg::set_last_error(std::string("Failed to write ") + path); return PTG_E_IO; }
    return PTG_OK;
}

} // extern "C"
