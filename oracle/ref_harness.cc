// Driver for the UNMODIFIED reference renderer, compiled from
// /root/reference in place (see oracle/Makefile).  Test-oracle infrastructure
// only: tests/ and bench.py's cpu_baseline leg execute the binaries built from
// this file; the product never links or calls them.
//
// Every command runs the reference's own code: load_scene (scene.cc:135),
// setup_animation_frame (scene.cc:271), path_trace_pixel / tonemap_pixel
// (path_tracer.hh:637 / :753), the ray_query API (ray_query.hh:111-290),
// pcg4d (math.hh:466) and baseline_render itself (main.cc:12-46; main.cc is
// compiled with its main() renamed away, see Makefile).
//
// usage: ref_pt <assets_dir> <command> ...
//   dump     <frame> <outdir>                        scene arrays as raw files
//   samples  <frame> <x0> <y0> <w> <h> <j0> <j1> <out.f32>
//                                                    path_trace_pixel outputs, [y][x][j][4]
//   render   <frame> <out_prefix>                    baseline_render semantics over the
//                                                    whole image: <p>.f32 radiance (after /SPP,
//                                                    [H][W][4]) and <p>.bgra
//   baseline <frame> <out.bgra>                      calls main.cc's baseline_render itself and
//                                                    prints one JSON line with its wall time
//   rays     <frame> <subframe> <in.f32> <out.bin>   closest-hit + any-hit per ray
//                                                    in: N x 8 floats (o.xyz, d.xyz, tmin, tmax)
//                                                    out: N x 8 words (bary.xyz f32, thit f32,
//                                                    instance u32, primitive u32, back u32,
//                                                    shadow u32)
//   tonemap  <in.f32> <out.bgra>                     tonemap_pixel over N x 4 floats
//   pcg      <in.u32> <out.u32>                      N x 4 seeds -> pcg4d(seed), then
//                                                    generate_uniform_random4 bits
//   anim_hashes <f0> <f1> <out.txt>                  per-frame SHA-256 of instances, subframes,
//                                                    TLAS nodes and links, frames [f0, f1)
//   anim_render <f0> <f1> <out.txt>                  per-frame SHA-256 of the whole rendered
//                                                    image (radiance bits, BGRA), frames [f0, f1)
//   spots    <in.txt> <out.bin>                      baseline_render over listed rectangles
#include "scene.hh"
#include "path_tracer.hh"
#include "bmp.hh"
#include "sha256.h"
#include <chrono>
#include <clocale>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <pthread.h>
#include <unistd.h>
#include <omp.h>

void baseline_render(const scene& s, uchar4* image);  // main.cc:12

static std::vector<char> read_all(const char* path)
{
    FILE* f = fopen(path, "rb");
    if(!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<char> buf(n);
    if(n && fread(buf.data(), 1, n, f) != (size_t)n) { fprintf(stderr, "short read %s\n", path); exit(2); }
    fclose(f);
    return buf;
}

static void write_all(const std::string& path, const void* data, size_t bytes)
{
    FILE* f = fopen(path.c_str(), "wb");
    if(!f) { fprintf(stderr, "cannot write %s\n", path.c_str()); exit(2); }
    if(bytes && fwrite(data, 1, bytes, f) != bytes) { fprintf(stderr, "short write %s\n", path.c_str()); exit(2); }
    fclose(f);
}

template<typename T>
static void write_vec(const std::string& path, const std::vector<T>& v)
{
    write_all(path, v.data(), v.size() * sizeof(T));
}

static scene load(const char* assets, uint frame)
{
    char cwd[4096];
    if(!getcwd(cwd, sizeof(cwd))) exit(2);
    if(chdir(assets) != 0) { fprintf(stderr, "cannot chdir %s\n", assets); exit(2); }
    setlocale(LC_ALL, "C");
    scene s = load_scene();
    setup_animation_frame(s, frame);
    if(chdir(cwd) != 0) exit(2);
    return s;
}

static int cmd_dump(const char* assets, int argc, char** argv)
{
    uint frame = atoi(argv[0]);
    std::string out = argv[1];
    scene s = load(assets, frame);
    write_vec(out + "/nodes.bin", s.bvh_buf.nodes);
    write_vec(out + "/links.bin", s.bvh_buf.links);
    write_vec(out + "/indices.bin", s.mesh_buf.indices);
    write_vec(out + "/pos.bin", s.mesh_buf.pos);
    write_vec(out + "/normal.bin", s.mesh_buf.normal);
    write_vec(out + "/albedo.bin", s.mesh_buf.albedo);
    write_vec(out + "/material.bin", s.mesh_buf.material);
    write_vec(out + "/instances.bin", s.instances);
    write_vec(out + "/subframes.bin", s.subframes);
    FILE* f = fopen((out + "/meta.txt").c_str(), "w");
    fprintf(f, "width %d\nheight %d\nspp %d\nbounces %d\nframe %u\n", IMAGE_WIDTH, IMAGE_HEIGHT,
            SAMPLES_PER_PIXEL, MAX_BOUNCES, frame);
    fprintf(f, "static_instance_count %u\nsubframes %zu\ninstances %zu\nnodes %zu\n",
            s.static_instance_count, s.subframes.size(), s.instances.size(), s.bvh_buf.nodes.size());
    // BLAS handles in load order (scene.cc:139-182) for cross-checks
    static const char* names[] = {"terrain", "leaf_tree", "maple_tree", "pine_tree", "tropical_tree",
        "willow_tree", "rock0", "rock1", "rock2", "rock3", "rock4", "armadillo", "buddha", "bunny",
        "dragon", "teapot", "end", "logo"};
    for(const char* n: names)
    {
        const auto& p = s.meshes.at(n);
        fprintf(f, "mesh %s %u %u %u %u %u %u\n", n, p.first.vertex_count, p.first.triangle_count,
                p.first.index_offset, p.first.base_vertex_offset, p.second.node_count, p.second.node_offset);
    }
    fclose(f);
    return 0;
}

static float3 sample_at(const scene& s, uint x, uint y, uint j)
{
    return path_trace_pixel(uint2{x, y}, j, s.subframes.data(), s.instances.data(),
        s.bvh_buf.nodes.data(), s.bvh_buf.links.data(), s.mesh_buf.indices.data(),
        s.mesh_buf.pos.data(), s.mesh_buf.normal.data(), s.mesh_buf.albedo.data(),
        s.mesh_buf.material.data());
}

static int cmd_samples(const char* assets, int argc, char** argv)
{
    uint frame = atoi(argv[0]);
    uint x0 = atoi(argv[1]), y0 = atoi(argv[2]), w = atoi(argv[3]), h = atoi(argv[4]);
    uint j0 = atoi(argv[5]), j1 = atoi(argv[6]);
    scene s = load(assets, frame);
    uint nj = j1 - j0;
    std::vector<float> out(size_t(w) * h * nj * 4);
    #pragma omp parallel for schedule(dynamic, 1)
    for(uint p = 0; p < w * h; ++p)
    {
        uint x = x0 + p % w, y = y0 + p / w;
        for(uint j = j0; j < j1; ++j)
        {
            float3 c = sample_at(s, x, y, j);
            float* o = &out[(size_t(p) * nj + (j - j0)) * 4];
            o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = 0.0f;
        }
    }
    write_vec(argv[7], out);
    return 0;
}

// baseline_render (main.cc:12-46) semantics with the accumulator on the heap
// so any resolution works; also keeps the averaged radiance.
static int cmd_render(const char* assets, int argc, char** argv)
{
    uint frame = atoi(argv[0]);
    std::string prefix = argv[1];
    scene s = load(assets, frame);
    const uint n = IMAGE_WIDTH * IMAGE_HEIGHT;
    std::vector<float3> colors(n);
    std::vector<uchar4> image(n);
    #pragma omp parallel for schedule(dynamic, 16)
    for(uint i = 0; i < n; ++i)
    {
        uint x = i % IMAGE_WIDTH, y = i / IMAGE_WIDTH;
        colors[i] = {0, 0, 0};
        for(uint j = 0; j < SAMPLES_PER_PIXEL; ++j)
            colors[i] += sample_at(s, x, y, j);
        colors[i] /= SAMPLES_PER_PIXEL;
        image[i] = tonemap_pixel(colors[i]);
    }
    write_vec(prefix + ".f32", colors);
    write_vec(prefix + ".bgra", image);
    return 0;
}

struct baseline_job { const scene* s; uchar4* image; double seconds; };

static void* baseline_thread(void* p)
{
    baseline_job* job = (baseline_job*)p;
    auto t0 = std::chrono::steady_clock::now();
    baseline_render(*job->s, job->image);
    auto t1 = std::chrono::steady_clock::now();
    job->seconds = std::chrono::duration<double>(t1 - t0).count();
    return nullptr;
}

static int cmd_baseline(const char* assets, int argc, char** argv)
{
    uint frame = atoi(argv[0]);
    auto t0 = std::chrono::steady_clock::now();
    scene s = load(assets, frame);
    auto t1 = std::chrono::steady_clock::now();
    std::vector<uchar4> image(IMAGE_WIDTH * IMAGE_HEIGHT);
    // baseline_render keeps float3 colors[W*H] on its stack (main.cc:14):
    // run it on a thread with a stack large enough for the configuration.
    baseline_job job{&s, image.data(), 0.0};
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, size_t(IMAGE_WIDTH) * IMAGE_HEIGHT * sizeof(float3) + (64u << 20));
    pthread_t th;
    if(pthread_create(&th, &attr, baseline_thread, &job) != 0) { fprintf(stderr, "pthread_create\n"); return 2; }
    pthread_join(th, nullptr);
    write_vec(argv[1], image);
    double samples = double(IMAGE_WIDTH) * IMAGE_HEIGHT * SAMPLES_PER_PIXEL;
    printf("{\"width\": %d, \"height\": %d, \"spp\": %d, \"bounces\": %d, \"frame\": %u, "
           "\"threads\": %d, \"load_scene_s\": %.3f, \"render_s\": %.6f, \"msamples_per_s\": %.6f}\n",
           IMAGE_WIDTH, IMAGE_HEIGHT, SAMPLES_PER_PIXEL, MAX_BOUNCES, frame, omp_get_max_threads(),
           std::chrono::duration<double>(t1 - t0).count(), job.seconds, samples / job.seconds * 1e-6);
    return 0;
}

static int cmd_rays(const char* assets, int argc, char** argv)
{
    uint frame = atoi(argv[0]);
    uint sub = atoi(argv[1]);
    scene s = load(assets, frame);
    std::vector<char> raw = read_all(argv[2]);
    size_t n = raw.size() / (8 * sizeof(float));
    const float* r = (const float*)raw.data();
    std::vector<uint32_t> out(n * 8);
    const subframe& sf = s.subframes[sub];
    #pragma omp parallel for schedule(dynamic, 64)
    for(size_t i = 0; i < n; ++i)
    {
        const float* q = r + i * 8;
        float3 o{q[0], q[1], q[2]}, d{q[3], q[4], q[5]};
        ray_query rq = ray_query_initialize(sf.tlas, s.instances.data(), s.bvh_buf.nodes.data(),
            s.bvh_buf.links.data(), s.mesh_buf.indices.data(), s.mesh_buf.pos.data(), o, d, q[6], q[7]);
        while(ray_query_proceed(&rq)) ray_query_confirm(&rq);
        ray_query sq = ray_query_initialize(sf.tlas, s.instances.data(), s.bvh_buf.nodes.data(),
            s.bvh_buf.links.data(), s.mesh_buf.indices.data(), s.mesh_buf.pos.data(), o, d, q[6], q[7]);
        bool shadow = ray_query_proceed(&sq);
        uint32_t* w = &out[i * 8];
        memcpy(&w[0], &rq.closest.barycentrics.x, 4);
        memcpy(&w[1], &rq.closest.barycentrics.y, 4);
        memcpy(&w[2], &rq.closest.barycentrics.z, 4);
        memcpy(&w[3], &rq.closest.thit, 4);
        w[4] = rq.closest.instance_id;
        w[5] = rq.closest.primitive_id;
        w[6] = rq.closest.back_face ? 1u : 0u;
        w[7] = shadow ? 1u : 0u;
    }
    write_vec(argv[3], out);
    return 0;
}

// ---- whole-animation pins ---------------------------------------------------
// The padding words of the reference structs are not data (never written by
// the reference): instances keep words 0-5 and 8-39 (bvh.hh:73-79), subframes
// the words make_golden.py's scene_hashes keeps (scene.hh:7-34).
static const int kInstKeep[] = {0, 1, 2, 3, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
                                26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39};
static const int kSubKeep[] = {0, 1, 4, 5, 6, 8, 9, 10, 12, 13, 14, 16, 17, 18, 20, 21, 22, 23, 24, 25,
                               28, 29, 30, 32, 33, 34, 36};

template<typename T, size_t N>
static std::string masked_hash(const std::vector<T>& v, const int (&keep)[N])
{
    static_assert(sizeof(T) == 160, "160-byte records");
    ptgref::Sha256 h;
    for(const T& r: v)
    {
        uint32_t w[40], out[N];
        memcpy(w, &r, 160);
        for(size_t k = 0; k < N; ++k) out[k] = w[keep[k]];
        h.update(out, sizeof(out));
    }
    return h.hex();
}

// anim_hashes <f0> <f1> <out.txt>: load_scene once, then for every frame
// f in [f0, f1) setup_animation_frame(s, f) (scene.cc:271-718, which pops the
// previous frame's TLASes itself) and one line
//   frame instances subframes tlas_nodes static_nodes sha(inst) sha(sub) sha(tlas nodes) sha(tlas links)
static int cmd_anim_hashes(const char* assets, int argc, char** argv)
{
    const uint f0 = atoi(argv[0]), f1 = atoi(argv[1]);
    scene s = load(assets, f0);
    const size_t stat = s.bvh_buf.nodes.size() - [&] {
        size_t n = 0;
        for(const subframe& sf: s.subframes) n += sf.tlas.node_count;
        return n;
    }();
    FILE* f = fopen(argv[2], "w");
    if(!f) { fprintf(stderr, "cannot write %s\n", argv[2]); return 2; }
    char cwd[4096];
    if(!getcwd(cwd, sizeof(cwd)) || chdir(assets) != 0) return 2;
    for(uint fr = f0; fr < f1; ++fr)
    {
        if(fr != f0) setup_animation_frame(s, fr);
        ptgref::Sha256 hn, hl;
        hn.update(s.bvh_buf.nodes.data() + stat, (s.bvh_buf.nodes.size() - stat) * sizeof(bvh_node));
        hl.update(s.bvh_buf.links.data() + 8 * stat, (s.bvh_buf.links.size() - 8 * stat) * sizeof(bvh_link));
        fprintf(f, "%u %zu %zu %zu %zu %s %s %s %s\n", fr, s.instances.size(), s.subframes.size(),
                s.bvh_buf.nodes.size() - stat, stat, masked_hash(s.instances, kInstKeep).c_str(),
                masked_hash(s.subframes, kSubKeep).c_str(), hn.hex().c_str(), hl.hex().c_str());
        fflush(f);
    }
    fclose(f);
    if(chdir(cwd) != 0) return 2;
    return 0;
}

// anim_render <f0> <f1> <out.txt>: every frame in [f0, f1) rendered whole with
// baseline_render's semantics (main.cc:16-43: j-ordered float sum, /SPP,
// tonemap_pixel); one line per frame
//   frame sha(radiance xyz f32 bits, [H][W][3]) sha(BGRA bytes, [H][W][4])
static int cmd_anim_render(const char* assets, int argc, char** argv)
{
    const uint f0 = atoi(argv[0]), f1 = atoi(argv[1]);
    scene s = load(assets, f0);
    FILE* f = fopen(argv[2], "w");
    if(!f) { fprintf(stderr, "cannot write %s\n", argv[2]); return 2; }
    char cwd[4096];
    if(!getcwd(cwd, sizeof(cwd))) return 2;
    const uint n = IMAGE_WIDTH * IMAGE_HEIGHT;
    std::vector<float> rad(size_t(n) * 3);
    std::vector<uchar4> image(n);
    for(uint fr = f0; fr < f1; ++fr)
    {
        if(fr != f0)
        {
            if(chdir(assets) != 0) return 2;
            setup_animation_frame(s, fr);
            if(chdir(cwd) != 0) return 2;
        }
        #pragma omp parallel for schedule(dynamic, 4)
        for(uint i = 0; i < n; ++i)
        {
            const uint x = i % IMAGE_WIDTH, y = i / IMAGE_WIDTH;
            float3 c = {0, 0, 0};
            for(uint j = 0; j < SAMPLES_PER_PIXEL; ++j) c += sample_at(s, x, y, j);
            c /= SAMPLES_PER_PIXEL;
            rad[size_t(i) * 3 + 0] = c.x;
            rad[size_t(i) * 3 + 1] = c.y;
            rad[size_t(i) * 3 + 2] = c.z;
            image[i] = tonemap_pixel(c);
        }
        ptgref::Sha256 hr, hb;
        hr.update(rad.data(), rad.size() * sizeof(float));
        hb.update(image.data(), image.size() * sizeof(uchar4));
        fprintf(f, "%u %s %s\n", fr, hr.hex().c_str(), hb.hex().c_str());
        fflush(f);
    }
    fclose(f);
    return 0;
}

// spots <in.txt> <out.bin>: rectangles "frame x0 y0 w h" (one per line,
// grouped by frame) rendered with baseline_render's semantics; out: per pixel
// (rectangles in input order, rows of each) radiance xyz f32 + BGRA (16 B).
// The samples of a pixel are computed in parallel and summed in j order.
static int cmd_spots(const char* assets, int argc, char** argv)
{
    FILE* in = fopen(argv[0], "r");
    if(!in) { fprintf(stderr, "cannot open %s\n", argv[0]); return 2; }
    struct Rect { uint f, x0, y0, w, h; };
    std::vector<Rect> rects;
    Rect r;
    while(fscanf(in, "%u %u %u %u %u", &r.f, &r.x0, &r.y0, &r.w, &r.h) == 5) rects.push_back(r);
    fclose(in);
    if(rects.empty()) return 2;
    scene s = load(assets, rects[0].f);
    uint cur = rects[0].f;
    char cwd[4096];
    if(!getcwd(cwd, sizeof(cwd))) return 2;
    std::vector<uint32_t> out;
    std::vector<float3> samp(SAMPLES_PER_PIXEL);
    for(const Rect& q: rects)
    {
        if(q.f != cur)
        {
            if(chdir(assets) != 0) return 2;
            setup_animation_frame(s, q.f);
            if(chdir(cwd) != 0) return 2;
            cur = q.f;
        }
        for(uint y = q.y0; y < q.y0 + q.h; ++y)
            for(uint x = q.x0; x < q.x0 + q.w; ++x)
            {
                #pragma omp parallel for schedule(dynamic, 8)
                for(uint j = 0; j < SAMPLES_PER_PIXEL; ++j) samp[j] = sample_at(s, x, y, j);
                float3 c = {0, 0, 0};
                for(uint j = 0; j < SAMPLES_PER_PIXEL; ++j) c += samp[j];
                c /= SAMPLES_PER_PIXEL;
                const uchar4 b = tonemap_pixel(c);
                uint32_t w[4];
                memcpy(&w[0], &c.x, 4);
                memcpy(&w[1], &c.y, 4);
                memcpy(&w[2], &c.z, 4);
                memcpy(&w[3], &b, 4);
                out.insert(out.end(), w, w + 4);
            }
    }
    write_vec(argv[1], out);
    return 0;
}

static int cmd_tonemap(int argc, char** argv)
{
    std::vector<char> raw = read_all(argv[0]);
    size_t n = raw.size() / 16;
    const float* c = (const float*)raw.data();
    std::vector<uchar4> out(n);
    for(size_t i = 0; i < n; ++i)
        out[i] = tonemap_pixel(float3{c[i * 4 + 0], c[i * 4 + 1], c[i * 4 + 2]});
    write_vec(argv[1], out);
    return 0;
}

static int cmd_pcg(int argc, char** argv)
{
    std::vector<char> raw = read_all(argv[0]);
    size_t n = raw.size() / 16;
    const uint* in = (const uint*)raw.data();
    std::vector<uint> out(n * 8);
    for(size_t i = 0; i < n; ++i)
    {
        uint4 s{in[i * 4 + 0], in[i * 4 + 1], in[i * 4 + 2], in[i * 4 + 3]};
        uint4 a = pcg4d(&s);
        float4 u = generate_uniform_random4(&s);
        out[i * 8 + 0] = a.x; out[i * 8 + 1] = a.y; out[i * 8 + 2] = a.z; out[i * 8 + 3] = a.w;
        memcpy(&out[i * 8 + 4], &u, 16);
    }
    write_vec(argv[1], out);
    return 0;
}

int main(int argc, char** argv)
{
    if(argc < 3) { fprintf(stderr, "usage: %s <assets_dir> <command> ...\n", argv[0]); return 2; }
    const char* assets = argv[1];
    std::string cmd = argv[2];
    int n = argc - 3;
    char** a = argv + 3;
    if(cmd == "dump" && n == 2) return cmd_dump(assets, n, a);
    if(cmd == "samples" && n == 8) return cmd_samples(assets, n, a);
    if(cmd == "render" && n == 2) return cmd_render(assets, n, a);
    if(cmd == "baseline" && n == 2) return cmd_baseline(assets, n, a);
    if(cmd == "rays" && n == 4) return cmd_rays(assets, n, a);
    if(cmd == "anim_hashes" && n == 3) return cmd_anim_hashes(assets, n, a);
    if(cmd == "anim_render" && n == 3) return cmd_anim_render(assets, n, a);
    if(cmd == "spots" && n == 2) return cmd_spots(assets, n, a);
    if(cmd == "tonemap" && n == 2) return cmd_tonemap(n, a);
    if(cmd == "pcg" && n == 2) return cmd_pcg(n, a);
    fprintf(stderr, "bad command %s\n", cmd.c_str());
    return 2;
}
