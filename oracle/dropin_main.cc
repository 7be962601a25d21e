// Drop-in proof (test infrastructure): the reference's own host code -
// load_scene / setup_animation_frame (scene.cc), the BVH builder (bvh.cc),
// the OBJ loader (mesh.cc) and write_bmp (bmp.cc), compiled unmodified from
// /root/reference by oracle/Makefile (target `dropin`) - with
// baseline_render (main.cc:12-46) replaced by the C-ABI calls shown in
// INTEGRATION.md.  tests/test_gpu_dropin.py runs the binary on the GPU box
// and compares its BMP with the reference's own render of the same frame.
//
// usage: dropin <assets_dir> <frame> <out.bmp>
#include "scene.hh"
#include "bmp.hh"
#include "ptg.h"

#include <clocale>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <unistd.h>

static ptg_context* gpu = nullptr;
static size_t static_nodes = 0;

static void ptg_check(int rc, const char* what)
{
    if(rc != PTG_OK)
    {
        fprintf(stderr, "%s: %s\n", what, ptg_last_error());
        exit(3);
    }
}

// once, after load_scene (main.cc:67)
static void gpu_upload_scene(const scene& s)
{
    ptg_check(ptg_context_create(0, &gpu), "ptg_context_create");
    static_nodes = s.bvh_buf.nodes.size();
    ptg_check(ptg_upload_scene(gpu, (const ptg_bvh_node*)s.bvh_buf.nodes.data(),
                               (const ptg_bvh_link*)s.bvh_buf.links.data(), static_nodes, s.mesh_buf.indices.data(),
                               s.mesh_buf.indices.size(), (const ptg_float3*)s.mesh_buf.pos.data(),
                               (const ptg_float3*)s.mesh_buf.normal.data(), (const ptg_float4*)s.mesh_buf.albedo.data(),
                               (const ptg_float4*)s.mesh_buf.material.data(), s.mesh_buf.pos.size()),
              "ptg_upload_scene");
}

// main.cc:12 signature, GPU body
static void baseline_render(const scene& s, uchar4* image)
{
    ptg_render_config cfg;
    ptg_render_config_default(&cfg);
    cfg.width = IMAGE_WIDTH;
    cfg.height = IMAGE_HEIGHT;
    cfg.samples_per_pixel = SAMPLES_PER_PIXEL;
    cfg.max_bounces = MAX_BOUNCES;
    const size_t frame_nodes = s.bvh_buf.nodes.size() - static_nodes;
    ptg_check(ptg_upload_frame(gpu, (const ptg_subframe*)s.subframes.data(), s.subframes.size(),
                               (const ptg_tlas_instance*)s.instances.data(), s.instances.size(),
                               (const ptg_bvh_node*)s.bvh_buf.nodes.data() + static_nodes,
                               (const ptg_bvh_link*)s.bvh_buf.links.data() + 8 * static_nodes, static_nodes,
                               frame_nodes),
              "ptg_upload_frame");
    const size_t bytes = sizeof(ptg_uchar4) * IMAGE_WIDTH * IMAGE_HEIGHT;
    void* d_image = nullptr;
    ptg_check(ptg_device_alloc(gpu, bytes, &d_image), "ptg_device_alloc");
    ptg_check(ptg_render(gpu, &cfg, 0, 0, IMAGE_WIDTH, IMAGE_HEIGHT, 0, SAMPLES_PER_PIXEL, nullptr,
                         (ptg_uchar4*)d_image),
              "ptg_render");
    ptg_check(ptg_memcpy_d2h(gpu, image, d_image, bytes), "ptg_memcpy_d2h");
    ptg_check(ptg_device_free(gpu, d_image), "ptg_device_free");
}

int main(int argc, char** argv)
{
    if(argc != 4)
    {
        fprintf(stderr, "usage: %s <assets_dir> <frame> <out.bmp>\n", argv[0]);
        return 2;
    }
    setlocale(LC_ALL, "C");
    char cwd[4096];
    if(!getcwd(cwd, sizeof cwd)) return 2;
    std::string out = argv[3];
    if(out[0] != '/') out = std::string(cwd) + "/" + out;
    if(chdir(argv[1]) != 0)   // load_scene reads data/... relative to the working directory
    {
        perror("chdir");
        return 2;
    }
    scene s = load_scene();
    gpu_upload_scene(s);
    setup_animation_frame(s, (uint)atoi(argv[2]));
    std::vector<uchar4> image(IMAGE_WIDTH * IMAGE_HEIGHT);
    baseline_render(s, image.data());
    write_bmp(out.c_str(), IMAGE_WIDTH, IMAGE_HEIGHT, 4, IMAGE_WIDTH * 4, (uint8_t*)image.data());
    ptg_context_destroy(gpu);
    return 0;
}
