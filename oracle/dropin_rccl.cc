// Multi-GPU drop-in (test infrastructure, and the C++ host route of
// INTEGRATION.md section 4): the reference's own host code - load_scene /
// setup_animation_frame (scene.cc), the BVH builder (bvh.cc), the OBJ loader
// (mesh.cc) and write_bmp (bmp.cc), compiled unmodified from /root/reference
// by oracle/Makefile (target `dropin_rccl`) - driving one frame over the
// ranks of an RCCL communicator.  It replaces the pixel-parallel loop of
// baseline_render (main.cc:16-17) and main()'s frame step (main.cc:74-101)
// with: ptg_render_tiles on each rank's interleaved tiles -> one ncclGather to
// rank 0 -> ptg_scatter_tiles (ptg_render_gather, include/ptg_rccl.h); rank 0
// writes the BMP.
//
// One process per GPU, ranks from the environment as torch.distributed.run or
// mpirun set them: RANK, WORLD_SIZE, LOCAL_RANK (defaults 0, 1, 0).  Rank 0
// creates the ncclUniqueId; with WORLD_SIZE > 1 it is handed to the other
// ranks through the file PTG_NCCL_ID_FILE (ptg_rccl_comm_init_env), so no MPI
// is needed.  No HIP or RCCL header is included here: theirs clash with the
// reference's vector types (math.hh).
//
// usage: dropin_rccl <assets_dir> <frame> <out.bmp> [tile_w tile_h]
#include "scene.hh"
#include "bmp.hh"
#include "ptg.h"
#include "ptg_rccl.h"

#include <chrono>
#include <clocale>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <unistd.h>

static void ptg_check(int rc, const char* what)
{
    if(rc != PTG_OK)
    {
        fprintf(stderr, "%s: %s\n", what, ptg_last_error());
        exit(3);
    }
}

int main(int argc, char** argv)
{
    if(argc != 4 && argc != 6)
    {
        fprintf(stderr, "usage: %s <assets_dir> <frame> <out.bmp> [tile_w tile_h]\n", argv[0]);
        return 2;
    }
    setlocale(LC_ALL, "C");
    const uint32_t tw = argc == 6 ? uint32_t(atoi(argv[4])) : 32u, th = argc == 6 ? uint32_t(atoi(argv[5])) : 16u;
    char cwd[4096];
    if(!getcwd(cwd, sizeof cwd)) return 2;
    std::string out = argv[3];
    if(out[0] != '/') out = std::string(cwd) + "/" + out;
    if(chdir(argv[1]) != 0)   // load_scene reads data/... relative to the working directory
    {
        perror("chdir");
        return 2;
    }
    // the communicator: one rank per GPU, rank layout from the environment
    struct ncclComm* comm = nullptr;
    int rank = 0, world = 1, local = 0;
    if(ptg_rccl_comm_init_env(&comm, &rank, &world, &local, 300) != PTG_OK)
    {
        fprintf(stderr, "ptg_rccl_comm_init_env: %s\n", ptg_rccl_last_error());
        return 4;
    }
    ptg_context* gpu = nullptr;
    ptg_check(ptg_context_create(local, &gpu), "ptg_context_create");

    // load_scene (main.cc:67), once per run: static arrays to HBM
    scene s = load_scene();
    const size_t static_nodes = s.bvh_buf.nodes.size();
    ptg_check(ptg_upload_scene(gpu, (const ptg_bvh_node*)s.bvh_buf.nodes.data(),
                               (const ptg_bvh_link*)s.bvh_buf.links.data(), static_nodes, s.mesh_buf.indices.data(),
                               s.mesh_buf.indices.size(), (const ptg_float3*)s.mesh_buf.pos.data(),
                               (const ptg_float3*)s.mesh_buf.normal.data(), (const ptg_float4*)s.mesh_buf.albedo.data(),
                               (const ptg_float4*)s.mesh_buf.material.data(), s.mesh_buf.pos.size()),
              "ptg_upload_scene");

    // setup_animation_frame (main.cc:82), every rank the same frame
    setup_animation_frame(s, (uint)atoi(argv[2]));
    const size_t frame_nodes = s.bvh_buf.nodes.size() - static_nodes;
    ptg_check(ptg_upload_frame(gpu, (const ptg_subframe*)s.subframes.data(), s.subframes.size(),
                               (const ptg_tlas_instance*)s.instances.data(), s.instances.size(),
                               (const ptg_bvh_node*)s.bvh_buf.nodes.data() + static_nodes,
                               (const ptg_bvh_link*)s.bvh_buf.links.data() + 8 * static_nodes, static_nodes,
                               frame_nodes),
              "ptg_upload_frame");

    // baseline_render (main.cc:88), over the ranks: tiles -> ncclGather -> rank 0
    ptg_render_config cfg;
    ptg_render_config_default(&cfg);
    cfg.width = IMAGE_WIDTH;
    cfg.height = IMAGE_HEIGHT;
    cfg.samples_per_pixel = SAMPLES_PER_PIXEL;
    cfg.max_bounces = MAX_BOUNCES;
    const size_t bytes = sizeof(ptg_uchar4) * IMAGE_WIDTH * IMAGE_HEIGHT;
    void* d_image = nullptr;
    if(rank == 0) ptg_check(ptg_device_alloc(gpu, bytes, &d_image), "ptg_device_alloc");
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = ptg_render_gather(gpu, &cfg, tw, th, comm, (ptg_uchar4*)d_image);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if(rc != PTG_OK)
    {
        fprintf(stderr, "rank %d: ptg_render_gather: %s\n", rank, ptg_rccl_last_error());
        return 5;
    }
    printf("rank %d of %d: frame %s %ux%u x%u spp in %ux%u tiles: %.1f ms (render + gather)\n", rank, world, argv[2],
           IMAGE_WIDTH, IMAGE_HEIGHT, SAMPLES_PER_PIXEL, tw, th, ms);
    if(rank == 0)
    {   // write_bmp (main.cc:97-101)
        std::vector<uchar4> image(IMAGE_WIDTH * IMAGE_HEIGHT);
        ptg_check(ptg_memcpy_d2h(gpu, image.data(), d_image, bytes), "ptg_memcpy_d2h");
        ptg_check(ptg_device_free(gpu, d_image), "ptg_device_free");
        write_bmp(out.c_str(), IMAGE_WIDTH, IMAGE_HEIGHT, 4, IMAGE_WIDTH * 4, (uint8_t*)image.data());
    }
    ptg_rccl_comm_destroy(comm);
    ptg_context_destroy(gpu);
    return 0;
}
