#!/usr/bin/env python3
"""Benchmark of the hot path: path_trace_pixel -> ray_query BVH traversal ->
tonemap_pixel under baseline_render, on MI355X.

Workload (the configuration BASELINE.json's metric is quoted on, "1280x720
1024spp"; configs[1] is the same frame at 256 spp): frame 0 of the reference
animation, 1280x720, 1024 samples per pixel, MAX_BOUNCES = 4 (the shipped
TESTING preset), the reference scene (reference OBJ assets + committed substitutes for
the three missing meshes).  One step = one baseline_render of the frame on the GPU (+ the RCCL
framebuffer gather in --shard tiles mode) with the scene and the frame's
TLAS/instances/subframes already resident in HBM: `value`.  A second timed
loop runs what main.cc does per frame - setup_animation_frame (host C++) +
H2D upload of the frame data + render - issued asynchronously so the host
setup of step k+1 overlaps the render of step k (ptg_upload_frame waits for
the previous render before overwriting the frame buffers); it is reported
as "with_frame_setup" (PCIe-inclusive, never `value`).

Multi-GPU: one process per GPU (torch.distributed.run).  --shard frames
(default): rank r renders frame (frame + r) - weak scaling, no collective on
the data path (BASELINE config 4 style).  --shard tiles: one frame split into
interleaved 32x16 tiles, rank 0 gathers the BGRA tiles over RCCL and
assembles the framebuffer - strong scaling (config 3 style).

Prints ONE JSON line (rank 0) with the driver contract fields plus
"roofline" (the dominant kernel k_wf_walk<closest>: its algorithmic bytes
from the deterministic work counters / its device time from HIP events on the
launch stream, vs 8 TB/s HBM) and "cpu_baseline" (the reference's own baseline_render built
from its sources, timed on this host's cores on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PROFILES = os.path.join(ROOT, "profiles")


def pmc_traffic(kind, workload, ms_per_launch):
    """HBM-side bytes per launch of `kind` from committed rocprofv3 PMC passes
    of this same workload and code (tools/profile_gpu.sh + summarize_prof.py):
    FETCH_SIZE x 1 KiB x 2 (gfx950 correction) + WRITE_SIZE x 1 KiB.  A
    profile counts only if its kernel-trace average launch time agrees with the
    live measurement within 15% (a profile of older code or another chunking
    is not used), the newest (by profile name) when several do; None when
    none does."""
    import glob
    import re

    def natural(path):   # r01_wavefront11 after r01_wavefront9
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", path)]
    best = None
    for f in sorted(glob.glob(os.path.join(PROFILES, "*", "pmc_summary.json")), key=natural):
        try:
            with open(f) as fh:
                prof = json.load(fh)
            ent = prof[kind]
            if prof.get("_workload") != workload or "hbm_side_bytes" not in ent["derived"]:
                continue
            if abs(ent["trace_avg_ms"] - ms_per_launch) > 0.15 * ms_per_launch:
                continue
            best = (int(ent["derived"]["hbm_side_bytes"]), os.path.relpath(f, ROOT))   # the newest that qualifies
        except (OSError, KeyError, ValueError, TypeError):
            continue
    return best if best else (None, None)


def algorithmic_bytes(c):
    """B = 32 N_node + 60 N_tri + 88 N_enter + 156 N_hit + 160 per sample.

    32 B TravRec per node visit (24 B box + 8 B link in the reference layout),
    60 B per triangle test (3 x u32 index + 3 x 16 B position), 88 B per BLAS
    entry (blas + mesh + inv_transform), 156 B per closest-hit shade (3 x u32 +
    9 x 16 B vertex attributes), 160 B subframe per sample."""
    samples, visits, tris, enters, queries, shades = [int(x) for x in c[:6]]
    return 32 * visits + 60 * tris + 88 * enters + 156 * shades + 160 * samples


def extend_bytes(c):
    """Algorithmic bytes of the closest-hit walk kernel: per node visit one 32 B
    TravRec, per triangle test 60 B (3 x u32 + 3 x 16 B in reference layout),
    per BLAS entry 88 B, plus per ray 48 B of ray state in and 32 B of hit out."""
    visits, tris, enters, queries = int(c[1]), int(c[2]), int(c[3]), int(c[4])
    return 32 * visits + 60 * tris + 88 * enters + 80 * queries


def cpu_baseline(assets, frame):
    """Reference baseline_render (main.cc:12) on this host, bounded sample."""
    from oracle import Reference
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    ref = Reference("v3", 1280, 720, 16, 4)
    if not ref.available():
        return {"value": None, "unit": "Msamples/s", "cores": threads, "kind": "reference",
                "sample": "unavailable: %s not built" % ref.exe}
    r = ref.baseline(assets, frame, threads=threads, timeout=900)
    return {"value": round(r["msamples_per_s"], 4), "unit": "Msamples/s", "cores": r["threads"], "kind": "reference",
            "sample": "frame %d, 1280x720 x 16 spp (%.1f M samples, full frame) through the reference's own "
                      "baseline_render (main.cc:12-46, OpenMP static schedule) built from /root/reference sources "
                      "with the reference flags (-O3 -ffast-math, -march=x86-64-v3); render %.2f s"
                      % (frame, 1280 * 720 * 16 / 1e6, r["render_s"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frame", type=int, default=0)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--shard", choices=["frames", "tiles"], default="frames")
    ap.add_argument("--tile", type=str, default="32x16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--config", type=int, default=None, choices=[1, 2, 3, 4],
                    help="BASELINE.json configs[i] preset: 1 = 1280x720x256 frame 0; 2 = 1280x720x1024 frame 0 "
                         "in pixel tiles (the metric config; tiles over the ranks); 3 = the animation at 1024 spp "
                         "(frames/min over --animation K frames, default 30); 4 = 3840x2160x4096 frame 690 "
                         "(dragon + buddha in view) in pixel tiles")
    ap.add_argument("--no-frame-setup", action="store_true",
                    help="skip the second (PCIe-inclusive, per-frame host setup) timing loop")
    ap.add_argument("--animation", type=int, default=0, metavar="K",
                    help="also render K frames spread evenly over the whole animation (frame-parallel over the "
                         "ranks) and report frames/min for the full animation (BASELINE config 4)")
    args = ap.parse_args()
    if args.config == 1:
        args.width, args.height, args.spp, args.frame = 1280, 720, 256, 0
    elif args.config == 2:
        args.width, args.height, args.spp, args.frame, args.shard = 1280, 720, 1024, 0, "tiles"
    elif args.config == 3:
        args.width, args.height, args.spp = 1280, 720, 1024
        args.animation = args.animation or 30
    elif args.config == 4:
        args.width, args.height, args.spp, args.frame, args.shard = 3840, 2160, 4096, 690, "tiles"

    import numpy as np
    import torch
    import torch.distributed as dist
    import ptlumi_loader  # noqa: F401
    from ptlumi import native as N
    from ptlumi.renderer import GpuRenderer
    from ptlumi import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    # PTG_BENCH_REHEARSE=1: rehearse the N>1 code paths with more ranks than GPUs
    # (ranks share devices, gloo instead of RCCL, which cannot put two ranks on
    # one GPU); never used for a measurement
    rehearse = os.environ.get("PTG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    assets = os.path.join(ROOT, "assets")
    cfg = N.RenderConfig.make(args.width, args.height, args.spp, args.bounces)
    scene = N.Scene(assets, cfg)
    r = GpuRenderer(local)
    stream = torch.cuda.current_stream(local)
    r.set_stream(stream)
    tw, th = [int(v) for v in args.tile.split("x")]
    frame = args.frame + (rank if args.shard == "frames" else 0)

    # static scene once (load_scene output) - resident in HBM before timing
    scene.setup_frame(frame)
    r.upload(scene, include_static=True)
    dev = torch.device("cuda", local)
    image = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device=dev)
    shard = D.TileShard(cfg, tw, th, rank, world) if args.shard == "tiles" else None

    def render_step():
        if shard is None:
            r.render(cfg, out_bgra=image)
        else:
            D.render_and_gather(r, cfg, shard, image, stream=stream)

    def frame_step():
        scene.setup_frame(frame)                     # setup_animation_frame (host)
        r.upload(scene, include_static=False)        # per-frame TLAS/instances/subframes over PCIe
        render_step()

    long_steps = cfg.width * cfg.height * cfg.samples_per_pixel > 4e9

    def timed(fn, timing):
        """K steps of fn between barrier + synchronize on both sides; max over ranks."""
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(local)
        r.enable_timing(timing)
        t0 = time.perf_counter()
        for k in range(args.steps):
            fn()    # asynchronous: host work of step k+1 overlaps the kernels of step k
            if long_steps:   # progress for multi-minute configurations (completes step k-1 first)
                print("step %d/%d issued at %.1f s" % (k + 1, args.steps, time.perf_counter() - t0),
                      file=sys.stderr, flush=True)
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(local)
        el = time.perf_counter() - t0
        kt = r.kernel_times() if timing else {}
        r.enable_timing(False)
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device="cpu" if rehearse else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, kt

    # (1) the metric: render steps over a frame whose inputs are resident in HBM
    elapsed, kt = timed(render_step, True)
    # per-kernel device times of the K timed steps (HIP events recorded on the launch stream)
    step_kernel_ms = {k: v[0] for k, v in kt.items() if v[1]}
    step_kernel_n = {k: v[1] for k, v in kt.items() if v[1]}
    # (2) the reference's per-frame loop: host setup_animation_frame + PCIe upload + render
    elapsed_frame = None if args.no_frame_setup else timed(frame_step, False)[0]

    anim = None
    if args.animation > 0:
        # BASELINE config 4: the animation frame-parallel over the ranks, one frame
        # per GPU at a time; K frames spread evenly over all 1800 (frame cost varies ~7x)
        total_frames = scene.frame_count()
        picks = [round(i * total_frames / args.animation) % total_frames for i in range(args.animation)]
        mine = picks[rank::world]
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(len(mine) + 1)]
        marks[0].record(stream)
        for k, f in enumerate(mine):
            scene.setup_frame(f)
            r.upload(scene, include_static=False)
            r.render(cfg, out_bgra=image)
            marks[k + 1].record(stream)
        torch.cuda.synchronize(local)
        per_frame = sorted(((marks[k].elapsed_time(marks[k + 1]), f) for k, f in enumerate(mine)), reverse=True)
        if world > 1:
            dist.barrier()
        anim_s = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([anim_s], dtype=torch.float64, device="cpu" if rehearse else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            anim_s = float(t.item())
        anim = {"frames_per_min": round(len(picks) / anim_s * 60.0, 3),
                "full_animation_min": round(total_frames / (len(picks) / anim_s * 60.0), 2),
                "msamples_per_s": round(len(picks) * cfg.width * cfg.height * cfg.samples_per_pixel / anim_s / 1e6, 3),
                "frames": len(picks), "frame_stride": total_frames // max(1, args.animation),
                "seconds": round(anim_s, 3),
                "slowest_frames_ms": [[f, round(ms, 1)] for ms, f in per_frame[:5]],
                "step": "setup_animation_frame + per-frame upload + render per frame, frames dealt to ranks round-robin"}

    samples_per_step = cfg.width * cfg.height * cfg.samples_per_pixel * (world if args.shard == "frames" else 1)
    value = samples_per_step * args.steps / elapsed / 1e6
    value_frame = samples_per_step * args.steps / elapsed_frame / 1e6 if elapsed_frame else None

    is_metric = (cfg.width, cfg.height, cfg.samples_per_pixel) == (1280, 720, 1024)
    workload = "frame %d, %dx%d, %d spp, %d bounces" % (args.frame, cfg.width, cfg.height, cfg.samples_per_pixel,
                                                         cfg.max_bounces)
    result = None
    if rank == 0:
        roof = None
        if not args.no_roofline:
            # deterministic work counters of the same render (separate counting pass, untimed)
            if long_steps:
                print("counting pass", file=sys.stderr, flush=True)
            r.enable_counters(True)
            if shard is None:
                r.render(cfg, out_bgra=image)
            else:
                r.render_tiles(cfg, tw, th, shard.first, shard.stride, shard.count)
            r.synchronize()
            kc = r.kernel_counters()
            r.enable_counters(False)
            total = sum(kc[k] for k in kc)
            per_step_samples = int(total[0])
            # dominant kernel: the closest-hit BVH walk (k_wf_walk<closest>, "extend")
            ext_ms, ext_n = step_kernel_ms["extend"], step_kernel_n["extend"]
            ext_bytes = extend_bytes(kc["extend"])
            ms_per_launch = ext_ms / ext_n
            bytes_per_launch = ext_bytes / (ext_n / args.steps)
            achieved = bytes_per_launch / (ms_per_launch * 1e-3) / 1e9
            # whole hot path per step: wall time of the timed steps (the sky kernel runs
            # on a second stream, overlapped with the walks, so kernel times do not add up)
            path_ms = elapsed / args.steps * 1e3
            path_bytes = algorithmic_bytes(total)
            traffic, traffic_src = pmc_traffic("extend", workload, ms_per_launch)
            # the same kernel with nothing beside it: one untimed render with every
            # kernel on one stream (the timed steps run up to 4 kernels at once)
            if long_steps:
                print("isolated-walk pass", file=sys.stderr, flush=True)
            r.set_concurrency(0)
            r.enable_timing(True)
            if shard is None:
                r.render(cfg, out_bgra=image)
            else:
                r.render_tiles(cfg, tw, th, shard.first, shard.stride, shard.count)
            r.synchronize()
            kt_iso = r.kernel_times()
            r.enable_timing(False)
            r.set_concurrency(2)
            iso_ms = kt_iso["extend"][0] / max(1, kt_iso["extend"][1])
            iso_bytes = ext_bytes / max(1, kt_iso["extend"][1])   # one render's bytes over its launches
            iso_achieved = iso_bytes / (iso_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "traffic_source": traffic_src and ("%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                                                       "this workload, per launch)" % traffic_src),
                    "kernel": "k_wf_walk<closest> (extend: closest-hit BVH walk)",
                    "ms_per_launch": round(ms_per_launch, 4), "launches_per_step": ext_n / args.steps,
                    "bytes_per_launch": int(bytes_per_launch),
                    "kernel_ms_per_step": {k: round(v / args.steps, 3) for k, v in step_kernel_ms.items()},
                    "isolated": {"ms_per_launch": round(iso_ms, 4), "achieved": round(iso_achieved, 2),
                                 "frac": round(iso_achieved / HBM_PEAK_GBS, 5),
                                 "basis": "one extra untimed render with every kernel on one stream "
                                          "(ptg_set_concurrency(0)); the timed steps overlap the walk with the sky, "
                                          "shadow and the other chunk's kernels, which lengthens its launches"},
                    "hot_path": {"achieved_GBps": round(path_bytes / (path_ms * 1e-3) / 1e9, 2),
                                 "basis": "wall time per step",
                                 "algorithmic_bytes_per_sample": round(path_bytes / per_step_samples, 1),
                                 "formula": "32 visits + 60 tri + 88 enter + 156 shade + 160 per sample (SURVEY 8d)"},
                    "per_sample": {"node_visits": round(total[1] / per_step_samples, 2),
                                   "triangle_tests": round(total[2] / per_step_samples, 2),
                                   "blas_entries": round(total[3] / per_step_samples, 2),
                                   "ray_queries": round(total[4] / per_step_samples, 3),
                                   "shades": round(total[5] / per_step_samples, 3)}}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(assets, args.frame)
            except Exception as e:  # reported, never fatal to the GPU measurement
                cpu = {"value": None, "unit": "Msamples/s", "cores": None, "kind": "reference",
                       "sample": "failed: %s" % str(e)[:300]}
        result = {
            "metric": "Msamples/sec (whole node) at %dx%d %dspp" % (cfg.width, cfg.height, cfg.samples_per_pixel),
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if args.shard == "frames" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference scene assets + deterministic substitutes, frame %d" % args.frame,
            "config": {"workload": workload + (" (BASELINE metric config)" if is_metric else ""),
                       "baseline_config": args.config,
                       "shard": args.shard, "parallelism": "%s x%d" % (args.shard, world)},
            "animation": anim,
            "with_frame_setup": None if value_frame is None else {
                "value": round(value_frame, 3), "unit": "Msamples/s",
                "ms_per_step": round(elapsed_frame / args.steps * 1e3, 3),
                "step": "setup_animation_frame (host) + per-frame H2D upload + render, "
                        "pipelined (PCIe-inclusive; not the metric)"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if cpu and cpu.get("value"):
            result["gpu_vs_cpu"] = round(value / cpu["value"], 2)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    r.close()
    return result


if __name__ == "__main__":
    main()
