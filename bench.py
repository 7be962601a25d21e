#!/usr/bin/env python3
"""Benchmark of the hot path: path_trace_pixel -> ray_query BVH traversal ->
tonemap_pixel under baseline_render, on MI355X.

Workload (the configuration BASELINE.json's metric is quoted on, "1280x720
1024spp"; configs[1] is the same frame at 256 spp): frame 0 of the reference
animation, 1280x720, 1024 samples per pixel, MAX_BOUNCES = 4 (the shipped
TESTING preset), the reference scene (reference OBJ assets + committed
substitutes for the three missing meshes).  One step = one baseline_render of
the frame on the GPU (+ the RCCL framebuffer gather in --shard tiles mode)
with the scene and the frame's TLAS/instances/subframes already resident in
HBM: `value`.  The bench process owns its GPU (--gpu-memory owned, the
default): sample chunks of up to 2^28 paths with 40% of HBM per chunk
pipeline (ptg_set_chunk_paths / ptg_set_hbm_share); --gpu-memory shared keeps
the library's defaults for a shared GPU; the bits are the same.

Beside `value` the line carries (rank 0):
  with_frame_setup  what main.cc does per frame - setup_animation_frame (host
                    C++) + H2D upload + render, pipelined (PCIe-inclusive,
                    never `value`);
  heavy_frame       the same metric on frame 450 (buddha close-up, ~7x the
                    per-sample work of frame 0; SURVEY 8(d) config 2's heavy
                    companion);
  animation         30 frames spread evenly over the 1800-frame animation
                    (the whole animation, measured: tools/full_animation.py),
                    each set up, uploaded, rendered and written as a BMP
                    asynchronously (main.cc:78-101, bmp.cc) - frames/min and
                    the average Msamples/s; spot rectangles of every frame's
                    radiance are saved for the oracle check
                    (tests/test_animation_spots.py);
  roofline          the dominant kernel, k_wf_walk<closest> (the closest-hit
                    BVH walk), against ceilings measured per level of the
                    memory hierarchy;
  cpu_baseline      the reference's own baseline_render built from its sources,
                    timed on this host's cores (bounded samples).

Multi-GPU: one process per GPU (torch.distributed.run).  `--gpus N` with N >
1 and no WORLD_SIZE in the environment starts the N ranks itself (a child
torch.distributed.run, before anything touches a GPU) and forwards its
output and exit code; a WORLD_SIZE that is not --gpus exits with status 2.
At N > 1 the line also carries `strong`: the metric frame in interleaved
tiles over the same ranks, gathered on rank 0 by one RCCL gather.  --shard frames
(default): rank r renders frame (frame + r) - weak scaling, no collective on
the data path (BASELINE config 4 style).  --shard tiles: one frame split into
interleaved 32x16 tiles, rank 0 gathers the BGRA tiles over RCCL and
assembles the framebuffer - strong scaling (config 3 style).  --shard samples:
one frame's samples split into whole motion-blur groups, rank 0 sum-reduces
the radiance over RCCL and tonemaps it - strong scaling, within float32
rounding of the single-GPU frame.
"""
import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PROFILES = os.path.join(ROOT, "profiles")
CEILINGS = os.path.join(PROFILES, "r02_probe", "ceilings.json")


def _natural(path):   # r01_wavefront11 after r01_wavefront9
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", path)]


def pmc_profile(kind, workload, ms_per_launch):
    """Per-launch PMC counters of `kind` from the newest committed rocprofv3
    profile of this workload (tools/profile_gpu.sh + summarize_prof.py) whose
    kernel-trace average launch time agrees with `ms_per_launch` (the same
    kernel measured alone in this run) within 15%: a profile of other code or
    another chunking is never used.  Returns (counters dict, path) or (None, None)."""
    import glob
    best = (None, None)
    for f in sorted(glob.glob(os.path.join(PROFILES, "*", "pmc_summary.json")), key=_natural):
        try:
            with open(f) as fh:
                prof = json.load(fh)
            ent = prof[kind]
            if prof.get("_workload") != workload or "hbm_side_bytes" not in ent["derived"]:
                continue
            if abs(ent["trace_avg_ms"] - ms_per_launch) > 0.15 * ms_per_launch:
                continue
            best = (ent, os.path.relpath(f, ROOT))
        except (OSError, KeyError, ValueError, TypeError):
            continue
    return best


def algorithmic_bytes(c):
    """B = 32 N_node + 60 N_tri + 88 N_enter + 156 N_hit + 160 per sample.

    32 B per node visit (24 B box + 8 B link in the reference layout), 60 B per
    triangle test (3 x u32 index + 3 x 16 B position), 88 B per BLAS entry
    (blas + mesh + inv_transform), 156 B per closest-hit shade (3 x u32 + 9 x
    16 B vertex attributes), 160 B subframe per sample."""
    samples, visits, tris, enters, queries, shades = [int(x) for x in c[:6]]
    return 32 * visits + 60 * tris + 88 * enters + 156 * shades + 160 * samples


def walker_bytes(w, c):
    """Bytes the closest-hit walk's own vector-memory instructions move per
    step, from the counting pass (ptg_last_walk_stats + work counters): a
    node phase reads a block copy's 7 x 16 B rows per lane that steps, a leaf
    phase 4 x 16 B rows per lane (a 48-B TriRec and the next 16 B, or a 64-B
    InstTrav), a started ray 48 B of path state (meta, origin, direction); a
    finished ray writes 16 B of hit record and 16 B of barycentrics."""
    queries = int(c[4])
    return 112 * w["node_lanes"] + 64 * w["leaf_lanes"] + 48 * w["refill_lanes"] + 32 * queries


def hierarchy_roofline(ent, launch_s):
    """Time floor of one walk launch from its PMC counts and the ceilings
    measured on this GPU for the walk's own access shape (random 16-B-per-lane
    gathers, tools/ta_probe.hip -> profiles/r02_probe/ceilings.json):

      vmem_issue  wave-level vector-memory instructions (SQ_INSTS_VMEM) vs the
                  per-CU issue floor (one per ~7.5 ns whatever the active lanes)
      l2          L2 line requests (TCC_HIT + TCC_MISS) vs the L2-resident
                  random-line rate
      fabric      L2 misses (TCC_MISS) vs the Infinity-Cache-resident
                  random-line rate
      hbm         HBM-side bytes (FETCH_SIZE x 2 + WRITE_SIZE, the guide's
                  gfx950 correction) vs 8 TB/s
      valu_issue  wave-level VALU instructions (SQ_INSTS_VALU) x 2 cycles per
                  SIMD (wave64 FP32 issue on gfx950, MI355X_MICROARCH.md) over
                  the 1024 SIMDs at the clock the profile measured
      salu_issue  wave-level SALU instructions (SQ_INSTS_SALU), one per cycle
                  per CU (256)

    Each level's time is count / rate; the largest is the floor t_min and
    names the bound.  frac = t_min / measured time (<= 1 by construction when
    the ceilings hold), each level in its own unit."""
    try:
        with open(CEILINGS) as fh:
            ceil = json.load(fh)
    except (OSError, ValueError):
        return None
    pmc = ent["per_dispatch_avg"]
    d = ent["derived"]
    levels = {}

    def level(name, count, rate, unit):
        t = count / rate
        levels[name] = {"count": count, "unit": unit, "ceiling_per_s": rate, "seconds": t, "frac": t / launch_s}

    level("vmem_issue", pmc["SQ_INSTS_VMEM"], ceil["vmem_issue_per_s"], "wave-instructions")
    level("l2", pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"], ceil["l2_lines_per_s"], "64-B line requests")
    level("fabric", pmc["TCC_MISS_sum"], ceil["ic_lines_per_s"], "64-B line requests (L2 misses)")
    level("hbm", d["hbm_side_bytes"], HBM_PEAK_GBS * 1e9, "bytes")
    clock = d.get("clock_GHz") or 2.4
    if "SQ_INSTS_VALU" in pmc:
        level("valu_issue", pmc["SQ_INSTS_VALU"] * 2.0, 1024 * clock * 1e9, "SIMD cycles (2 per wave64 VALU)")
    if "SQ_INSTS_SALU" in pmc:
        level("salu_issue", pmc["SQ_INSTS_SALU"], 256 * clock * 1e9, "CU scalar cycles")
    bound = max(levels, key=lambda k: levels[k]["seconds"])
    t_min = levels[bound]["seconds"]
    return {"bound": bound, "t_min_s": t_min, "levels": levels, "ceilings_source": os.path.relpath(CEILINGS, ROOT)}


def host_topology():
    """lscpu sockets/cores/model, nproc, this job's cgroup CPU quota and affinity."""
    import subprocess
    topo = {}
    try:
        out = subprocess.run(["lscpu"], stdout=subprocess.PIPE, text=True, timeout=30).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k = k.strip()
            if k in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)", "NUMA node(s)"):
                topo[k] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        topo["nproc"] = int(subprocess.run(["nproc"], stdout=subprocess.PIPE, text=True, timeout=30).stdout)
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        topo["cgroup_cpu_quota"] = None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        topo["cgroup_cpu_quota"] = None
    aff = sorted(os.sched_getaffinity(0))
    topo["affinity_cpus"] = len(aff)
    topo["_first_cpu"] = aff[0] if aff else 0
    return topo


def cpu_baseline(assets, frame, heavy_frame):
    """Reference baseline_render (main.cc:12) on this host, bounded samples:
    frame `frame` and `heavy_frame` at 1280x720 x 16 spp (Msamples/s is
    nearly SPP-invariant) with as many OpenMP threads as this job may use
    (the cgroup CPU quota, at most the CPUs in its affinity mask), pinned one
    per allowed CPU; and BASELINE configs[0] (frame 0, 640x360 x 32 spp) on
    one pinned core.  A whole socket cannot be timed under the quota, so the
    socket figure is a range: the per-core rate of the quota-sized run and of
    the one-core run, each times the socket's cores."""
    from oracle import Reference
    topo = host_topology()
    try:
        socket_cores = int(topo["Core(s) per socket"])
    except (KeyError, ValueError):
        socket_cores = os.cpu_count() or 1
    quota = topo.get("cgroup_cpu_quota")
    allowed = sorted(os.sched_getaffinity(0))
    threads = int(os.environ.get("PTG_CPU_THREADS", "0")) or max(1, min(len(allowed), int(quota) if quota else len(allowed)))
    cpus = allowed[:threads]
    ref = Reference("v3", 1280, 720, 16, 4)
    if not ref.available():
        return {"value": None, "unit": "Msamples/s", "cores": threads, "kind": "reference",
                "sample": "unavailable: %s not built" % ref.exe}
    r0 = ref.baseline(assets, frame, threads=threads, timeout=900, cpus=cpus, bind="true")
    rh = ref.baseline(assets, heavy_frame, threads=threads, timeout=900, cpus=cpus, bind="true") \
        if heavy_frame is not None else None
    per_core = r0["msamples_per_s"] / threads
    out = {"value": round(r0["msamples_per_s"], 4), "unit": "Msamples/s", "cores": threads, "kind": "reference",
           "sample": "frame %d, 1280x720 x 16 spp (14.7 M samples, full frame) through the reference's own "
                     "baseline_render (main.cc:12-46, OpenMP static schedule) built from /root/reference sources "
                     "with the reference flags (-O3 -ffast-math, -march=x86-64-v3); %d OpenMP threads pinned one per "
                     "CPU (OMP_PROC_BIND=true, CPUs %d-%d of this job's %d, quota %s); render %.2f s"
                     % (frame, threads, cpus[0], cpus[-1], len(allowed), quota if quota else "none", r0["render_s"]),
           "per_core": round(per_core, 4),
           "host": {k: v for k, v in topo.items() if not k.startswith("_")}}
    if rh:
        out["heavy_frame"] = {"frame": heavy_frame, "value": round(rh["msamples_per_s"], 4), "threads": threads,
                              "render_s": round(rh["render_s"], 3)}
    ref0 = Reference("v3", 640, 360, 32, 4)
    one_core = None
    if ref0.available():
        c0 = ref0.baseline(assets, 0, threads=1, timeout=600, cpus=[cpus[0]], bind="true")
        one_core = c0["msamples_per_s"]
        out["config0_one_core"] = {"value": round(one_core, 4), "unit": "Msamples/s", "cores": 1,
                                   "sample": "BASELINE configs[0]: frame 0, 640x360 x 32 spp (7.37 M samples), "
                                             "OMP_NUM_THREADS=1 pinned to CPU %d; render %.2f s"
                                             % (cpus[0], c0["render_s"])}
    if socket_cores > threads:
        lo_hi = sorted([per_core * socket_cores] + ([one_core * socket_cores] if one_core else []))
        out["socket_estimate"] = {
            "range": [round(lo_hi[0], 3), round(lo_hi[-1], 3)], "cores": socket_cores,
            "basis": "per-core rate x the %d cores of one socket, from the %d-thread run (%.4f per core) and the "
                     "one-core config-0 run (%.4f); a socket cannot be timed in this job (quota %s CPUs)"
                     % (socket_cores, threads, per_core, one_core or float("nan"), quota)}
    return out


def libm_identity():
    """The host C library the reference's results depend on: glibc's version,
    whether its ifuncs take the FMA builds of exp / pow / sin / cos (glibc 2.35
    picks __exp_fma etc. when the CPU has FMA and AVX2; the device restates
    those, csrc/device/glibc_math.h), and libm's file hash."""
    import ctypes.util
    import hashlib
    out = {}
    try:
        out["glibc"] = os.confstr("CS_GNU_LIBC_VERSION")
    except (ValueError, OSError):
        out["glibc"] = None
    flags = set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    except OSError:
        pass
    out["cpu_fma"] = "fma" in flags
    out["cpu_avx2"] = "avx2" in flags
    out["variant"] = "fma (__exp_fma, __pow_fma, __sin_fma, __cos_fma)" if out["cpu_fma"] and out["cpu_avx2"] \
        else "non-fma (the GPU's restatement is of the FMA builds: the reference would differ)"
    name = ctypes.util.find_library("m")
    for d in ("/lib/x86_64-linux-gnu", "/usr/lib/x86_64-linux-gnu"):
        p = os.path.join(d, "libm.so.6")
        if os.path.exists(p):
            with open(p, "rb") as fh:
                out["libm"] = {"path": p, "sha256_16": hashlib.sha256(fh.read()).hexdigest()[:16], "soname": name}
            break
    return out


def frame_golden(cfg, frame):
    """The reference's whole-image hashes of `frame` at this configuration
    (tests/golden/full_render_s1024.json, made by make_anim_golden.py full1024),
    or None."""
    path = os.path.join(ROOT, "tests", "golden", "full_render_s1024.json")
    try:
        g = json.load(open(path))
    except (OSError, ValueError):
        return None
    if (g["width"], g["height"], g["spp"]) != (cfg.width, cfg.height, cfg.samples_per_pixel) or cfg.max_bounces != 4:
        return None
    return g["frames"].get(str(frame))


def image_hashes(acc, bgra):
    """(radiance xyz f32 bits [H][W][3], BGRA [H][W][4]) hashes, as the reference
    harness's anim_render computes them (tests/anim_check.py)."""
    import hashlib
    import numpy as np
    rad = np.ascontiguousarray(np.asarray(acc, np.float32)[..., :3])
    return {"sha_radiance": hashlib.sha256(rad.view(np.uint32).tobytes()).hexdigest()[:32],
            "sha_bgra": hashlib.sha256(np.ascontiguousarray(bgra, np.uint8).tobytes()).hexdigest()[:32]}


def spot_rects(frame, w, h):
    """Three 2x2 rectangles per animation frame (centre + two frame-dependent)."""
    a = (frame * 2654435761) & 0xFFFFFFFF
    b = (a * 2246822519 + 374761393) & 0xFFFFFFFF
    return [(w // 2 - 1, h // 2 - 1, 2, 2), (a % (w - 2), (a >> 16) % (h - 2), 2, 2),
            (b % (w - 2), (b >> 16) % (h - 2), 2, 2)]


def check_spots(spots_npz, cfg):
    """'k/n': how many of this run's animation spot rectangles equal, in
    radiance bits and BGRA bytes, the reference's own render of the same
    rectangles (tests/golden/bench_spots.npz: the reference built from its
    sources, baseline_render semantics, main.cc:12-46); None when the golden
    file holds another configuration."""
    import numpy as np
    path = os.path.join(ROOT, "tests", "golden", "bench_spots.npz")
    if not os.path.exists(path):
        return None
    g = np.load(path)
    if (int(g["width"]), int(g["height"]), int(g["spp"]), int(g["bounces"])) != \
            (cfg.width, cfg.height, cfg.samples_per_pixel, cfg.max_bounces):
        return None
    want = {(int(f),) + tuple(int(v) for v in rc): (a, b) for f, rc, a, b in
            zip(g["frames"], g["rects"], g["acc_bits"], g["bgra"])}
    d = np.load(spots_npz)
    ok = n = 0
    for f, rc, a, b in zip(d["frames"], d["rects"], d["acc_bits"], d["bgra"]):
        key = (int(f),) + tuple(int(v) for v in rc)
        n += 1
        if key in want and np.array_equal(want[key][0], a) and np.array_equal(want[key][1], b):
            ok += 1
    return "%d/%d" % (ok, n)


def launcher_command(n, argv, port):
    """The child command bench.py runs for `--gpus n > 1` when no launcher
    started it: one process per GPU under torch.distributed.run on this node,
    rendezvous on 127.0.0.1, each rank given the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def world_check(gpus, env):
    """None when this process may run as one rank of `gpus`; "launch" when
    --gpus > 1 and no launcher set WORLD_SIZE (bench.py starts the ranks
    itself); an error message when the launcher's WORLD_SIZE is not --gpus
    (a silent N=1 line under --gpus N would be a false measurement)."""
    w = env.get("WORLD_SIZE")
    if w is None:
        return "launch" if gpus > 1 else None
    try:
        w = int(w)
    except ValueError:
        return "WORLD_SIZE %r is not an integer" % w
    if w != gpus:
        return "--gpus %d but WORLD_SIZE %d: refusing to report a %d-rank run as %d GPUs" % (gpus, w, w, gpus)
    return None


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
    ap.add_argument("--shard", choices=["frames", "tiles", "samples"], default="frames",
                    help="frames: rank r renders frame + r (weak scaling); tiles: one frame in interleaved tiles, "
                         "one RCCL gather (strong, bit-identical); samples: one frame's sample range in whole "
                         "motion-blur groups, one RCCL sum-reduce (strong, within float32 rounding)")
    ap.add_argument("--tile", type=str, default="32x16")
    ap.add_argument("--concurrency", type=int, default=2, choices=[0, 1, 2],
                    help="ptg_set_concurrency level of the timed steps (profiling passes use 0)")
    ap.add_argument("--gpu-memory", choices=["owned", "shared"], default="owned",
                    help="owned (default: the bench process owns its GPU): 2^28-path sample chunks, <= 40%% of HBM "
                         "per chunk pipeline (ptg_set_chunk_paths / ptg_set_hbm_share); shared: the library's "
                         "defaults (2^27, 35%%), which leave most of the GPU to other tenants.  Same bits either way")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--config", type=int, default=None, choices=[1, 2, 3, 4],
                    help="BASELINE.json configs[i] preset: 1 = 1280x720x256 frame 0; 2 = 1280x720x1024 frame 0 "
                         "in pixel tiles (the metric config; tiles over the ranks); 3 = the animation at 1024 spp "
                         "(frames/min over --animation K frames, default 30); 4 = 3840x2160x4096 frame 690 "
                         "(dragon + buddha in view) in pixel tiles")
    ap.add_argument("--no-frame-setup", action="store_true",
                    help="skip the second (PCIe-inclusive, per-frame host setup) timing loop")
    ap.add_argument("--heavy-frame", type=int, default=450,
                    help="also time this frame at the same configuration (-1: skip)")
    ap.add_argument("--animation", type=int, default=None, metavar="K",
                    help="render K frames spread evenly over the whole animation (frame-parallel over the ranks), "
                         "write them as BMPs and report frames/min (default 30 at the metric config, else 0: "
                         "30 frames gave 40.1 frames/min against the whole animation's measured 40.2, 16 gave 37.6)")
    ap.add_argument("--frames-dir", default=None, help="where the animation BMPs go (default: a temp directory)")
    ap.add_argument("--spots-out", default=None,
                    help="npz of every animation frame's spot rectangles (default gpurun_out/anim_spots_r<rank>.npz)")
    args = ap.parse_args()
    # N > 1 without a launcher: start N ranks as a child process (before this
    # process imports torch or touches a GPU) and forward its output and exit
    # code; a launcher whose world size is not --gpus is an error, not a warning
    wc = world_check(args.gpus, os.environ)
    if wc == "launch":
        import subprocess
        cmd = launcher_command(args.gpus, sys.argv[1:], free_port())
        print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
        sys.exit(subprocess.call(cmd))
    if wc is not None:
        print("bench.py: %s" % wc, file=sys.stderr, flush=True)
        sys.exit(2)
    if args.config == 1:
        args.width, args.height, args.spp, args.frame = 1280, 720, 256, 0
    elif args.config == 2:
        args.width, args.height, args.spp, args.frame, args.shard = 1280, 720, 1024, 0, "tiles"
    elif args.config == 3:
        args.width, args.height, args.spp = 1280, 720, 1024
        args.animation = args.animation or 30
    elif args.config == 4:
        args.width, args.height, args.spp, args.frame, args.shard = 3840, 2160, 4096, 690, "tiles"
        args.heavy_frame = -1
    is_metric = (args.width, args.height, args.spp) == (1280, 720, 1024)
    if args.animation is None:
        args.animation = 30 if is_metric else 0

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
    # PTG_BENCH_REHEARSE=1: rehearse the N>1 code paths with more ranks than GPUs
    # (ranks share devices, gloo instead of RCCL, which cannot put two ranks on
    # one GPU); never used for a measurement
    rehearse = os.environ.get("PTG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    ranks = None
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # the communicator's own size and every rank's device identity, so the
        # line proves how many distinct GPUs took part
        import socket
        props = torch.cuda.get_device_properties(local)
        me = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "device": props.name,
              "pci": "%s:%s:%s" % (getattr(props, "pci_domain_id", "?"), getattr(props, "pci_bus_id", "?"),
                                   getattr(props, "pci_device_id", "?")),
              "uuid": str(getattr(props, "uuid", ""))}
        allp = [None] * dist.get_world_size()
        dist.all_gather_object(allp, me)
        ranks = {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "devices": allp,
                 "distinct_gpus": len({(d["host"], d["pci"], d["uuid"]) for d in allp})}

    assets = os.path.join(ROOT, "assets")
    cfg = N.RenderConfig.make(args.width, args.height, args.spp, args.bounces)
    scene = N.Scene(assets, cfg)
    r = GpuRenderer(local)
    # the arithmetic environment the bit-exact results rest on (ptg_arith_selftest)
    try:
        selftest = r.selftest()
    except RuntimeError as e:   # a timing variant without the self-test (tools/variants/at_commit.py): never "passed"
        selftest = "unavailable: %s" % e
    stream = torch.cuda.current_stream(local)
    r.set_stream(stream)
    r.set_concurrency(args.concurrency)
    # a GPU shared by several local ranks (PTG_BENCH_REHEARSE) is not owned:
    # the library's shared defaults then (each rank's 74% would not fit)
    shares_gpu = int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > max(1, torch.cuda.device_count())
    if args.gpu_memory == "owned" and shares_gpu:
        args.gpu_memory = "shared"
    if args.gpu_memory == "owned":
        r.set_hbm_share(40)
        try:
            r.set_chunk_paths(28)
        except N.PtgError:   # a timing build of older sources without ptg_set_chunk_paths
            args.gpu_memory = "shared (2^28-path chunks unavailable)"
    tw, th = [int(v) for v in args.tile.split("x")]
    frame = args.frame + (rank if args.shard == "frames" else 0)

    # static scene once (load_scene output) - resident in HBM before timing
    scene.setup_frame(frame)
    r.upload(scene, include_static=True)
    dev = torch.device("cuda", local)
    image = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device=dev)
    accum = torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device=dev)
    shard = D.TileShard(cfg, tw, th, rank, world) if args.shard == "tiles" else None
    sshard = D.SampleShard(cfg, rank, world) if args.shard == "samples" else None

    def render_step():
        if sshard is not None:
            D.render_and_reduce(r, cfg, sshard, image, accum=accum, stream=stream)
        elif shard is None:
            r.render(cfg, out_bgra=image, out_accum=accum)   # the radiance too: the last step is hashed
        else:
            D.render_and_gather(r, cfg, shard, image, stream=stream)

    def frame_step():
        scene.setup_frame(frame)                     # setup_animation_frame (host)
        r.upload(scene, include_static=False)        # per-frame TLAS/instances/subframes over PCIe
        render_step()

    def upload_step():
        r.upload(scene, include_static=False)        # ptg_upload_frame: block packing + H2D, then the render
        render_step()

    long_steps = cfg.width * cfg.height * cfg.samples_per_pixel > 4e9

    def gather_floats(v):
        """v of every rank, in rank order."""
        if world == 1:
            return [v]
        t = torch.tensor([v], dtype=torch.float64, device="cpu" if rehearse else dev)
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [float(x.item()) for x in out]

    per_rank_s = {}

    def timed(fn, timing, steps=None, warmup=None, tag=None):
        """K steps of fn between barrier + synchronize on both sides; max over ranks."""
        steps = args.steps if steps is None else steps
        for _ in range(args.warmup if warmup is None else warmup):
            fn()
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(local)
        r.enable_timing(timing)
        t0 = time.perf_counter()
        for k in range(steps):
            fn()    # asynchronous: host work of step k+1 overlaps the kernels of step k
            if long_steps:   # progress for multi-minute configurations (completes step k-1 first)
                print("step %d/%d issued at %.1f s" % (k + 1, steps, time.perf_counter() - t0),
                      file=sys.stderr, flush=True)
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(local)
        el = time.perf_counter() - t0
        kb = r.kernel_busy() if timing else {}
        r.enable_timing(False)
        ranks_el = gather_floats(el)
        if tag:
            per_rank_s[tag] = ranks_el
        return max(ranks_el), kb

    def frame_check(f):
        """This rank's last rendered frame (accum + image) against the reference's
        whole-image hashes of frame f at this configuration, if the golden holds it."""
        if shard is not None or (sshard is not None and (world > 1 or rank != 0)):
            return None   # tiles: BGRA only; sample shards over N > 1 ranks sum in another order
        want = frame_golden(cfg, f)
        if want is None:
            return None
        acc_host = accum.cpu().numpy()
        got = image_hashes(acc_host, image.cpu().numpy())
        # pixels whose accumulated radiance is NaN: a path that met a zero BSDF
        # pdf turns its sample, and so its pixel's sum, into NaN - in the
        # reference too (path_tracer.hh:735-737, main.cc:42)
        nan_px = int(np.isnan(acc_host[..., :3]).any(-1).sum())
        rad_ok, bgra_ok = got["sha_radiance"] == want["sha_radiance"], got["sha_bgra"] == want["sha_bgra"]
        out = {"frame": f, "exact": rad_ok and bgra_ok, "radiance": rad_ok, "bgra": bgra_ok, "nan_pixels": nan_px}
        if "nan_pixels_yx" in want:   # the strict build's NaN pixels (same places, same bits when exact)
            out["nan_pixels_reference"] = len(want["nan_pixels_yx"])
        return dict(out, **{
                "golden": "tests/golden/full_render_s1024.json (the reference's strict build, whole image)"})

    def walk_levels(kind, workload, busy_ms, launches, iso_ms):
        """The roofline levels of one walk kind (extend / shadow) from the committed
        PMC profile of this workload, or the reason there are none."""
        ent, src = pmc_profile(kind, workload, iso_ms)
        hier = hierarchy_roofline(ent, iso_ms * 1e-3) if ent else None
        if not hier:
            return {"bound": None, "ms_per_launch_isolated": round(iso_ms, 4),
                    "basis": "no committed PMC profile of this workload whose launch time agrees with this run's "
                             "(%.3f ms)" % iso_ms}, None, None
        live_s = busy_ms * 1e-3 / launches
        top = hier["levels"][hier["bound"]]
        out = {"bound": hier["bound"], "frac_live": round(top["seconds"] / live_s, 5),
               "frac_isolated": round(hier["t_min_s"] / (iso_ms * 1e-3), 5),
               "ms_per_launch_live": round(busy_ms / launches, 4), "ms_per_launch_isolated": round(iso_ms, 4),
               "launches_per_step": launches, "source": src,
               "levels": {k: {"frac_isolated": round(v["frac"], 4), "frac_live": round(v["seconds"] / live_s, 4)}
                          for k, v in hier["levels"].items()}}
        return out, (ent, src, hier, live_s), top

    def measure_roofline(workload, kb, steps, elapsed_s):
        """Roofline of the closest-hit walk (the dominant kernel) and the levels of
        both walks, for the frame currently uploaded: `kb` = the timed steps'
        kernel_busy record; then one counting pass and one isolated pass (every
        kernel on one stream), both untimed."""
        step_busy_ms = {k: v[0] for k, v in kb.items() if v[2]}
        step_sum_ms = {k: v[1] for k, v in kb.items() if v[2]}
        step_launches = {k: v[2] for k, v in kb.items() if v[2]}
        if long_steps:
            print("counting pass", file=sys.stderr, flush=True)
        r.enable_counters(True)
        if shard is not None:
            r.render_tiles(cfg, tw, th, shard.first, shard.stride, shard.count)
        else:
            r.render(cfg, out_bgra=image, samples=(sshard.j0, sshard.j1) if sshard else None)
        r.synchronize()
        kc = r.kernel_counters()
        ws = r.walk_stats()
        r.enable_counters(False)
        total = sum(kc[k] for k in kc)
        per_step_samples = int(total[0])
        # dominant kernel: the closest-hit BVH walk (k_wf_walk<closest>, "extend")
        wb = walker_bytes(ws["extend"], kc["extend"])           # bytes its own loads and stores move per step
        launches = step_launches["extend"] / steps
        busy_ms = step_busy_ms["extend"] / steps                 # union of its launch intervals per step
        # the same kernels with nothing beside them: one untimed render with every
        # kernel on one stream (the timed steps run up to 4 kernels at once)
        if long_steps:
            print("isolated-walk pass", file=sys.stderr, flush=True)
        r.set_concurrency(0)
        r.enable_timing(True)
        if shard is not None:
            r.render_tiles(cfg, tw, th, shard.first, shard.stride, shard.count)
        else:
            r.render(cfg, out_bgra=image, samples=(sshard.j0, sshard.j1) if sshard else None)
        r.synchronize()
        kb_iso = r.kernel_busy()
        r.enable_timing(False)
        r.set_concurrency(args.concurrency)
        iso = {k: kb_iso[k][1] / max(1, kb_iso[k][2]) for k in ("extend", "shadow")}
        walks = {}
        ext = None
        for k in ("extend", "shadow"):
            if step_launches.get(k):
                walks[k], info, top = walk_levels(k, workload, step_busy_ms[k] / steps, step_launches[k] / steps,
                                                  iso[k])
                if k == "extend":
                    ext = (info, top)
        iso_ms = iso["extend"]
        path_ms = elapsed_s / steps * 1e3
        path_bytes = algorithmic_bytes(total)
        w = ws["extend"]
        lanes = {"node_phase": round(w["node_lanes"] / max(1, w["node_phases"]), 2),
                 "leaf_phase": round(w["leaf_lanes"] / max(1, w["leaf_phases"]), 2),
                 "refill": round(w["refill_lanes"] / max(1, w["refills"]), 2),
                 "active_per_iteration": round(w["active_lanes"] / max(1, w["iterations"]), 2)}
        wsh = ws["shadow"]
        lanes_any = {"node_phase": round(wsh["node_lanes"] / max(1, wsh["node_phases"]), 2),
                     "leaf_phase": round(wsh["leaf_lanes"] / max(1, wsh["leaf_phases"]), 2),
                     "refill": round(wsh["refill_lanes"] / max(1, wsh["refills"]), 2),
                     "active_per_iteration": round(wsh["active_lanes"] / max(1, wsh["iterations"]), 2)}
        roof = {"kernel": "k_wf_walk<closest> (extend: closest-hit BVH walk)", "workload": workload}
        if ext and ext[0]:
            (ent, prof_src, hier, live_s), top = ext
            roof.update({
                "bound": hier["bound"],
                # in the bound level's own unit: its count per launch over the
                # live time per launch, against that level's measured ceiling
                "achieved": round(top["count"] / live_s / 1e9, 3),
                "peak": round(top["ceiling_per_s"] / 1e9, 3),
                "unit": "G " + top["unit"] + " per s",
                "frac": round(top["count"] / live_s / top["ceiling_per_s"], 5),
                "traffic": int(ent["derived"]["hbm_side_bytes"]),
                "traffic_source": "%s (rocprofv3 --pmc passes of this workload, per launch: FETCH_SIZE x 1 KiB "
                                  "x 2 + WRITE_SIZE x 1 KiB)" % prof_src,
                "basis": "bound = the memory/issue level with the largest time floor for one launch (count "
                         "from the committed PMC profile of this workload / ceiling measured on MI355X for the "
                         "walk's access shape, see 'levels'); achieved = that count / the launch's live time "
                         "(busy time per step, union of its launch intervals on HIP events, / launches per "
                         "step); frac = achieved / peak = floor / live time",
                "levels": {k: {"count_per_launch": v["count"], "unit": v["unit"],
                               "ceiling_per_s": v["ceiling_per_s"], "frac_isolated": round(v["frac"], 4),
                               "frac_live": round(v["seconds"] / live_s, 4)} for k, v in hier["levels"].items()},
                "ceilings_source": hier["ceilings_source"],
                "hbm": {"bytes_per_launch": int(ent["derived"]["hbm_side_bytes"]),
                        "achieved_GBps": round(ent["derived"]["hbm_side_bytes"] / live_s / 1e9, 2),
                        "peak_GBps": HBM_PEAK_GBS,
                        "frac": round(ent["derived"]["hbm_side_bytes"] / live_s / 1e9 / HBM_PEAK_GBS, 5)}})
        else:
            roof.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                         "traffic": None,
                         "basis": "no committed PMC profile of this workload whose launch time agrees with "
                                  "this run's (%.3f ms): levels not derived" % iso_ms})
        roof.update({
            "ms_per_launch": round(busy_ms / launches, 4), "launches_per_step": launches,
            "isolated": {"ms_per_launch": round(iso_ms, 4),
                         "frac": walks.get("extend", {}).get("frac_isolated"),
                         "basis": "one extra untimed render with every kernel on one stream "
                                  "(ptg_set_concurrency(0))"},
            "walks": walks,
            "walker_bytes": {"per_launch": int(wb / launches),
                             "achieved_GBps": round(wb / (busy_ms * 1e-3) / 1e9, 2),
                             "basis": "bytes the walk's own vector-memory instructions move (counting pass, "
                                      "ptg_last_walk_stats): 7 x 16 B block rows per node-phase lane, 4 x 16 B "
                                      "record rows per leaf-phase lane, 48 B of ray state per started ray, 32 B "
                                      "of result per finished ray; mostly served by L2 and the Infinity Cache, "
                                      "so it is compared with no HBM figure"},
            "lanes_per_vmem_instruction": lanes,
            "lanes_per_vmem_instruction_any_hit": lanes_any,
            "kernel_busy_ms_per_step": {k: round(v / steps, 3) for k, v in step_busy_ms.items()},
            "kernel_sum_ms_per_step": {k: round(v / steps, 3) for k, v in step_sum_ms.items()},
            "reference_equivalent_bytes_rate": {
                "GBps": round(path_bytes / (path_ms * 1e-3) / 1e9, 2),
                "bytes_per_sample": round(path_bytes / per_step_samples, 1),
                "basis": "SURVEY 8(d)'s formula, 32 visits + 60 tri + 88 enter + 156 shade + 160 per sample: "
                         "what the REFERENCE's stackless walk would read per sample, over the wall time per "
                         "step.  Not a memory rate of this code (the block walker reads other records, mostly "
                         "from cache) and not comparable with HBM peak"},
            "per_sample": {"node_visits": round(total[1] / per_step_samples, 2),
                           "triangle_tests": round(total[2] / per_step_samples, 2),
                           "blas_entries": round(total[3] / per_step_samples, 2),
                           "ray_queries": round(total[4] / per_step_samples, 3),
                           "shades": round(total[5] / per_step_samples, 3)}})
        return roof

    def workload_of(f):
        return "frame %d, %dx%d, %d spp, %d bounces" % (f, cfg.width, cfg.height, cfg.samples_per_pixel,
                                                         cfg.max_bounces)

    # (1) the metric: render steps over a frame whose inputs are resident in HBM
    elapsed, kb = timed(render_step, True, tag="metric")
    main_check = frame_check(frame)   # this rank's last timed image against the reference's
    # (2) SURVEY 8(d)'s definition: W.H.SPP / (upload-frame + render + gather)
    elapsed_upload = None if args.no_frame_setup else timed(upload_step, False)[0]
    # (3) the reference's per-frame loop: host setup_animation_frame + PCIe upload + render
    elapsed_frame = None if args.no_frame_setup else timed(frame_step, False)[0]

    samples_per_step = cfg.width * cfg.height * cfg.samples_per_pixel * (world if args.shard == "frames" else 1)
    value = samples_per_step * args.steps / elapsed / 1e6
    value_upload = samples_per_step * args.steps / elapsed_upload / 1e6 if elapsed_upload else None
    value_frame = samples_per_step * args.steps / elapsed_frame / 1e6 if elapsed_frame else None

    # (3b) N > 1 under the default frame shard: the strong-scaling companion,
    # the metric frame itself cut into interleaved tiles over the same ranks
    # and assembled on rank 0 by one RCCL gather (BASELINE configs[2])
    strong = None
    if world > 1 and args.shard == "frames":
        scene.setup_frame(args.frame)
        r.upload(scene, include_static=False)
        tshard = D.TileShard(cfg, tw, th, rank, world)
        full = torch.zeros_like(image)

        def strong_step():
            D.render_and_gather(r, cfg, tshard, full, stream=stream)

        el_s, _ = timed(strong_step, False, tag="strong_tiles")
        strong = {"value": round(cfg.width * cfg.height * cfg.samples_per_pixel * args.steps / el_s / 1e6, 3),
                  "unit": "Msamples/s", "ms_per_step": round(el_s / args.steps * 1e3, 3), "steps": args.steps,
                  "scaling": "strong", "frame": args.frame, "shard": "tiles %dx%d round-robin over %d ranks" % (tw, th, world),
                  "step": "render this rank's tiles + one gather of the BGRA tiles to rank 0 + scatter into the "
                          "framebuffer (distributed.render_and_gather)"}
        if rank == 0:
            want = frame_golden(cfg, args.frame)
            if want is not None:
                import hashlib
                got = hashlib.sha256(np.ascontiguousarray(full.cpu().numpy()).tobytes()).hexdigest()[:32]
                strong["bgra_exact"] = got == want["sha_bgra"]

    # (3) the heavy companion frame at the same configuration, with its own roofline
    heavy = None
    if args.heavy_frame >= 0:
        hf = args.heavy_frame + (rank if args.shard == "frames" else 0)
        scene.setup_frame(hf)
        r.upload(scene, include_static=False)
        hsteps = max(1, min(args.steps, 3))
        el_h, kb_h = timed(render_step, True, steps=hsteps, warmup=1, tag="heavy_frame")
        heavy = {"frame": args.heavy_frame, "value": round(samples_per_step * hsteps / el_h / 1e6, 3),
                 "unit": "Msamples/s", "ms_per_step": round(el_h / hsteps * 1e3, 3), "steps": hsteps,
                 "frame_check": frame_check(hf)}
        if rank == 0 and not args.no_roofline:
            heavy["roofline"] = measure_roofline(workload_of(args.heavy_frame), kb_h, hsteps, el_h)

    # (4) the animation (BASELINE config 4): K frames spread evenly over all 1800 (frame
    # cost varies ~7x), frame-parallel over the ranks; each frame is set up on the host,
    # uploaded, rendered, copied back and written as a BMP by a writer thread while the
    # next frame renders (main.cc:78-101)
    anim = None
    if args.animation > 0:
        import tempfile
        from concurrent.futures import ThreadPoolExecutor
        total_frames = scene.frame_count()
        picks = [round(i * total_frames / args.animation) % total_frames for i in range(args.animation)]
        mine = picks[rank::world]
        frames_dir = args.frames_dir or tempfile.mkdtemp(prefix="ptg_frames_")
        os.makedirs(frames_dir, exist_ok=True)
        acc_img = torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device=dev)
        host = [torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        pending = [None, None]
        spots = {"frames": [], "rects": [], "acc_bits": [], "bgra": []}
        writer = ThreadPoolExecutor(1)

        def write(path, buf, ev):
            ev.synchronize()
            N.write_bmp(path, buf.numpy())

        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(len(mine) + 1)]
        marks[0].record(stream)
        for k, f in enumerate(mine):
            scene.setup_frame(f)
            r.upload(scene, include_static=False)
            r.render(cfg, out_bgra=image, out_accum=acc_img)
            marks[k + 1].record(stream)
            b = k % 2
            if pending[b] is not None:
                pending[b].result()             # the writer is done with this staging buffer
            host[b].copy_(image, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            pending[b] = writer.submit(write, os.path.join(frames_dir, "frame_%04d.bmp" % f), host[b], ev)
            for x0, y0, rw, rh in spot_rects(f, cfg.width, cfg.height):
                # device-side copies (asynchronous, in stream order); read back after the loop
                spots["frames"].append(f)
                spots["rects"].append((x0, y0, rw, rh))
                spots["acc_bits"].append(acc_img[y0:y0 + rh, x0:x0 + rw, :3].clone())
                spots["bgra"].append(image[y0:y0 + rh, x0:x0 + rw].clone())
        for p in pending:
            if p is not None:
                p.result()
        torch.cuda.synchronize(local)
        per_frame = sorted(((marks[k].elapsed_time(marks[k + 1]), f) for k, f in enumerate(mine)), reverse=True)
        writer.shutdown()
        if world > 1:
            dist.barrier()
        anim_ranks = gather_floats(time.perf_counter() - t0)
        per_rank_s["animation"] = anim_ranks
        anim_s = max(anim_ranks)
        spots_out = args.spots_out or os.path.join(ROOT, "gpurun_out", "anim_spots_r%d.npz" % rank)
        os.makedirs(os.path.dirname(spots_out), exist_ok=True)
        np.savez_compressed(spots_out, frames=np.array(spots["frames"], np.int32),
                            rects=np.array(spots["rects"], np.int32),
                            acc_bits=np.array([t.cpu().numpy().view(np.uint32) for t in spots["acc_bits"]]),
                            bgra=np.array([t.cpu().numpy() for t in spots["bgra"]]), width=cfg.width, height=cfg.height,
                            spp=cfg.samples_per_pixel, bounces=cfg.max_bounces)
        bmps = sum(1 for f in mine if os.path.exists(os.path.join(frames_dir, "frame_%04d.bmp" % f)))
        spots_exact = check_spots(spots_out, cfg)
        anim = {"frames_per_min": round(len(picks) / anim_s * 60.0, 3),
                "full_animation_min": round(total_frames / (len(picks) / anim_s * 60.0), 2),
                "msamples_per_s": round(len(picks) * cfg.width * cfg.height * cfg.samples_per_pixel / anim_s / 1e6, 3),
                "frames": len(picks), "frame_stride": total_frames // max(1, args.animation),
                "seconds": round(anim_s, 3), "bmps_written": bmps, "frames_dir": frames_dir,
                "spots": os.path.relpath(spots_out, ROOT) if spots_out.startswith(ROOT) else spots_out,
                "slowest_frames_ms": [[f, round(ms, 1)] for ms, f in per_frame[:5]],
                "spots_exact": spots_exact,
                "step": "setup_animation_frame + per-frame upload + render + BMP write (writer thread, overlapped "
                        "with the next frame) per frame; frames dealt to ranks round-robin; spots_exact: the spot "
                        "rectangles of every frame (radiance bits and BGRA) against the reference's own render of "
                        "them (tests/golden/bench_spots.npz, made by tests/golden/make_anim_golden.py)"}

    workload = workload_of(args.frame)
    result = None
    if rank == 0:
        roof = None
        if not args.no_roofline:
            if heavy is not None or anim is not None:   # back to the metric frame for the counting passes
                scene.setup_frame(frame)
                r.upload(scene, include_static=False)
            roof = measure_roofline(workload, kb, args.steps, elapsed)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(assets, args.frame, args.heavy_frame if args.heavy_frame >= 0 else None)
            except Exception as e:  # reported, never fatal to the GPU measurement
                cpu = {"value": None, "unit": "Msamples/s", "cores": None, "kind": "reference",
                       "sample": "failed: %s" % str(e)[:300]}
        result = {
            "metric": "Msamples/sec (whole node) at %dx%d %dspp" % (cfg.width, cfg.height, cfg.samples_per_pixel),
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": ranks["world_size"] if ranks else world,
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
                       "shard": args.shard, "parallelism": "%s x%d" % (args.shard, world),
                       "gpu_memory": ("owned: sample chunks of <= 2^28 paths, <= 40% of HBM per chunk pipeline"
                                      if args.gpu_memory == "owned" else
                                      "shared: the library's defaults, <= 2^27 paths and 35% of HBM per pipeline")},
            "frame_exact": None if main_check is None else main_check["exact"],
            "frame_check": main_check,
            "selftest": selftest,
            "libm": libm_identity(),
            "ranks": ranks,
            "per_rank_seconds": {k: [round(x, 4) for x in v] for k, v in per_rank_s.items()} if world > 1 else None,
            "strong": strong,
            "heavy_frame": heavy,
            "animation": anim,
            "value_survey_def": None if value_upload is None else {
                "value": round(value_upload, 3), "unit": "Msamples/s",
                "ms_per_step": round(elapsed_upload / args.steps * 1e3, 3),
                "step": "SURVEY 8(d): ptg_upload_frame (TLAS block packing + H2D of the frame's records) + render "
                        "(+ gather), the frame's host arrays already set up"},
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
            if cpu.get("socket_estimate"):
                lo, hi = cpu["socket_estimate"]["range"]
                result["gpu_vs_cpu_socket_estimate"] = [round(value / hi, 2), round(value / lo, 2)]
            if heavy and cpu.get("heavy_frame"):
                result["heavy_gpu_vs_cpu"] = round(heavy["value"] / cpu["heavy_frame"]["value"], 2)
        # the evidence a reader of the line's tail needs, last and flat (the
        # driver keeps only the last ~2000 characters of stdout)
        result["summary"] = {
            "value": result["value"], "n_gpus": result["n_gpus"], "ms_per_step": result["ms_per_step"],
            "frame_exact": result["frame_exact"],
            "heavy_ms": heavy["ms_per_step"] if heavy else None,
            "heavy_value": heavy["value"] if heavy else None,
            "heavy_frame_exact": (heavy.get("frame_check") or {}).get("exact") if heavy else None,
            "nan_pixels": [(main_check or {}).get("nan_pixels"), ((heavy or {}).get("frame_check") or {}).get("nan_pixels")],
            "anim_frames_per_min": anim["frames_per_min"] if anim else None,
            "anim_spots": anim["spots_exact"] if anim else None,
            "strong_value": strong["value"] if strong else None,
            "strong_bgra_exact": strong.get("bgra_exact") if strong else None,
            "distinct_gpus": ranks["distinct_gpus"] if ranks else 1,
            "roofline_frac": roof.get("frac") if roof else None,
            "roofline_bound": roof.get("bound") if roof else None,
            "heavy_roofline_frac": ((heavy or {}).get("roofline") or {}).get("frac"),
            "cpu_value": cpu.get("value") if cpu else None,
            "gpu_vs_cpu": result.get("gpu_vs_cpu"),
            "selftest": selftest}
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    r.close()
    return result


if __name__ == "__main__":
    main()
