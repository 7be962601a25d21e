#!/usr/bin/env python3
"""Timing ablations (NOT parity builds): renders the bench frame and prints
per-kernel device times.  PTG_LIB selects an alternative libptg.so.
Usage: python tools/ablate.py [--spp 64] [--bounces 4] [--pipeline wavefront|megakernel]"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--bounces", type=int, default=4)
ap.add_argument("--frame", type=int, default=0)
ap.add_argument("--width", type=int, default=1280)
ap.add_argument("--height", type=int, default=720)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--pipeline", default="wavefront")
ap.add_argument("--counters", action="store_true")
ap.add_argument("--concurrency", type=int, default=2)
ap.add_argument("--owned", action="store_true", help="the bench's owned-GPU chunking: 2^28 paths, 40%% HBM share")
a = ap.parse_args()
import torch  # noqa
import ptlumi_loader  # noqa
from ptlumi import native as N
from ptlumi.renderer import GpuRenderer
cfg = N.RenderConfig.make(a.width, a.height, a.spp, a.bounces)
s = N.Scene(os.path.join(ROOT, "assets"), cfg); s.setup_frame(a.frame)
r = GpuRenderer(0); r.upload(s); r.set_pipeline(a.pipeline); r.set_concurrency(a.concurrency)
if a.owned:
    r.set_hbm_share(40); r.set_chunk_paths(28)
img, _ = r.render(cfg); r.synchronize()
r.enable_timing(True)
best, kt = 1e30, None
for _ in range(a.reps):
    t = time.perf_counter(); r.render(cfg, out_bgra=img); r.synchronize(); wall = (time.perf_counter() - t) * 1e3
    times = r.kernel_times()   # reading clears the record
    if wall < best:
        best, kt = wall, times
extra = {}
if a.counters:
    r.enable_timing(False); r.enable_counters(True); r.render(cfg, out_bgra=img); r.synchronize()
    kc = r.kernel_counters()
    names = ["samples", "visits", "tri_tests", "blas_entries", "queries", "shades", "tlas_visits", "wave_iters"]
    extra = {k: {n: int(v[i]) for i, n in enumerate(names)} for k, v in kc.items() if int(v[:8].sum())}
    if a.pipeline == "wavefront":
        extra["redo"] = r.redo_stats()
import hashlib, numpy as np
sha_bgra = hashlib.sha256(np.ascontiguousarray(img.cpu().numpy(), np.uint8).tobytes()).hexdigest()[:32]
print(json.dumps({"sha_bgra": sha_bgra, "counters": extra, "lib": os.path.basename(N.LIB_PATH), "pipeline": a.pipeline, "spp": a.spp, "bounces": a.bounces,
                  "frame": a.frame, "wall_ms": round(best, 2), "msamples_per_s": round(a.width * a.height * a.spp / best / 1e3, 2),
                  "kernels_ms": {k: round(v[0], 2) for k, v in kt.items() if v[1]}}))
