#!/usr/bin/env python3
"""The whole config.hh animation at the metric configuration, measured
(BASELINE.json's second metric: frames/min over the full animation; the
bench's `animation` leg samples 16 of the 1800 frames).

Renders frames start, start+stride, ... < stop on one GPU the way
main.cc:78-101 does per frame - host setup_animation_frame, the frame's
upload, render, the image back to the host (a writer thread hashes it in
place of the BMP write) - and appends one line per frame to
gpurun_out/full_anim_<start>_<stop>_<stride>.txt (frame, ms, BGRA hash), so
a long run shows progress.  Four calls of 450 frames (stride 4, start 0 /
1 / 2 / 3) cover the animation within gpurun's per-call limit;
tools/full_animation_sum.py adds them up.

Usage: python tools/full_animation.py --start 0 --stop 1800 --stride 4
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=0)
    ap.add_argument("--stop", type=int, default=1800)
    ap.add_argument("--stride", type=int, default=4)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--bounces", type=int, default=4)
    a = ap.parse_args()

    import torch
    from concurrent.futures import ThreadPoolExecutor
    import ptlumi_loader  # noqa: F401
    from ptlumi import native as N
    from ptlumi.renderer import GpuRenderer

    torch.cuda.set_device(0)
    cfg = N.RenderConfig.make(a.width, a.height, a.spp, a.bounces)
    scene = N.Scene(os.path.join(ROOT, "assets"), cfg)
    frames = list(range(a.start, min(a.stop, scene.frame_count()), a.stride))
    r = GpuRenderer(0)
    stream = torch.cuda.current_stream(0)
    r.set_stream(stream)
    r.set_hbm_share(40)        # the bench's owned-GPU chunking (bench.py --gpu-memory owned)
    r.set_chunk_paths(28)
    scene.setup_frame(frames[0])
    r.upload(scene, include_static=True)
    dev = torch.device("cuda", 0)
    image = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device=dev)
    acc = torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device=dev)
    host = [torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    pending = [None, None]
    writer = ThreadPoolExecutor(1)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    tag = "%d_%d_%d" % (a.start, a.stop, a.stride)
    log = open(os.path.join(ROOT, "gpurun_out", "full_anim_%s.txt" % tag), "w", buffering=1)

    def digest(buf, ev):
        ev.synchronize()
        return hashlib.sha256(buf.numpy().tobytes()).hexdigest()[:16]

    r.render(cfg, out_bgra=image, out_accum=acc)      # warm-up: the first render allocates the path state
    torch.cuda.synchronize()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(len(frames) + 1)]
    hashes = [None] * len(frames)
    t0 = time.perf_counter()
    marks[0].record(stream)
    for k, f in enumerate(frames):
        scene.setup_frame(f)
        r.upload(scene, include_static=False)
        r.render(cfg, out_bgra=image, out_accum=acc)
        marks[k + 1].record(stream)
        b = k % 2
        if pending[b] is not None:
            j, fut = pending[b]
            hashes[j] = fut.result()
            log.write("%d %.1f %s\n" % (frames[j], marks[j].elapsed_time(marks[j + 1]), hashes[j]))
        host[b].copy_(image, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        pending[b] = (k, writer.submit(digest, host[b], ev))
    for p in sorted((p for p in pending if p is not None), key=lambda p: p[0]):
        j, fut = p
        hashes[j] = fut.result()
        log.write("%d %.1f %s\n" % (frames[j], marks[j].elapsed_time(marks[j + 1]), hashes[j]))
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = [marks[k].elapsed_time(marks[k + 1]) for k in range(len(frames))]
    out = {"config": {"width": a.width, "height": a.height, "spp": a.spp, "bounces": a.bounces},
           "frames": frames, "frame_ms": [round(x, 2) for x in ms], "bgra_sha": hashes,
           "wall_s": round(wall, 3), "frames_per_min": round(len(frames) / wall * 60.0, 3),
           "msamples_per_s": round(len(frames) * a.width * a.height * a.spp / wall / 1e6, 2),
           "step": "host setup_animation_frame + per-frame upload + render + image to host (hashed by a writer "
                   "thread) per frame, one GPU, the bench's owned-GPU chunking"}
    with open(os.path.join(ROOT, "gpurun_out", "full_anim_%s.json" % tag), "w") as fh:
        json.dump(out, fh)
    print(json.dumps({k: out[k] for k in ("wall_s", "frames_per_min", "msamples_per_s")}, sort_keys=True),
          len(frames), "frames")


if __name__ == "__main__":
    main()
