#!/usr/bin/env python3
"""Timing experiment (not a parity path): does the GPU render a frame faster
when two independent halves of its sample range run concurrently (two
renderer contexts, two stream sets), so that one half's round-0 walk and
shade overlap the other half's sky and shadow kernels?
Usage: python tools/ab_two.py [--frame F] [--spp S] [--reps R]"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--frame", type=int, default=0)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
import torch  # noqa
import ptlumi_loader  # noqa
from ptlumi import native as N
from ptlumi.renderer import GpuRenderer
cfg = N.RenderConfig.make(1280, 720, a.spp, 4)
s = N.Scene(os.path.join(ROOT, "assets"), cfg)
s.setup_frame(a.frame)
ra, rb = GpuRenderer(0), GpuRenderer(0)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
ra.set_stream(sa)
rb.set_stream(sb)
ra.upload(s)
rb.upload(s)
img_a = torch.empty((720, 1280, 4), dtype=torch.uint8, device="cuda:0")
img_b = torch.empty_like(img_a)
half = (a.spp // 2) // 8 * 8


def one():
    ra.render(cfg, out_bgra=img_a)
    torch.cuda.synchronize()


def two():
    ra.render(cfg, samples=(0, half), out_bgra=img_a)
    rb.render(cfg, samples=(half, a.spp), out_bgra=img_b)
    torch.cuda.synchronize()


res = {}
for name, fn in (("one", one), ("two", two), ("one_again", one)):
    fn()
    best = 1e30
    for _ in range(a.reps):
        t = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t)
    res[name] = round(best * 1e3, 2)
print(json.dumps({"frame": a.frame, "spp": a.spp, "ms": res}))
