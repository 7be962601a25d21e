#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs the reference renderer compiled from its own sources under
/root/reference (oracle/Makefile, strict IEEE mode; driver oracle/ref_harness.cc)
on deterministic inputs and stores inputs + outputs as small .npz fixtures:

  pcg4d.npz         2048 seeds -> pcg4d / generate_uniform_random4 (math.hh:466-485)
  tonemap.npz       4096+ colours -> tonemap_pixel BGRA (path_tracer.hh:753-771)
  rays_f450.npz     4096 rays through frame 450, subframe 1 -> closest hit + any hit
                    (ray_query.hh:111-290)
  samples_fNNN.npz  path_trace_pixel outputs, 16x16 pixels x 8 samples, frames 0/450/1750
                    at 640x360 / 32 spp / 4 bounces (path_tracer.hh:637-741)
  frame_160x90.npz  baseline_render semantics over a whole 160x90 x 32 spp frame 0:
                    averaged radiance + BGRA (main.cc:12-46)
  scene_hashes.json SHA-256 of every scene array (padding masked) for frames 0 and 450
                    at 640x360 / 32 spp (load_scene + setup_animation_frame)
  frame_0000_ref.npz the reference's own committed output/frame_0000.bmp (640x360,
                    256 spp, built by its authors with GCC -ffast-math on the
                    original assets) as RGB, for the validator-PSNR check

Needs /root/reference (this container only); the GPU box never runs this.
Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import ptlumi_loader  # noqa: E402,F401
from ptlumi import validator  # noqa: E402
from oracle import Reference  # noqa: E402

ASSETS = os.path.join(ROOT, "assets")
SAMPLE_REGIONS = {0: (312, 168), 450: (300, 150), 1750: (320, 200)}


def scene_hashes(dump_dir):
    f3 = lambda a: np.ascontiguousarray(a.reshape(-1, 4)[:, :3])
    out = {}
    for name in ["nodes", "links", "indices", "albedo", "material"]:
        out[name] = hashlib.sha256(open(os.path.join(dump_dir, name + ".bin"), "rb").read()).hexdigest()
    for name in ["pos", "normal"]:
        a = np.fromfile(os.path.join(dump_dir, name + ".bin"), np.float32)
        out[name] = hashlib.sha256(f3(a).tobytes()).hexdigest()
    inst = np.fromfile(os.path.join(dump_dir, "instances.bin"), np.uint32).reshape(-1, 40)
    out["instances"] = hashlib.sha256(np.ascontiguousarray(inst[:, [0, 1, 2, 3, 4, 5] + list(range(8, 40))]).tobytes()).hexdigest()
    sf = np.fromfile(os.path.join(dump_dir, "subframes.bin"), np.uint32).reshape(-1, 40)
    keep = [0, 1] + [4 + 4 * r + c for r in range(3) for c in range(3)] + [16, 17, 18] + list(range(20, 26)) + \
           [28, 29, 30, 32, 33, 34, 36]
    out["subframes"] = hashlib.sha256(np.ascontiguousarray(sf[:, keep]).tobytes()).hexdigest()
    out["counts"] = {k: int(v) for k, v in (l.split()[:2] for l in open(os.path.join(dump_dir, "meta.txt"))
                                             if l.split()[0] in ("nodes", "instances", "subframes", "static_instance_count"))}
    return out


def main():
    ref = Reference("strict", 640, 360, 32, 4)
    small = Reference("strict", 160, 90, 32, 4)
    assert ref.available() and small.available(), "build the reference first: python -c 'import __graft_entry__ as g; g.build()'"
    rng = np.random.default_rng(20261015)
    import tempfile

    # pcg4d KATs
    seeds = np.concatenate([rng.integers(0, 2 ** 32, (2040, 4), dtype=np.uint64).astype(np.uint32),
                            np.array([[0, 0, 0, 0], [1, 2, 3, 4], [0xFFFFFFFF] * 4, [0, 0, 0, 152121358],
                                      [639, 359, 255, 152121358], [1919, 1079, 1023, 152121358], [7, 0, 0, 0],
                                      [0x80000000, 1, 0x7FFFFFFF, 3]], np.uint32)])
    with tempfile.TemporaryDirectory() as d:
        seeds.tofile(os.path.join(d, "in"))
        ref.run(ASSETS, "pcg", os.path.join(d, "in"), os.path.join(d, "out"))
        o = np.fromfile(os.path.join(d, "out"), np.uint32).reshape(-1, 8)
    np.savez_compressed(os.path.join(HERE, "pcg4d.npz"), seeds=seeds, pcg=o[:, :4], uniform_bits=o[:, 4:])

    # tonemap
    colors = np.concatenate([
        np.linspace(0, 4, 2048, dtype=np.float32)[:, None].repeat(4, 1),
        rng.exponential(0.7, (2048, 4)).astype(np.float32),
        np.array([[0, 0, 0, 0], [0.0031308, 0.0031307, 0.00313081, 0], [1e-30, 1e30, 65504, 0],
                  [-1, -0.0, 0.5, 0], [np.inf, 0, 0, 0]], np.float32)])
    colors[:, 3] = 0
    with tempfile.TemporaryDirectory() as d:
        colors.tofile(os.path.join(d, "in"))
        ref.run(ASSETS, "tonemap", os.path.join(d, "in"), os.path.join(d, "out"))
        bgra = np.fromfile(os.path.join(d, "out"), np.uint8).reshape(-1, 4)
    np.savez_compressed(os.path.join(HERE, "tonemap.npz"), colors=colors, bgra=bgra)

    # rays through frame 450 (buddha + vegetation), subframe 1
    n = 4096
    o = rng.uniform([-100, 0, -100], [100, 60, 100], (n, 3)).astype(np.float32)
    dvec = rng.normal(size=(n, 3)).astype(np.float32)
    dvec /= np.linalg.norm(dvec, axis=1, keepdims=True)
    dvec[:64] = np.array([0, -1, 0], np.float32)              # straight down onto the terrain
    dvec[64:80] = np.array([1, 0, 0], np.float32)             # axis-aligned: zero components -> 1e40
    rays = np.concatenate([o, dvec, np.full((n, 1), 1e-4, np.float32), np.full((n, 1), 1e9, np.float32)], 1)
    rays[80:96, 7] = 5.0                                      # short tmax
    hits = ref.rays(ASSETS, 450, 1, rays)
    np.savez_compressed(os.path.join(HERE, "rays_f450.npz"), rays=rays, hits=hits, frame=450, subframe=1)

    # per-sample outputs
    for frame, (x0, y0) in SAMPLE_REGIONS.items():
        s = ref.samples(ASSETS, frame, x0, y0, 16, 16, 0, 8)
        np.savez_compressed(os.path.join(HERE, "samples_f%04d.npz" % frame), x0=x0, y0=y0, w=16, h=16, j0=0, j1=8,
                            radiance=s[..., :3])

    # whole small frame
    acc, bgra = small.render(ASSETS, 0)
    np.savez_compressed(os.path.join(HERE, "frame_160x90.npz"), radiance=acc[..., :3], bgra=bgra)

    # scene array hashes
    hashes = {}
    for frame in (0, 450):
        with tempfile.TemporaryDirectory() as d:
            ref.dump(ASSETS, frame, d)
            hashes[str(frame)] = scene_hashes(d)
    with open(os.path.join(HERE, "scene_hashes.json"), "w") as f:
        json.dump({"config": "640x360, 32 spp, 4 bounces", "hashes": hashes}, f, indent=1)

    # the reference's committed golden frame
    rgb = validator.read_bmp("/root/reference/output/frame_0000.bmp")
    np.savez_compressed(os.path.join(HERE, "frame_0000_ref.npz"), rgb=rgb)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
