#!/usr/bin/env python3
"""Whole-animation fixtures from the REFERENCE built from its own sources.

The reference harness (oracle/ref_harness.cc, strict IEEE build of
/root/reference's scene.cc / bvh.cc / mesh.cc / main.cc / path_tracer.hh) is
run over every one of the 1800 animation frames (scene.cc:720-724):

  anim_scene_s1024.json  per frame: SHA-256 of instances, subframes, the 128
                         subframe TLASes' nodes and links at 1280x720, 1024 spp
                         (setup_animation_frame, scene.cc:271-718; the subframe
                         timestamps frame + i/128, scene.cc:648-661)
  anim_scene_s32.json    the same at 640x360, 32 spp (4 subframes)
  anim_scene_s8.json     the same at 160x90, 8 spp (1 subframe)
  anim_render_s8.json    per frame: SHA-256 of the whole 160x90 x 8 spp image,
                         radiance bits after /SPP and BGRA (baseline_render,
                         main.cc:12-46)
  anim_scene_s256.json   the same at 1280x720, 256 spp (32 subframes)
  anim_scene_s4096_4k.json  the same at 3840x2160, 4096 spp (512 subframes) over
                         frames 660-720 (BASELINE configs[4]: dragon + buddha fly-by)
  full_render_s1024.json whole 1280x720 x 1024 spp images of frames 0 and 450 (the
                         bench's metric frame and its heavy companion), hashed as
                         anim_render_s8.json: radiance bits after /SPP and BGRA
  config4_spots.npz      the spot rectangles tests/test_gpu_full.py checks at BASELINE
                         configs[4]'s full size (3840x2160 x 4096 spp, frame 690)
  bench_spots.npz        the spot rectangles bench.py checks after its
                         animation leg (bench.spot_rects over the 16-frame and
                         the 30-frame picks) at 1280x720 x 1024 spp: radiance
                         bits + BGRA

Hashes are truncated to their first 32 hex digits (128 bits).  The padding
words of the 160-byte records are excluded as in make_golden.py.

Needs /root/reference (this container only).  Takes ~1-2 h on 8 cores.
Usage: python tests/golden/make_anim_golden.py [scene1024 scene32 scene8 render8 spots scene256 scene4k full1024 spots4k]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import Reference  # noqa: E402

ASSETS = os.path.join(ROOT, "assets")
FRAMES = 1800
DIGITS = 32


def ensure(mode, w, h, spp):
    ref = Reference(mode, w, h, spp, 4)
    if not ref.available():
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref", "REF_MODE=" + mode,
                               "REF_W=%d" % w, "REF_H=%d" % h, "REF_SPP=%d" % spp, "REF_BOUNCES=4"])
    return ref


def run_lines(ref, cmd, f0, f1):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.txt")
        ref.run(ASSETS, cmd, f0, f1, out, timeout=24 * 3600)
        return [l.split() for l in open(out)]


def scene_hashes(w, h, spp, name, f0=0, f1=FRAMES):
    ref = ensure("strict", w, h, spp)
    rows = run_lines(ref, "anim_hashes", f0, f1)
    assert len(rows) == f1 - f0
    frames = {}
    for r in rows:
        frames[r[0]] = {"instances": int(r[1]), "subframes": int(r[2]), "tlas_nodes": int(r[3]),
                        "sha_instances": r[5][:DIGITS], "sha_subframes": r[6][:DIGITS],
                        "sha_tlas_nodes": r[7][:DIGITS], "sha_tlas_links": r[8][:DIGITS]}
    doc = {"config": "%dx%d, %d spp, 4 bounces" % (w, h, spp), "width": w, "height": h, "spp": spp,
           "static_nodes": int(rows[0][4]), "frames": frames,
           "source": "reference strict build, ref_pt anim_hashes %d %d (load_scene once, then "
                     "setup_animation_frame for every frame in order)" % (f0, f1)}
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)


def render_hashes(w, h, spp, name):
    ref = ensure("strict", w, h, spp)
    rows = run_lines(ref, "anim_render", 0, FRAMES)
    assert len(rows) == FRAMES
    doc = {"config": "%dx%d, %d spp, 4 bounces" % (w, h, spp), "width": w, "height": h, "spp": spp,
           "frames": {r[0]: {"sha_radiance": r[1][:DIGITS], "sha_bgra": r[2][:DIGITS]} for r in rows},
           "source": "reference strict build, ref_pt anim_render 0 %d: baseline_render semantics over the whole "
                     "image, radiance = float32 xyz after /SPP ([H][W][3]), BGRA [H][W][4]" % FRAMES}
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)


def full_render_hashes(w, h, spp, frames, name):
    """Whole images at a full BASELINE size, one ref_pt anim_render run per frame
    (load_scene + setup_animation_frame(frame), then baseline_render semantics)."""
    ref = ensure("strict", w, h, spp)
    out = {}
    for f in frames:
        rows = run_lines(ref, "anim_render", f, f + 1)
        assert len(rows) == 1 and int(rows[0][0]) == f
        out[str(f)] = {"sha_radiance": rows[0][1][:DIGITS], "sha_bgra": rows[0][2][:DIGITS]}
        print("frame", f, out[str(f)], flush=True)
    doc = {"config": "%dx%d, %d spp, 4 bounces" % (w, h, spp), "width": w, "height": h, "spp": spp, "frames": out,
           "source": "reference strict build, ref_pt anim_render f f+1 per frame: baseline_render semantics over the "
                     "whole image, radiance = float32 xyz after /SPP ([H][W][3]), BGRA [H][W][4]"}
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)


CONFIG4_RECTS = [(0, 0, 2, 2), (1900, 1000, 4, 4), (3000, 1500, 4, 2), (2400, 1200, 2, 4), (3836, 2158, 4, 2)]


def config4_spots():
    """BASELINE configs[4] at full size (3840x2160 x 4096 spp, frame 690): the
    spot rectangles tests/test_gpu_full.py checks, rendered by the reference."""
    w, h, spp, frame = 3840, 2160, 4096, 690
    ref = ensure("strict", w, h, spp)
    rects = [(frame,) + r for r in CONFIG4_RECTS]
    with tempfile.TemporaryDirectory() as d:
        i, o = os.path.join(d, "in.txt"), os.path.join(d, "out.bin")
        with open(i, "w") as fh:
            for r in rects:
                fh.write("%d %d %d %d %d\n" % r)
        ref.run(ASSETS, "spots", i, o, timeout=24 * 3600)
        raw = np.fromfile(o, np.uint32).reshape(-1, 4)
    acc, bgra, k = [], [], 0
    for (_, _, _, rw, rh) in rects:
        blk = raw[k:k + rw * rh]
        k += rw * rh
        acc.append(blk[:, :3].reshape(rh, rw, 3).copy())
        bgra.append(blk[:, 3:].copy().view(np.uint8).reshape(rh, rw, 4))
    assert k == len(raw)
    np.savez_compressed(os.path.join(HERE, "config4_spots.npz"), frame=frame,
                        rects=np.array([r[1:] for r in rects], np.int32),
                        acc_bits=np.concatenate([a.reshape(-1, 3) for a in acc]),
                        bgra=np.concatenate([b.reshape(-1, 4) for b in bgra]), width=w, height=h, spp=spp, bounces=4)


def bench_spots():
    import bench
    w, h, spp = 1280, 720, 1024
    ref = ensure("strict", w, h, spp)
    picks = sorted(set(round(i * FRAMES / k) % FRAMES for k in (16, 30) for i in range(k)))
    rects = [(f,) + tuple(r) for f in picks for r in bench.spot_rects(f, w, h)]
    with tempfile.TemporaryDirectory() as d:
        i, o = os.path.join(d, "in.txt"), os.path.join(d, "out.bin")
        with open(i, "w") as fh:
            for r in rects:
                fh.write("%d %d %d %d %d\n" % r)
        ref.run(ASSETS, "spots", i, o, timeout=24 * 3600)
        raw = np.fromfile(o, np.uint32).reshape(-1, 4)
    per = [rw * rh for (_, _, _, rw, rh) in rects]
    assert sum(per) == len(raw)
    acc, bgra, k = [], [], 0
    for (_, _, _, rw, rh) in rects:
        blk = raw[k:k + rw * rh]
        k += rw * rh
        acc.append(blk[:, :3].reshape(rh, rw, 3))
        bgra.append(blk[:, 3:].copy().view(np.uint8).reshape(rh, rw, 4))
    np.savez_compressed(os.path.join(HERE, "bench_spots.npz"), frames=np.array([r[0] for r in rects], np.int32),
                        rects=np.array([r[1:] for r in rects], np.int32), acc_bits=np.array(acc, np.uint32),
                        bgra=np.array(bgra, np.uint8), width=w, height=h, spp=spp, bounces=4)


def main():
    jobs = sys.argv[1:] or ["scene1024", "scene32", "scene8", "render8", "spots"]
    for j in jobs:
        print("==", j, flush=True)
        if j == "scene1024":
            scene_hashes(1280, 720, 1024, "anim_scene_s1024.json")
        elif j == "scene32":
            scene_hashes(640, 360, 32, "anim_scene_s32.json")
        elif j == "scene8":
            scene_hashes(160, 90, 8, "anim_scene_s8.json")
        elif j == "render8":
            render_hashes(160, 90, 8, "anim_render_s8.json")
        elif j == "spots":
            bench_spots()
        elif j == "scene256":
            scene_hashes(1280, 720, 256, "anim_scene_s256.json")
        elif j == "scene4k":
            scene_hashes(3840, 2160, 4096, "anim_scene_s4096_4k.json", 660, 721)
        elif j == "spots4k":
            config4_spots()
        elif j == "full1024":
            full_render_hashes(1280, 720, 1024, [0, 450], "full_render_s1024.json")
        else:
            raise SystemExit("unknown job " + j)


if __name__ == "__main__":
    main()
