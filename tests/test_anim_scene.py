"""Every frame of the animation, pinned to the reference.

setup_animation_frame (scene.cc:271-718) makes ceil(SPP/8) subframes per
frame with timestamps frame + i/n (scene.cc:648-661), so the per-frame
arrays depend on the sample count.  The reference built from its own
sources (tests/golden/make_anim_golden.py) hashed the instances, subframes
and subframe TLAS nodes/links of all 1800 frames at 8, 32, 256 and 1024 spp
(1, 4, 32 and 128 subframes; 1280x720 for 256 and 1024: the camera's aspect
ratio depends on W/H, scene.cc:284) and of frames 660-720 at BASELINE
configs[4]'s 3840x2160 x 4096 spp (512 subframes, the dragon + buddha
fly-by); the host restatement (csrc/host/scene.cpp,
data/animation_track.csv) must produce the very same bytes for every frame.
The frames are set up in order in one scene per worker, as the reference
harness did; test_scene_parity.py covers fresh loads.
"""
import json
import multiprocessing as mp
import os

import pytest

from anim_check import scene_hash_range
from conftest import GOLDEN, ROOT

# golden file -> (W, H, SPP, first frame, frames)
CONFIGS = {"s8": (160, 90, 8, 0, 1800), "s32": (640, 360, 32, 0, 1800), "s256": (1280, 720, 256, 0, 1800),
           "s1024": (1280, 720, 1024, 0, 1800), "s4096_4k": (3840, 2160, 4096, 660, 61)}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_every_frame_scene_arrays_match_reference(assets_dir, name):
    w, h, spp, f0, n = CONFIGS[name]
    golden = json.load(open(os.path.join(GOLDEN, "anim_scene_%s.json" % name)))
    assert (golden["width"], golden["height"], golden["spp"]) == (w, h, spp)
    frames = len(golden["frames"])
    assert frames == n and min(int(f) for f in golden["frames"]) == f0
    workers = max(1, min(8, os.cpu_count() or 1))
    cuts = [f0 + n * k // workers for k in range(workers + 1)]
    with mp.get_context("spawn").Pool(workers) as pool:
        parts = pool.map(scene_hash_range, [(ROOT, w, h, spp, cuts[k], cuts[k + 1]) for k in range(workers)])
    got = {}
    for p in parts:
        got.update(p)
    assert len(got) == frames
    bad = [(f, k) for f in sorted(golden["frames"], key=int) for k, v in golden["frames"][f].items() if got[f][k] != v]
    assert not bad, "%d frame/array mismatches, first %s" % (len(bad), bad[:10])
