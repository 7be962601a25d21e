"""The committed whole-animation measurement (tools/full_animation.py, four
parts of 450 frames on one MI355X, summed by tools/full_animation_sum.py):
every frame 0..1799 rendered once at 1280x720 x 1024 spp, and the two frames
whose whole images are pinned to the reference's strict build
(full_render_s1024.json) came out with the reference's BGRA hash."""
import json
import os

from conftest import GOLDEN, ROOT

REC = os.path.join(ROOT, "profiles", "r06k_full_animation", "full_animation.json")


def test_full_animation_record():
    r = json.load(open(REC))
    assert r["config"] == {"width": 1280, "height": 720, "spp": 1024, "bounces": 4}
    assert r["frames"] == 1800 and len(r["bgra_sha"]) == 1800
    assert abs(r["frames_per_min"] - 1800 / r["wall_s"] * 60.0) < 1e-2
    g = json.load(open(os.path.join(GOLDEN, "full_render_s1024.json")))["frames"]
    for f in ("0", "450"):
        assert r["bgra_sha"][int(f)] == g[f]["sha_bgra"][:16]
