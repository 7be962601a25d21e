"""Every frame of a bench animation run, checked against the oracle (CPU).

`bench.py` (animation leg, BASELINE config 4 / SURVEY 8(f) row 2) renders
frames spread over the whole 1800-frame animation at the metric configuration
(1280x720, 1024 spp), writes each one as a BMP while the next renders, and
saves three 2x2 spot rectangles of every frame's averaged radiance and BGRA
bytes (`anim_spots_r<rank>.npz`).  The dumps of the committed runs live under
profiles/; this test recomputes every spot of every frame with the oracle (each
distinct frame and rectangle once across the dumps)
(pt_oracle.c, pinned to the reference build) and requires bit equality -
per-frame validation of the animation without re-rendering it on the CPU.
"""
import glob
import os

import numpy as np
import pytest

from conftest import ROOT, arrays_copy, scene_for
from oracle import Oracle

DUMPS = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "anim_spots_r*.npz")))


@pytest.mark.skipif(not DUMPS, reason="no committed animation spot dump under profiles/")
def test_every_animation_frame_matches_oracle(assets_dir):
    """Every spot of every committed dump; the dumps of several runs share
    frames (the bench's sample), so each (configuration, frame) is set up once
    and each rectangle rendered by the oracle once, whatever dump holds it."""
    groups = {}   # (w, h, spp, bounces) -> frame -> [(dump, rect, radiance bits, bgra)]
    for path in DUMPS:
        d = np.load(path)
        key = (int(d["width"]), int(d["height"]), int(d["spp"]), int(d["bounces"]))
        frames, rects, acc_bits, bgra = d["frames"], d["rects"], d["acc_bits"], d["bgra"]
        assert len(frames) == len(rects) == len(acc_bits) == len(bgra) and len(frames) >= 3, path
        g = groups.setdefault(key, {})
        for f, rc, a, b in zip(frames.tolist(), rects, acc_bits, bgra):
            g.setdefault(int(f), []).append((os.path.relpath(path, ROOT), tuple(int(v) for v in rc), a, b))
    checked = 0
    for (w, h, spp, bounces), g in sorted(groups.items()):
        for f in sorted(g):
            s = scene_for(assets_dir, w, h, spp, bounces, frame=f)
            orc = Oracle(arrays_copy(s), s.cfg)
            ref = {}
            for path, rc, a, b in g[f]:
                if rc not in ref:
                    ref[rc] = orc.render_rect(*rc)
                acc_o, bgra_o = ref[rc]
                assert np.array_equal(a, acc_o[..., :3].view(np.uint32)), (path, f, rc)
                assert np.array_equal(b, bgra_o), (path, f, rc)
                checked += 1
    assert checked == sum(len(np.load(p)["frames"]) for p in DUMPS)
