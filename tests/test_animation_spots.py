"""Every frame of a bench animation run, checked against the oracle (CPU).

`bench.py` (animation leg, BASELINE config 4 / SURVEY 8(f) row 2) renders
frames spread over the whole 1800-frame animation at the metric configuration
(1280x720, 1024 spp), writes each one as a BMP while the next renders, and
saves three 2x2 spot rectangles of every frame's averaged radiance and BGRA
bytes (`anim_spots_r<rank>.npz`).  The dumps of the committed runs live under
profiles/; this test recomputes every spot of every frame with the oracle
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
@pytest.mark.parametrize("path", DUMPS, ids=[os.path.relpath(p, ROOT) for p in DUMPS])
def test_every_animation_frame_matches_oracle(assets_dir, path):
    d = np.load(path)
    w, h, spp, bounces = int(d["width"]), int(d["height"]), int(d["spp"]), int(d["bounces"])
    frames, rects, acc_bits, bgra = d["frames"], d["rects"], d["acc_bits"], d["bgra"]
    assert len(frames) == len(rects) == len(acc_bits) == len(bgra) and len(frames) >= 3
    checked = set()
    for f in sorted(set(frames.tolist())):
        s = scene_for(assets_dir, w, h, spp, bounces, frame=f)
        orc = Oracle(arrays_copy(s), s.cfg)
        for i in np.nonzero(frames == f)[0]:
            x0, y0, rw, rh = (int(v) for v in rects[i])
            acc_o, bgra_o = orc.render_rect(x0, y0, rw, rh)
            assert np.array_equal(acc_bits[i], acc_o[..., :3].view(np.uint32)), (f, x0, y0)
            assert np.array_equal(bgra[i], bgra_o), (f, x0, y0)
        checked.add(f)
    assert len(checked) == len(set(frames.tolist()))
