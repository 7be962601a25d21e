"""Drop-in proof: the reference's own host code (load_scene /
setup_animation_frame / write_bmp, compiled unmodified from its sources)
with baseline_render's body replaced by the C-ABI calls of INTEGRATION.md
(oracle/dropin_main.cc) writes the same BMP bytes as the reference renderer
itself (tests/golden/frame_160x90.npz, made by the reference's own
baseline_render semantics, strict IEEE build)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from ptlumi import validator as V

pytestmark = pytest.mark.gpu

DROPIN = os.path.join(ROOT, "oracle", "_ref", "strict_160x90_s32_b4", "dropin")


def test_reference_main_with_gpu_baseline_render(assets_dir, tmp_path):
    assert os.path.exists(DROPIN), "build the drop-in first: __graft_entry__.build() (oracle/Makefile dropin)"
    out = tmp_path / "frame_0000.bmp"
    r = subprocess.run([DROPIN, assets_dir, "0", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rgb = V.read_bmp(out)
    want = np.load(os.path.join(GOLDEN, "frame_160x90.npz"))["bgra"][..., [2, 1, 0]]
    assert np.array_equal(rgb, want)
