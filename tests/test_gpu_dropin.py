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


DROPIN_RCCL = os.path.join(ROOT, "oracle", "_ref", "strict_160x90_s32_b4", "dropin_rccl")


@pytest.mark.parametrize("tile", [(32, 16), (48, 40)])
def test_reference_main_over_rccl_gather(assets_dir, tmp_path, tile):
    """The C++ host's multi-GPU route: the reference's own
    host code creates an RCCL communicator from RANK / WORLD_SIZE /
    LOCAL_RANK and calls ptg_render_gather (ptg_render_tiles -> ncclGather ->
    ptg_scatter_tiles, include/ptg_rccl.h).  At world size 1 on this box the
    gathered BMP equals the reference's own render byte for byte."""
    assert os.path.exists(DROPIN_RCCL), "build the drop-in first: __graft_entry__.build() (oracle/Makefile dropin_rccl)"
    out = tmp_path / "frame_0000.bmp"
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([DROPIN_RCCL, assets_dir, "0", str(out), str(tile[0]), str(tile[1])], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "rank 0 of 1" in r.stdout
    rgb = V.read_bmp(out)
    want = np.load(os.path.join(GOLDEN, "frame_160x90.npz"))["bgra"][..., [2, 1, 0]]
    assert np.array_equal(rgb, want)
