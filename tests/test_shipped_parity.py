"""How far the reference AS SHIPPED (-O3 -ffast-math, Makefile:2) is from its
strict-IEEE build - which the GPU path reproduces bit for bit - on the SURVEY
8(c) tiers (tests/golden/parity_stats.py; the whole-frame numbers are
committed in tests/golden/parity_stats.json and quoted in DESIGN.md).

Here a 16-row band of frames 0 and 450 (640x360 x 32 spp) is recomputed from
both reference builds and held to the tier bars: T2 image mean within 5e-3
relative per channel, T3 PSNR >= 32 dB (validator.py's acceptance)."""
import json
import os

import pytest

from conftest import GOLDEN
from oracle import Reference

import importlib.util

_spec = importlib.util.spec_from_file_location("parity_stats", os.path.join(GOLDEN, "parity_stats.py"))
PS = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(PS)


def _builds_present():
    return all(Reference(m, PS.W, PS.H, PS.SPP, PS.BOUNCES).available() for m in ("strict", "v3"))


def test_committed_whole_frame_stats_meet_tiers():
    res = json.load(open(os.path.join(GOLDEN, "parity_stats.json")))
    assert [f["frame"] for f in res["frames"]] == [0, 450]
    for f in res["frames"]:
        assert f["rows"] == [0, PS.H] and f["pixels"] == PS.W * PS.H
        assert max(f["T2_image_mean_rel_diff"]) < 5e-3
        assert f["T3_psnr_db"] >= 32.0
        assert 0.0 < f["T1_samples_within_1e-4"] < 1.0      # the builds differ; GPU == strict exactly


def test_committed_metric_config_stats():
    """The same tiers at the metric configuration's image (1280x720, 256 and
    1024 spp; parity_stats.py --metric).  What holds there:
    validator.py's own acceptance (PSNR of the 2x-downscaled frames >= 32 dB)
    and the image means within 5e-3; "accumulated radiance within 1e-4
    relative" holds for a minority of frame 450's pixels and falls with SPP
    (a pixel with more samples has more chances that one of its paths takes
    another branch under fast-math), which DESIGN.md section 2 reports."""
    res = json.load(open(os.path.join(GOLDEN, "parity_stats.json")))["metric_config"]
    assert (res["width"], res["height"]) == (1280, 720)
    rows = {(r["frame"], r["spp"]): r for r in res["rows"]}
    assert (0, 256) in rows and (450, 256) in rows
    for r in rows.values():
        assert r["pixels"] == 1280 * 720
        assert r["T3v_validator_good"] and r["T3v_validator_psnr_db"] >= 32.0
        assert r["T3_psnr_db"] >= 32.0
        assert max(r["T2_image_mean_rel_diff"]) < 5e-3
        assert 0.5 < r["T1_samples_within_1e-4"] < 1.0
    # more samples per pixel: fewer pixels within 1e-4 (frame 450: 49% at 32 spp, 640x360)
    small = {f["frame"]: f for f in json.load(open(os.path.join(GOLDEN, "parity_stats.json")))["frames"]}
    assert rows[(450, 256)]["T2_pixels_within_1e-4"] < small[450]["T2_pixels_within_1e-4"]


def test_committed_frame450_metric_spp_row():
    """Frame 450 at the metric's own 1280x720 x 1024 spp (VERDICT r05 item 4;
    parity_stats.py --metric --spp 1024, ~2.5 CPU hours for the two builds):
    validator.py's acceptance holds; the tier-2 fractions keep falling with
    SPP; and both reference builds carry exactly one NaN pixel - a path that
    met a zero BSDF pdf (path_tracer.hh:735-737) - which the image means and
    the median leave out.  The strict build's NaN pixel is pinned by location
    in full_render_s1024.json, where the GPU's whole frame 450 (hash-equal to
    that build) is checked to carry it (tests/test_gpu_full_frames.py)."""
    res = json.load(open(os.path.join(GOLDEN, "parity_stats.json")))["metric_config"]
    r = {(x["frame"], x["spp"]): x for x in res["rows"]}[(450, 1024)]
    assert r["pixels"] == 1280 * 720
    assert r["T3v_validator_good"] and r["T3v_validator_psnr_db"] >= 32.0 and r["T3_psnr_db"] >= 32.0
    assert r["nan_pixels_strict"] == 1 and r["nan_pixels_shipped"] == 1
    assert all(x == x for x in r["T2_image_mean_rel_diff"]) and max(r["T2_image_mean_rel_diff"]) < 5e-3
    assert r["T2_median_rel_diff"] == r["T2_median_rel_diff"]          # not NaN
    assert r["T2_pixels_within_1e-4"] < {(x["frame"], x["spp"]): x for x in res["rows"]}[(450, 256)]["T2_pixels_within_1e-4"]
    full = json.load(open(os.path.join(GOLDEN, "full_render_s1024.json")))
    assert full["frames"]["450"]["nan_pixels_yx"] == [[159, 97]]


@pytest.mark.skipif(not _builds_present(), reason="reference builds not present (build())")
@pytest.mark.parametrize("frame", [0, 450])
def test_band_strict_vs_shipped(assets_dir, frame):
    st = PS.frame_stats(assets_dir, frame, 170, 186)
    print(json.dumps(st))
    assert max(st["T2_image_mean_rel_diff"]) < 5e-3
    assert st["T3_psnr_db"] >= 32.0
    assert st["T1_samples_within_1e-4"] > 0.5


def test_shipped_band_fixture_matches_committed_rows():
    """The fixture the GPU test recomputes against (make_shipped_band.py):
    its strict-vs-shipped validator PSNR is the committed whole-frame row's,
    and its arrays have the shapes the GPU test reads."""
    import numpy as np
    fx = json.load(open(os.path.join(GOLDEN, "shipped_band_s1024.json")))
    arr = np.load(os.path.join(GOLDEN, "shipped_band_s1024.npz"))
    rows = {(r["frame"], r["spp"]): r for r in json.load(open(os.path.join(GOLDEN, "parity_stats.json")))["metric_config"]["rows"]}
    y0, y1 = fx["band_rows"]
    for f in (0, 450):
        st = fx["frames"][str(f)]
        assert st["T3v_validator_good"] and max(st["band_mean_rel_diff"]) < 5e-3
        if (f, 1024) in rows:
            assert st["T3v_validator_psnr_db"] == rows[(f, 1024)]["T3v_validator_psnr_db"]
        assert arr["shipped_half_f%d" % f].shape == (fx["height"] // 2, fx["width"] // 2, 3)
        assert arr["shipped_band_f%d" % f].shape == (y1 - y0, fx["width"], 3)
        assert arr["shipped_bgra_band_f%d" % f].shape == (y1 - y0, fx["width"], 4)
