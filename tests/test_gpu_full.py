"""The GPU hot path at BASELINE.json's full size (1280x720, 256 spp, 4 bounces).

The oracle cannot render a whole 236-Msample frame in test time, so at full
size the checks are:
  * spot rectangles of the full frame vs the oracle, bit for bit - chosen at
    the image corners, the centre and across the wavefront pipeline's chunk
    boundaries (render_map splits a frame into chunks of ~2^24 paths);
  * determinism: a second render gives the same bits;
  * the reference's own acceptance test (validator.py): PSNR of the 2x
    downscaled frame 0 against its committed output/frame_0000.bmp;
  * API edges: errors instead of faults, non-default streams, per-frame
    re-upload through the scene handle.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, N, arrays_copy, scene_for
from oracle import Oracle
from ptlumi import validator as V

pytestmark = pytest.mark.gpu

W, H, SPP = 1280, 720, 256


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def full_frame(gpu, assets_dir):
    s = scene_for(assets_dir, W, H, SPP, frame=0)
    arr = arrays_copy(s)
    gpu.upload_arrays(arr)
    bgra, acc = gpu.render(s.cfg, want_accum=True)
    gpu.synchronize()
    return arr, s.cfg, bgra.cpu().numpy(), acc.cpu().numpy()


def test_full_frame_spot_rects_bit_exact(full_frame):
    arr, cfg, bgra, acc = full_frame
    orc = Oracle(arr, cfg)
    # corners, centre, and rows either side of chunk boundaries (2^24 / (1280*256) = 51.2 rows per chunk)
    rects = [(0, 0, 4, 4), (W - 4, H - 4, 4, 4), (638, 358, 4, 4), (300, 49, 4, 6), (900, 100, 4, 6),
             (1000, 614, 4, 6), (W - 4, 0, 4, 2)]
    for x0, y0, w, h in rects:
        acc_o, bgra_o = orc.render_rect(x0, y0, w, h)
        assert np.array_equal(_bits(acc[y0:y0 + h, x0:x0 + w, :3]), _bits(acc_o[..., :3])), (x0, y0)
        assert np.array_equal(bgra[y0:y0 + h, x0:x0 + w], bgra_o), (x0, y0)


def test_full_frame_deterministic(gpu, full_frame):
    arr, cfg, bgra, acc = full_frame
    bgra2, acc2 = gpu.render(cfg, want_accum=True)
    gpu.synchronize()
    assert np.array_equal(_bits(acc2.cpu().numpy()), _bits(acc))
    assert np.array_equal(bgra2.cpu().numpy(), bgra)
    assert (bgra[..., 3] == 255).all()
    assert np.isfinite(acc).all() and (acc[..., :3] >= 0).all()


def test_validator_psnr_against_reference_frame(full_frame):
    """validator.py's check: 2x-downscaled frame vs output/frame_0000.bmp.
    The reference image was made by its authors with fast-math (and with
    original terrain/bunny/tree assets the reference repository does not
    ship - see DESIGN.md), and it is a 640x360 render while the validator
    downscales our 1280x720 frame, so the comparison is statistical; the
    reference accepts >= 32 dB."""
    ref = np.load(os.path.join(GOLDEN, "frame_0000_ref.npz"))["rgb"]
    p, good = V.validate_frame(ref, full_frame[2])
    print("frame 0 PSNR vs reference output/frame_0000.bmp: %.2f dB" % p)
    assert good, "PSNR %.2f dB < %.1f dB" % (p, V.ACCEPT_MIN_PSNR)


def test_render_on_user_stream(gpu, full_frame):
    import torch
    arr, cfg, bgra, acc = full_frame
    st = torch.cuda.Stream()
    gpu.set_stream(st)
    try:
        out, _ = gpu.render(cfg, rect=(600, 300, 64, 32))
        st.synchronize()
    finally:
        gpu.set_stream(torch.cuda.default_stream())
    assert np.array_equal(out.cpu().numpy(), bgra[300:332, 600:664])


def test_errors_not_faults(gpu, assets_dir):
    s = scene_for(assets_dir, 640, 360, 32, frame=0)
    gpu.upload_arrays(arrays_copy(s))
    cfg = s.cfg
    with pytest.raises(N.PtgError, match=r"\(-6\).*rectangle"):
        gpu.render(cfg, rect=(600, 300, 64, 64))
    with pytest.raises(N.PtgError, match=r"\(-1\).*empty"):
        gpu.render(cfg, samples=(5, 5))
    with pytest.raises(N.PtgError, match=r"\(-6\)"):
        gpu.render(cfg, samples=(0, 40))                        # 5 subframes needed, the frame has 4
    with pytest.raises(N.PtgError, match=r"\(-6\)"):
        gpu.trace_rays(9, np.zeros((4, 8), np.float32))
    # a negative or -0 tmin is outside ptg_trace_rays' contract (ptg.h): refused, not traced
    for tmin in (-1.0, -0.0):
        rays = np.zeros((4, 8), np.float32)
        rays[:, 5], rays[:, 7] = 1.0, 1e9
        rays[2, 6] = tmin
        with pytest.raises(N.PtgError, match=r"\(-1\).*ray 2 .*tmin"):
            gpu.trace_rays(0, rays)
    with pytest.raises(N.PtgError, match=r"\(-6\)"):
        gpu.path_trace_samples(cfg, np.array([[640, 0]]), np.array([0]))
    with pytest.raises(N.PtgError, match=r"\(-6\)"):
        gpu.render_tiles(cfg, 32, 16, 10_000, 1, 4)
    # a TLAS leaf naming a missing instance is rejected at upload, not faulted on in the walk
    bad = arrays_copy(s)
    inst = bad["instances"]
    bad["instances"] = inst[: len(inst) // 2]
    with pytest.raises(N.PtgError, match=r"\(-6\)"):
        gpu.upload_arrays(bad, include_static=False)
    # the context stays usable
    gpu.upload_arrays(arrays_copy(s))
    out, _ = gpu.render(cfg, rect=(0, 0, 8, 8), samples=(0, 2))
    gpu.synchronize()
    assert out.shape == (8, 8, 4)


def test_frame_sequence_through_scene_handle(gpu, assets_dir):
    """main.cc's loop: setup_animation_frame + per-frame upload, static data uploaded once."""
    from ptlumi.renderer import GpuRenderer
    s = N.Scene(assets_dir, N.RenderConfig.make(320, 180, 16))
    r = GpuRenderer(0)
    try:
        rng = np.random.default_rng(5)
        for k, f in enumerate([0, 451, 1200, 1799]):
            s.setup_frame(f)
            r.upload(s, include_static=(k == 0))
            xy = np.stack([rng.integers(0, 320, 64), rng.integers(0, 180, 64)], 1).astype(np.uint32)
            js = rng.integers(0, 16, 64).astype(np.int32)
            got = r.path_trace_samples(s.cfg, xy, js)
            want = Oracle(arrays_copy(s), s.cfg).samples(xy, js)
            assert np.array_equal(_bits(got[:, :3]), _bits(want[:, :3])), f
    finally:
        r.close()


def test_reference_frame_0000_same_config(gpu, assets_dir):
    """output/frame_0000.bmp is the reference's 640x360 x 256 spp TESTING
    render of frame 0.  Rendered at that same configuration the
    GPU frame must match it to within fast-math noise: SURVEY measured ~63 dB
    for a correct renderer on the substitute scene, below ~50 dB means a
    semantic bug (RNG, camera, tonemap, BGRA order)."""
    s = scene_for(assets_dir, 640, 360, 256, frame=0)
    gpu.upload_arrays(arrays_copy(s))
    bgra, _ = gpu.render(s.cfg)
    gpu.synchronize()
    own = V.bgra_to_rgb(bgra.cpu().numpy())
    ref = np.load(os.path.join(GOLDEN, "frame_0000_ref.npz"))["rgb"]
    p = V.psnr(ref, own)
    exact = float((own == ref).all(-1).mean())
    print("frame 0 640x360x256 vs output/frame_0000.bmp: %.2f dB, %.1f%% pixels byte-exact" % (p, 100 * exact))
    assert p >= 50.0 and exact > 0.8


# BASELINE.json's other GPU configurations, through spot rectangles against the
# oracle: the metric config (1024 spp, 4 sample chunks of 256) on the light
# frame 0 and the heavy frame 450, and config 5's 3840x2160 frame with the
# dragon and the buddha in view (frame 690; 32 spp keeps the render short -
# the sample count changes only how many chunks the frame is cut into).
@pytest.mark.parametrize("w,h,spp,frame,rects", [
    (1280, 720, 1024, 0, [(0, 0, 2, 2), (640, 360, 2, 2), (1278, 718, 2, 2)]),
    (1280, 720, 1024, 450, [(100, 80, 2, 2), (700, 400, 2, 2)]),
    (3840, 2160, 32, 690, [(0, 0, 4, 4), (1900, 1000, 6, 4), (3000, 1500, 4, 4), (3836, 2156, 4, 4)]),
], ids=["metric-f0", "metric-f450", "4k-f690"])
def test_baseline_configs_spot_rects_bit_exact(gpu, assets_dir, w, h, spp, frame, rects):
    s = scene_for(assets_dir, w, h, spp, frame=frame)
    arr = arrays_copy(s)
    gpu.upload_arrays(arr)
    bgra, acc = gpu.render(s.cfg, want_accum=True)
    gpu.synchronize()
    bgra, acc = bgra.cpu().numpy(), acc.cpu().numpy()
    assert bgra.shape == (h, w, 4)
    orc = Oracle(arr, s.cfg)
    for x0, y0, rw, rh in rects:
        acc_o, bgra_o = orc.render_rect(x0, y0, rw, rh)
        assert np.array_equal(_bits(acc[y0:y0 + rh, x0:x0 + rw, :3]), _bits(acc_o[..., :3])), (x0, y0)
        assert np.array_equal(bgra[y0:y0 + rh, x0:x0 + rw], bgra_o), (x0, y0)


def test_failed_frame_upload_leaves_no_stale_records(gpu, assets_dir):
    """a frame upload that fails after its instance loop must not
    leave the packed-BLAS/mesh sets claiming records it never wrote.  Sequence:
    upload_scene (clears the sets), a frame whose TLAS names a missing instance
    (rejected after every instance was checked), then the good frame without
    the static part - which must repack and render bit-exact."""
    s = scene_for(assets_dir, 320, 180, 16, frame=450)
    arr = arrays_copy(s)
    gpu.upload_arrays(arr, include_static=True, include_frame=False)
    bad = dict(arr)
    bad["instances"] = arr["instances"][: len(arr["instances"]) // 2]
    with pytest.raises(N.PtgError, match=r"\(-6\).*TLAS.*leaf payload"):
        gpu.upload_arrays(bad, include_static=False)
    gpu.upload_arrays(arr, include_static=False)
    rect = (150, 80, 6, 4)
    _, acc = gpu.render(s.cfg, rect=rect, want_accum=True)
    gpu.synchronize()
    acc_o, _ = Oracle(arr, s.cfg).render_rect(*rect)
    assert np.array_equal(_bits(acc.cpu().numpy()[..., :3]), _bits(acc_o[..., :3]))


@pytest.mark.timeout(600)
def test_config4_full_4096spp_spot_rects_bit_exact(gpu, assets_dir):
    """BASELINE configs[4] at its full size: 3840x2160, 4096 spp (512
    subframes), frame 690 with the dragon and the buddha in view - the render
    the bench times (~70 s).  The frame's scene arrays equal the reference's
    (anim_scene_s4096_4k.json), and the spot rectangles equal, bit for bit,
    both the reference's own render of them (config4_spots.npz, the strict
    reference build at this configuration) and the oracle's."""
    import json
    from anim_check import scene_frame_hashes
    w, h, spp, frame = 3840, 2160, 4096, 690
    s = scene_for(assets_dir, w, h, spp, frame=frame)
    scenes = json.load(open(os.path.join(GOLDEN, "anim_scene_s4096_4k.json")))
    assert (scenes["width"], scenes["height"], scenes["spp"]) == (w, h, spp)
    assert scene_frame_hashes(s.view()) == scenes["frames"][str(frame)]
    arr = arrays_copy(s)
    gpu.upload_arrays(arr)
    bgra, acc = gpu.render(s.cfg, want_accum=True)
    gpu.synchronize()
    ref = np.load(os.path.join(GOLDEN, "config4_spots.npz"))
    assert (int(ref["width"]), int(ref["height"]), int(ref["spp"]), int(ref["frame"])) == (w, h, spp, frame)
    rects = [tuple(int(v) for v in r) for r in ref["rects"]]
    acc_h = acc.cpu().numpy()
    bgra_h = bgra.cpu().numpy()
    orc = Oracle(arr, s.cfg)
    k = 0
    for x0, y0, rw, rh in rects:
        got_acc = _bits(acc_h[y0:y0 + rh, x0:x0 + rw, :3])
        got_bgra = bgra_h[y0:y0 + rh, x0:x0 + rw]
        n = rw * rh
        assert np.array_equal(got_acc.reshape(-1, 3), ref["acc_bits"][k:k + n]), ("reference", x0, y0)
        assert np.array_equal(got_bgra.reshape(-1, 4), ref["bgra"][k:k + n]), ("reference", x0, y0)
        k += n
        acc_o, bgra_o = orc.render_rect(x0, y0, rw, rh)
        assert np.array_equal(got_acc, _bits(acc_o[..., :3])), ("oracle", x0, y0)
        assert np.array_equal(got_bgra, bgra_o), ("oracle", x0, y0)
    assert np.isfinite(acc_h).all() and (bgra_h[..., 3] == 255).all()
