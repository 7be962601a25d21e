"""GPU hot path vs the oracle (pt_oracle.c): bit-exact.

The oracle itself is pinned bit-for-bit to the reference renderer built from
its sources in strict IEEE mode (tests/test_oracle.py); here the HIP kernels
must reproduce the oracle exactly:
  * per-sample path_trace_pixel outputs (float32 bits) on pixel grids spread
    over the image, across frames with different content (logo intro, teapot
    close-up with a polygon aperture, buddha, vegetation, the end card);
  * the whole-frame baseline_render result (accumulated radiance bits and
    tonemapped BGRA bytes) on a small configuration;
  * ray-level closest-hit/any-hit records and tonemap_pixel.
Tolerance: none (integer/bit equality) - the kernel performs the reference's
float/double operations in the reference's order.
"""
import numpy as np
import pytest

from conftest import ASSETS, arrays_copy, scene_for
from oracle import Oracle, tonemap as oracle_tonemap

pytestmark = pytest.mark.gpu

FRAMES = [0, 300, 450, 1000, 1750]


def _grid(w, h, n, seed):
    rng = np.random.default_rng(seed)
    xs = rng.integers(0, w, n)
    ys = rng.integers(0, h, n)
    return np.stack([xs, ys], 1).astype(np.uint32)


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("frame", FRAMES)
def test_samples_bit_exact(gpu, assets_dir, frame):
    W, H, SPP = 640, 360, 32
    s = scene_for(assets_dir, W, H, SPP, frame=frame)
    arr = arrays_copy(s)
    cfg = s.cfg
    gpu.upload_arrays(arr)
    orc = Oracle(arr, cfg)
    xy = np.concatenate([_grid(W, H, 256, frame), np.array([[x, y] for y in range(170, 178) for x in range(316, 324)],
                                                            np.uint32)])
    xy = np.repeat(xy, 8, axis=0)
    js = np.tile(np.array([0, 1, 7, 8, 15, 16, 30, 31], np.int32), len(xy) // 8)
    got = gpu.path_trace_samples(cfg, xy, js)
    want = orc.samples(xy, js)
    bad = np.nonzero((_bits(got[:, :3]) != _bits(want[:, :3])).any(1))[0]
    assert len(bad) == 0, "frame %d: %d/%d samples differ, first %s: gpu %s oracle %s" % (
        frame, len(bad), len(js), xy[bad[0]].tolist() + [int(js[bad[0]])], got[bad[0]], want[bad[0]])


def test_frame_render_bit_exact(gpu, assets_dir):
    W, H, SPP = 160, 90, 32
    s = scene_for(assets_dir, W, H, SPP, frame=0)
    arr = arrays_copy(s)
    gpu.upload_arrays(arr)
    bgra, acc = gpu.render(s.cfg, want_accum=True)
    gpu.synchronize()
    acc_o, bgra_o = Oracle(arr, s.cfg).render_rect(0, 0, W, H)
    assert np.array_equal(_bits(acc.cpu().numpy()[..., :3]), _bits(acc_o[..., :3]))
    assert np.array_equal(bgra.cpu().numpy(), bgra_o)


def test_tonemap_bit_exact(gpu):
    rng = np.random.default_rng(1)
    c = np.concatenate([
        np.linspace(0, 2, 4096, dtype=np.float32)[:, None].repeat(3, 1),
        rng.exponential(0.5, (4096, 3)).astype(np.float32),
        np.array([[0, 0, 0], [1e-8, 0.0031308, 0.0031307], [1e6, 50, 3], [-1, -0.0, 2.5]], np.float32),
    ])
    got = gpu.tonemap(c)
    want = oracle_tonemap(c)
    assert np.array_equal(got, want)


def test_rays_bit_exact(gpu, assets_dir):
    W, H, SPP = 640, 360, 32
    s = scene_for(assets_dir, W, H, SPP, frame=450)
    arr = arrays_copy(s)
    gpu.upload_arrays(arr)
    rng = np.random.default_rng(7)
    n = 2048
    o = rng.uniform([-100, 0, -100], [100, 60, 100], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, np.full((n, 1), 1e-4, np.float32), np.full((n, 1), 1e9, np.float32)], 1)
    got = gpu.trace_rays(1, rays)
    want = Oracle(arr, s.cfg).trace_rays(1, rays)
    assert (want[:, 3].view(np.float32) > 0).sum() > n // 10      # the set actually hits geometry
    assert np.array_equal(got, want)


def test_pipelines_identical(gpu, assets_dir):
    """Wavefront and megakernel executions give the same bits (frame 450, 64x36 crop, 24 spp)."""
    W, H, SPP = 640, 360, 32
    s = scene_for(assets_dir, W, H, SPP, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    outs = []
    for p in ("wavefront", "megakernel"):
        gpu.set_pipeline(p)
        bgra, acc = gpu.render(s.cfg, rect=(300, 150, 64, 36), samples=(0, 24), want_accum=True)
        gpu.synchronize()
        outs.append((bgra.cpu().numpy(), acc.cpu().numpy()))
    gpu.set_pipeline("wavefront")
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(_bits(outs[0][1]), _bits(outs[1][1]))


def test_concurrency_levels_identical(gpu, assets_dir):
    """One stream, two streams, and two sample chunks in flight (the default)
    give the same bits; at 64 spp the frame is cut into two chunks, which the
    two chunk pipelines render concurrently and fold in sample order."""
    W, H, SPP = 640, 360, 64
    s = scene_for(assets_dir, W, H, SPP, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    outs = []
    for level in (0, 1, 2):
        gpu.set_concurrency(level)
        bgra, acc = gpu.render(s.cfg, want_accum=True)
        gpu.synchronize()
        outs.append((bgra.cpu().numpy(), acc.cpu().numpy()))
    gpu.set_concurrency(2)
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0])
        assert np.array_equal(_bits(outs[0][1]), _bits(o[1]))
    with pytest.raises(Exception):
        gpu.set_concurrency(3)


def test_chunks_fit_free_memory(gpu, assets_dir):
    """With most of HBM taken by another tenant (a torch tensor here), a fresh
    context sizes its chunks to what is free instead of failing, and the frame
    comes out with the same bits (more, smaller chunks fold in sample order)."""
    import torch
    from ptlumi.renderer import GpuRenderer
    W, H, SPP = 640, 360, 64
    s = scene_for(assets_dir, W, H, SPP, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    bgra0, acc0 = gpu.render(s.cfg, want_accum=True)
    gpu.synchronize()
    want = (bgra0.cpu().numpy(), acc0.cpu().numpy())
    del bgra0, acc0
    free, _ = torch.cuda.mem_get_info()
    hog = torch.empty(max(0, free - (6 << 30)), dtype=torch.uint8, device="cuda:0")
    r = GpuRenderer(0)
    try:
        r.upload_arrays(arrays_copy(s))
        bgra, acc = r.render(s.cfg, want_accum=True)
        r.synchronize()
        assert np.array_equal(want[0], bgra.cpu().numpy())
        assert np.array_equal(_bits(want[1]), _bits(acc.cpu().numpy()))
        del bgra, acc
    finally:
        r.close()
        del hog
        torch.cuda.empty_cache()


@pytest.mark.parametrize("w,h,spp,bounces,frame,rect,samples", [
    (67, 43, 13, 4, 300, None, None),            # ragged image, spp not a multiple of the 8-sample group
    (33, 17, 5, 0, 450, None, None),             # camera ray + sky/shading only, no bounce
    (50, 29, 9, 1, 1000, (7, 3, 31, 19), None),  # one bounce, a rectangle off the origin
    (41, 23, 24, 7, 1750, None, (3, 21)),        # deep paths, a sample range across group borders
])
def test_ragged_configs_bit_exact(gpu, assets_dir, w, h, spp, bounces, frame, rect, samples):
    """Sizes, sample counts and bounce limits off the power-of-two grid the
    kernels tile by: the accumulated radiance bits and BGRA bytes equal the
    oracle's baseline_render over the same rectangle and sample range."""
    s = scene_for(assets_dir, w, h, spp, bounces=bounces, frame=frame)
    arr = arrays_copy(s)
    gpu.upload_arrays(arr)
    x0, y0, rw, rh = rect if rect else (0, 0, w, h)
    j0, j1 = samples if samples else (0, spp)
    bgra, acc = gpu.render(s.cfg, rect=rect, samples=samples, want_accum=True)
    gpu.synchronize()
    acc_o, bgra_o = Oracle(arr, s.cfg).render_rect(x0, y0, rw, rh, j0, j1)
    assert np.array_equal(_bits(acc.cpu().numpy()[..., :3]), _bits(acc_o[..., :3]))
    assert np.array_equal(bgra.cpu().numpy(), bgra_o)


def _nan_aware_equal(a, b):
    """Bit equality, with any NaN equal to any NaN (x86 and gfx950 quiet NaNs
    carry different sign/payload bits)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(_bits(np.where(na, 0, a)), _bits(np.where(nb, 0, b)))


@pytest.mark.parametrize("color,cos", [
    ((float("nan"), 4.0, 4.0), None),        # a NaN colour component without its sign bit
    ((1e37, 1e37, 1e37), None),              # finite, but colour x the sun disk's pdf overflows
    ((3e38, 2.0, 1.0), None),                # near FLT_MAX: colour / mis_pdf overflows
    ((float("inf"), 4.0, 4.0), None),
    ((4.0, 4.0, 4.0), 1.0),                  # degenerate sun cone: the disk's pdf is infinite
])
def test_unvalidated_light_takes_no_shortcut(gpu, assets_dir, color, cos):
    """the zero-throughput shortcuts (untraced moot shadow rays,
    the skipped sky integrals, the retired last bounce) are exact only when
    the term they skip is finite.  A light uploaded through ptg_upload_frame
    is not validated, so a NaN, infinite or huge colour, or a cone of cos 1,
    must take the full computation: the frame equals the oracle's (NaN where
    it has NaN)."""
    W, H, SPP = 48, 27, 16
    s = scene_for(assets_dir, W, H, SPP, frame=450)
    arr = arrays_copy(s)
    arr["subframes"]["light"]["color"][:, :3] = np.array(color, np.float32)
    if cos is not None:
        arr["subframes"]["light"]["cos_solid_angle"] = np.float32(cos)
    gpu.upload_arrays(arr)
    bgra, acc = gpu.render(s.cfg, want_accum=True)
    gpu.synchronize()
    acc_o, bgra_o = Oracle(arr, s.cfg).render_rect(0, 0, W, H)
    got = acc.cpu().numpy()[..., :3]
    assert _nan_aware_equal(got, acc_o[..., :3])
    fin = ~np.isnan(got).any(-1)
    assert np.array_equal(bgra.cpu().numpy()[fin], bgra_o[fin])
