"""The reference's plugin functions with their own signatures on the GPU
(include/ptg_device.h, verdict r1 item 4).

A user kernel (tests/device_dropin/user_kernel.hip, built against
ptg_device.h alone) calls

    path_trace_pixel(uint2 xy, int sample_index, const subframe*, const tlas_instance*,
                     const bvh_node*, const bvh_link*, const uint*, const float3*,
                     const float3*, const float4*, const float4*)   path_tracer.hh:637-654
    tonemap_pixel(float3)                                           path_tracer.hh:753

over the REFERENCE-LAYOUT arrays (the scene's own nodes / 8 link orders /
indices / positions ..., no repacking) in device memory.  Its outputs must
equal, bit for bit, the reference's own outputs stored in the golden fixtures
(tests/golden/samples_f*.npz: path_trace_pixel of the strict reference build
over 16x16 pixels x 8 samples of frames 0, 450 and 1750; tonemap.npz) and the
oracle on further samples.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, arrays_copy, scene_for
from oracle import Oracle

LIB = os.path.join(ROOT, "tests", "device_dropin", "_build", "libuser_kernel.so")


def _lib():
    assert os.path.exists(LIB), "build it first: __graft_entry__.build() (tests/device_dropin/Makefile)"
    L = C.CDLL(LIB)
    P, U32 = C.c_void_p, C.c_uint32
    L.user_path_trace.argtypes = [P, U32, P, P] + [P] * 9 + [P]
    L.user_path_trace.restype = C.c_int
    L.user_tonemap_device.argtypes = [U32, P, P]
    L.user_tonemap_device.restype = C.c_int
    L.user_tonemap_host.argtypes = [U32, P, P]
    L.user_tonemap_host.restype = None
    return L


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_host_tonemap_pixel_matches_reference(native_lib):
    """tonemap_pixel called on the host (no GPU work) == the reference's bytes."""
    g = np.load(os.path.join(GOLDEN, "tonemap.npz"))
    colors = np.ascontiguousarray(g["colors"], np.float32)
    out = np.zeros((len(colors), 4), np.uint8)
    _lib().user_tonemap_host(len(colors), colors.ctypes.data, out.ctypes.data)
    assert np.array_equal(out, g["bgra"])


def _device_arrays(arr):
    import torch
    keys = ["subframes", "instances", "nodes", "links", "indices", "pos", "normal", "albedo", "material"]
    dev = {}
    for k in keys:
        a = np.ascontiguousarray(arr[k])
        dev[k] = torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to("cuda:0")
    return dev, [C.c_void_p(dev[k].data_ptr()) for k in keys]


def _run_samples(L, arrays, cfg, xy, js):
    import torch
    dev, ptrs = _device_arrays(arrays)
    xy_d = torch.from_numpy(np.ascontiguousarray(xy, np.uint32)).to("cuda:0")
    js_d = torch.from_numpy(np.ascontiguousarray(js, np.int32)).to("cuda:0")
    out = torch.zeros((len(js), 4), dtype=torch.float32, device="cuda:0")
    rc = L.user_path_trace(C.byref(cfg), len(js), C.c_void_p(xy_d.data_ptr()), C.c_void_p(js_d.data_ptr()), *ptrs,
                           C.c_void_p(out.data_ptr()))
    assert rc == 0
    return out.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("frame", [0, 450, 1750])
def test_path_trace_pixel_signature_matches_reference_goldens(assets_dir, frame):
    g = np.load(os.path.join(GOLDEN, "samples_f%04d.npz" % frame))
    x0, y0, w, h, j0, j1 = (int(g[k]) for k in ("x0", "y0", "w", "h", "j0", "j1"))
    s = scene_for(assets_dir, 640, 360, 32, frame=frame)
    arr = arrays_copy(s)
    yy, xx, jj = np.meshgrid(np.arange(y0, y0 + h), np.arange(x0, x0 + w), np.arange(j0, j1), indexing="ij")
    xy = np.stack([xx.reshape(-1), yy.reshape(-1)], 1).astype(np.uint32)
    js = jj.reshape(-1).astype(np.int32)
    got = _run_samples(_lib(), arr, s.cfg, xy, js)
    want = g["radiance"].reshape(-1, 3)
    bad = np.nonzero((_bits(got[:, :3]) != _bits(want)).any(1))[0]
    assert len(bad) == 0, "frame %d: %d/%d samples differ" % (frame, len(bad), len(js))


@pytest.mark.gpu
def test_path_trace_pixel_signature_matches_oracle_hexagon_aperture(assets_dir):
    """Frame 300: the teapot close-up with the hexagonal aperture (the camera's
    polygon branch, evaluated in-line here rather than from the frame
    renderer's table) and motion blur across subframes."""
    s = scene_for(assets_dir, 640, 360, 32, frame=300)
    arr = arrays_copy(s)
    rng = np.random.default_rng(300)
    xy = np.stack([rng.integers(0, 640, 512), rng.integers(0, 360, 512)], 1).astype(np.uint32)
    js = rng.integers(0, 32, 512).astype(np.int32)
    got = _run_samples(_lib(), arr, s.cfg, xy, js)
    want = Oracle(arr, s.cfg).samples(xy, js)
    assert np.array_equal(_bits(got[:, :3]), _bits(want[:, :3]))


@pytest.mark.gpu
def test_device_tonemap_pixel_matches_reference():
    import torch
    g = np.load(os.path.join(GOLDEN, "tonemap.npz"))
    colors = torch.from_numpy(np.ascontiguousarray(g["colors"], np.float32)).to("cuda:0")
    out = torch.zeros((len(colors), 4), dtype=torch.uint8, device="cuda:0")
    assert _lib().user_tonemap_device(len(colors), C.c_void_p(colors.data_ptr()), C.c_void_p(out.data_ptr())) == 0
    assert np.array_equal(out.cpu().numpy(), g["bgra"])


@pytest.mark.gpu
def test_device_selftest_passes(native_lib):
    """ptg_device_selftest() (ptg_device.h), compiled with the documented
    flags in the user's library: every known-answer check passes."""
    L = _lib()
    L.user_selftest.restype = C.c_int
    assert L.user_selftest() == 0


@pytest.mark.gpu
def test_device_selftest_flags_contraction(native_lib):
    """The same user code built with -ffp-contract=fast: the self-test reports
    the contraction (bit 0) instead of passing silently."""
    path = os.path.join(ROOT, "tests", "device_dropin", "_build", "libuser_kernel_contract.so")
    assert os.path.exists(path), "build it first: __graft_entry__.build() (tests/device_dropin/Makefile)"
    L = C.CDLL(path)
    L.user_selftest.restype = C.c_int
    r = L.user_selftest()
    assert r > 0 and (r & 1), r


LIB_2TU = os.path.join(ROOT, "tests", "device_dropin", "_build", "libuser_kernel_2tu.so")


def test_two_translation_units_link():
    """A user library whose two .hip files both include ptg_device.h links
    (the header's definitions are inline or internal), and exports both TUs'
    entry points (no GPU work)."""
    assert os.path.exists(LIB_2TU), "build it first: __graft_entry__.build() (tests/device_dropin/Makefile)"
    L = C.CDLL(LIB_2TU)
    for sym in ("user_selftest", "user_selftest_tu2", "user_tonemap_device", "user_tonemap_device_tu2"):
        assert hasattr(L, sym), sym


@pytest.mark.gpu
def test_two_translation_units_selftest_and_tonemap():
    """Both translation units' copies of the header run: each self-test passes
    and each TU's tonemap_pixel kernel gives the reference's bytes."""
    import torch
    L = C.CDLL(LIB_2TU)
    L.user_selftest.restype = C.c_int
    L.user_selftest_tu2.restype = C.c_int
    assert L.user_selftest() == 0
    assert L.user_selftest_tu2() == 0
    g = np.load(os.path.join(GOLDEN, "tonemap.npz"))
    colors = torch.from_numpy(np.ascontiguousarray(g["colors"], np.float32)).to("cuda:0")
    for fn in (L.user_tonemap_device, L.user_tonemap_device_tu2):
        fn.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p]
        fn.restype = C.c_int
        out = torch.zeros((len(colors), 4), dtype=torch.uint8, device="cuda:0")
        assert fn(len(colors), C.c_void_p(colors.data_ptr()), C.c_void_p(out.data_ptr())) == 0
        assert np.array_equal(out.cpu().numpy(), g["bgra"])
