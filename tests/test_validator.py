"""validator.py-equivalent checks (numpy) and the BMP output path (bmp.cc)."""
import os

import numpy as np

from conftest import GOLDEN, N
from ptlumi import validator as V


def test_downscale_is_truncated_block_mean():
    img = np.arange(4 * 6 * 3, dtype=np.uint8).reshape(4, 6, 3)
    out = V.downscale_half(img)
    want = img.astype(np.float64).reshape(2, 2, 3, 2, 3).mean(axis=(1, 3)).astype(np.uint8)
    assert out.shape == (2, 3, 3) and np.array_equal(out, want)
    # truncation, not rounding: mean 0.75 -> 0
    assert V.downscale_half(np.array([[[1], [1]], [[1], [0]]], np.uint8))[0, 0, 0] == 0


def test_psnr_formula():
    a = np.zeros((4, 4, 3), np.uint8)
    b = a.copy()
    assert V.psnr(a, b) == float("inf")
    b[0, 0, 0] = 255
    mse = 255.0 ** 2 / a.size
    assert abs(V.psnr(a, b) - 10 * np.log10(255 ** 2 / mse)) < 1e-12
    p, good = V.validate_frame(np.zeros((2, 2, 3), np.uint8), np.zeros((4, 4, 4), np.uint8))
    assert good and p == float("inf")


def test_bmp_round_trip_and_layout(tmp_path, native_lib):
    rng = np.random.default_rng(3)
    bgra = rng.integers(0, 256, (5, 7, 4), dtype=np.uint8)
    path = tmp_path / "f.bmp"
    N.write_bmp(path, bgra)
    data = path.read_bytes()
    pitch = (7 * 3 + 3) // 4 * 4
    assert data[:2] == b"BM" and len(data) == 54 + pitch * 5                     # bmp.cc:14-15
    assert int.from_bytes(data[0x1C:0x1E], "little") == 24
    rgb = V.read_bmp(path)
    assert np.array_equal(rgb, bgra[..., [2, 1, 0]])


def test_reference_golden_frame_readable():
    ref = np.load(os.path.join(GOLDEN, "frame_0000_ref.npz"))["rgb"]
    assert ref.shape == (360, 640, 3) and ref.dtype == np.uint8
    half = V.downscale_half(ref)
    assert half.shape == (180, 320, 3)
    # a rendered frame, not a blank: it spans a real tonal range
    assert ref.min() == 0 and ref.max() > 200 and ref.std() > 10
