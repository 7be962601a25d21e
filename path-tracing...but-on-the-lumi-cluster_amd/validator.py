"""Frame validator: numpy restatement of the reference's validator.py.

The reference validates every frame against course reference PNGs with
scikit-image (validator.py:27-70), which is not available here.  Its
arithmetic is reproduced exactly:
  1. own = our frame, [H, W, 3] uint8 (validator.py:41);
  2. ``downscale_local_mean(own, (2, 2, 1))`` = float64 mean of 2x2 blocks
     (validator.py:43; the image sides are even for every config);
  3. ``.astype(np.uint8)`` = truncation (validator.py:44);
  4. ``peak_signal_noise_ratio(ref, own)`` with data range 255 for uint8:
     10 log10(255^2 / mean((ref - own)^2)) in float64 (validator.py:45);
  5. GOOD iff PSNR >= 32 (validator.py:11, :50-54).
The reference frames are produced by the reference renderer itself (built
from its sources by the oracle recipe) and downscaled the same way.
"""
from __future__ import annotations

import numpy as np

ACCEPT_MIN_PSNR = 32.0
RESIZE_FACTOR = 2


def downscale_half(img: np.ndarray) -> np.ndarray:
    """downscale_local_mean(img, (2, 2, 1)).astype(uint8) for even sides."""
    img = np.asarray(img, dtype=np.float64)
    h, w = img.shape[:2]
    if h % 2 or w % 2:
        # skimage pads with zeros (cval=0) up to a multiple of the factor
        ph, pw = (-h) % 2, (-w) % 2
        img = np.pad(img, ((0, ph), (0, pw), (0, 0)))
        h, w = img.shape[:2]
    m = img.reshape(h // 2, 2, w // 2, 2, -1).mean(axis=(1, 3))
    return m.astype(np.uint8)


def psnr(ref: np.ndarray, own: np.ndarray) -> float:
    ref = np.asarray(ref, dtype=np.float64)
    own = np.asarray(own, dtype=np.float64)
    mse = np.mean((ref - own) ** 2)
    if mse == 0:
        return float("inf")
    return float(10.0 * np.log10(255.0 ** 2 / mse))


def bgra_to_rgb(bgra: np.ndarray) -> np.ndarray:
    """Our renderer's [H, W, 4] BGRA -> [H, W, 3] RGB (what imread of the BMP gives)."""
    return np.ascontiguousarray(bgra[..., [2, 1, 0]])


def validate_frame(ref_rgb_half: np.ndarray, own_bgra_full: np.ndarray):
    """Returns (psnr, good) for one frame, as validator.py reports it."""
    own = downscale_half(bgra_to_rgb(own_bgra_full))
    p = psnr(ref_rgb_half, own)
    return p, p >= ACCEPT_MIN_PSNR


def read_bmp(path) -> np.ndarray:
    """Read a 24-bit bottom-up BMP as written by write_bmp (bmp.cc) -> [H, W, 3] RGB."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:2] != b"BM":
        raise ValueError("not a BMP: %s" % path)
    off = int.from_bytes(data[10:14], "little")
    w = int.from_bytes(data[18:22], "little")
    h = int.from_bytes(data[22:26], "little")
    bpp = int.from_bytes(data[28:30], "little")
    if bpp != 24:
        raise ValueError("only 24-bit BMPs are supported")
    pitch = (w * 3 + 3) // 4 * 4
    rows = np.frombuffer(data, dtype=np.uint8, count=pitch * h, offset=off).reshape(h, pitch)[:, :w * 3]
    bgr = rows.reshape(h, w, 3)[::-1]
    return np.ascontiguousarray(bgr[..., ::-1])
