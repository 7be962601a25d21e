"""The oracle (oracle/pt_oracle.c) vs the reference's own outputs.

Every fixture in tests/golden/ was produced by the reference renderer
compiled from its sources (strict IEEE build, tests/golden/make_golden.py).
The oracle must reproduce them bit for bit: this pins the oracle, which then
serves as the checker of the GPU kernels (tests/test_gpu_*.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, arrays_copy, scene_for

import oracle as O


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_pcg4d_known_answers():
    g = load("pcg4d.npz")
    a, u = O.pcg(g["seeds"])
    assert np.array_equal(a, g["pcg"])
    assert np.array_equal(bits(u), g["uniform_bits"])


def test_pcg4d_numpy_restatement():
    """A third, vectorised statement of math.hh:466-473 agrees too."""
    g = load("pcg4d.npz")
    s = g["seeds"].astype(np.uint64)
    M = np.uint64(0xFFFFFFFF)
    x, y, z, w = [(s[:, i] * 1664525 + 1013904223) & M for i in range(4)]
    x, y, z, w = (x + y * w) & M, (y + z * x) & M, (z + x * y) & M, (w + y * z) & M
    x, y, z, w = x ^ (x >> 16), y ^ (y >> 16), z ^ (z >> 16), w ^ (w >> 16)
    x, y, z, w = (x + y * w) & M, (y + z * x) & M, (z + x * y) & M, (w + y * z) & M
    assert np.array_equal(np.stack([x, y, z, w], 1).astype(np.uint32), g["pcg"])


def test_tonemap_known_answers():
    g = load("tonemap.npz")
    assert np.array_equal(O.tonemap(g["colors"]), g["bgra"])


def test_ray_queries_match_reference(assets_dir):
    g = load("rays_f450.npz")
    s = scene_for(assets_dir, 640, 360, 32, frame=int(g["frame"]))
    got = O.Oracle(s.view(), s.cfg).trace_rays(int(g["subframe"]), g["rays"])
    assert np.array_equal(got, g["hits"])
    hit = g["hits"][:, 3].view(np.float32) > 0
    assert 0.1 < hit.mean() < 0.99 and g["hits"][:, 7].any()   # the fixture exercises hits, misses, shadows


@pytest.mark.parametrize("frame", [0, 450, 1750])
def test_samples_match_reference(assets_dir, frame):
    g = load("samples_f%04d.npz" % frame)
    s = scene_for(assets_dir, 640, 360, 32, frame=frame)
    orc = O.Oracle(s.view(), s.cfg)
    x0, y0, w, h, j1 = int(g["x0"]), int(g["y0"]), int(g["w"]), int(g["h"]), int(g["j1"])
    xy = np.array([[x0 + i % w, y0 + i // w] for i in range(w * h)], np.uint32).repeat(j1, 0)
    js = np.tile(np.arange(j1, dtype=np.int32), w * h)
    got = orc.samples(xy, js)[:, :3].reshape(h, w, j1, 3)
    assert np.array_equal(bits(got), bits(g["radiance"]))
    assert (g["radiance"] > 0).any()


def test_whole_frame_matches_reference(assets_dir):
    g = load("frame_160x90.npz")
    s = scene_for(assets_dir, 160, 90, 32, frame=0)
    acc, bgra = O.Oracle(arrays_copy(s), s.cfg).render_rect(0, 0, 160, 90)
    assert np.array_equal(bits(acc[..., :3]), bits(g["radiance"]))
    assert np.array_equal(bgra, g["bgra"])
