"""Shared fixtures.  `-m gpu` tests need a gfx950 device; everything else runs on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import ptlumi_loader  # noqa: E402,F401  (registers the package as `ptlumi`)
import ptlumi  # noqa: E402
from ptlumi import native as N  # noqa: E402

ASSETS = os.path.join(ROOT, "assets")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def assets_dir():
    if not os.path.exists(os.path.join(ASSETS, "MANIFEST")):
        ptlumi.assets.prepare(ASSETS)
    return ASSETS


@pytest.fixture(scope="session")
def native_lib():
    return N.lib()


_scenes = {}


def scene_for(assets_dir, w, h, spp, bounces=4, frame=0):
    """Session-cached host scene (load_scene is ~2-3 s) set to `frame`."""
    key = (w, h, spp, bounces)
    if key not in _scenes:
        _scenes[key] = N.Scene(assets_dir, N.RenderConfig.make(w, h, spp, bounces))
    s = _scenes[key]
    if s.frame != frame:
        s.setup_frame(frame)
    return s


def arrays_copy(scene):
    v = scene.view()
    return {k: (np.array(x) if isinstance(x, np.ndarray) else x) for k, x in v.items()}


@pytest.fixture(scope="session")
def gpu():
    # a GPU test must never pass by skipping on a box without the device
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but torch.cuda.is_available() is False")
    from ptlumi.renderer import GpuRenderer
    r = GpuRenderer(0)
    yield r
    r.close()
