#!/usr/bin/env python3
"""Diagnostics: ptg_trace_rays on the golden rays of frame 450 vs the golden
hits (tests/golden/rays_f450.npz); prints the rays whose records differ."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa
import conftest
from conftest import scene_for, arrays_copy
from ptlumi.renderer import GpuRenderer
g = np.load(os.path.join(ROOT, "tests", "golden", "rays_f450.npz"))
s = scene_for(conftest.ASSETS, 640, 360, 32, frame=int(g["frame"]))
r = GpuRenderer(0)
r.upload_arrays(arrays_copy(s))
hits = r.trace_rays(int(g["subframe"]), g["rays"])
want = g["hits"]
bad = np.nonzero((hits != want).any(1))[0]
print("lib", os.environ.get("PTG_LIB", "default"), "rays differing:", len(bad), "of", len(want))
for i in bad[:12]:
    print(i, "got", hits[i].tolist(), "want", want[i].tolist())
