"""In-tree build of libptg.so (gfx950) and of the test oracle.

``build()`` is what ``__graft_entry__.build()`` runs: it compiles the HIP
kernels for gfx950 and the host C++ (make -C csrc), prepares the scene assets
and, for the tests only, builds the oracle (oracle/Makefile) - and, when the
reference tree is present (this container, not the GPU box), the reference
renderer from its sources as the oracle's checker - and the user-kernel test
library built against include/ptg_device.h.  Built files stay in the
tree (git-ignored) so they travel to the GPU box with the snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
ORACLE = os.path.join(ROOT, "oracle")
REFERENCE = "/root/reference"

# Reference builds the tests and the bench use: (mode, W, H, SPP, BOUNCES)
REF_CONFIGS = [
    ("strict", 640, 360, 32, 4),     # parity goldens (scene arrays, rays, samples)
    ("strict", 160, 90, 32, 4),      # small whole-frame golden
    ("strict", 1280, 720, 256, 4),   # bench workload: per-sample spot checks
    ("v3", 1280, 720, 16, 4),        # CPU baseline (reference flags, portable -march)
    ("v3", 640, 360, 32, 4),         # CPU baseline configs[0] (one core); strict-vs-shipped statistics
]
# reference host code + ptg_render in place of baseline_render (oracle/dropin_main.cc),
# and + ptg_render_gather over an RCCL communicator (oracle/dropin_rccl.cc)
DROPIN_CONFIGS = [("strict", 160, 90, 32, 4)]


def _run(cmd, cwd, verbose):
    if verbose:
        print("+", " ".join(cmd), "(in %s)" % cwd, flush=True)
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("command failed: %s" % " ".join(cmd))
    return r.stdout


def build_native(verbose=False, jobs=8):
    _run(["make", "-j%d" % jobs, "all", "certfail"], os.path.join(PKG, "csrc"), verbose)
    return os.path.join(PKG, "_build", "libptg.so")


def build_oracle(verbose=False, jobs=8, with_reference=None):
    _run(["make", "oracle"], ORACLE, verbose)
    if with_reference is None:
        with_reference = os.path.isdir(REFERENCE)
    if with_reference:
        for mode, w, h, spp, b in REF_CONFIGS:
            _run(["make", "-j%d" % jobs, "ref", "REF_MODE=%s" % mode, "REF_W=%d" % w, "REF_H=%d" % h,
                  "REF_SPP=%d" % spp, "REF_BOUNCES=%d" % b], ORACLE, verbose)
        for mode, w, h, spp, b in DROPIN_CONFIGS:   # needs libptg.so: build_native first
            _run(["make", "-j%d" % jobs, "dropin", "dropin_rccl", "REF_MODE=%s" % mode, "REF_W=%d" % w,
                  "REF_H=%d" % h, "REF_SPP=%d" % spp, "REF_BOUNCES=%d" % b], ORACLE, verbose)


def build_test_kernels(verbose=False):
    """The user-kernel library of tests/test_gpu_device_dropin.py: a HIP kernel
    built against include/ptg_device.h alone (test infrastructure)."""
    _run(["make"], os.path.join(ROOT, "tests", "device_dropin"), verbose)


def build_tools(verbose=False):
    """tools/_bin/walk_sim: the CPU model of the block walk over the upload's own
    packing (tests/test_block_bvh.py)."""
    _run(["make", "walk_sim"], os.path.join(ROOT, "tools"), verbose)


def prepare_assets():
    from . import assets
    return assets.prepare(assets.default_dir(ROOT))


def build(verbose=False):
    prepare_assets()
    build_native(verbose)
    build_test_kernels(verbose)
    build_tools(verbose)
    build_oracle(verbose)
