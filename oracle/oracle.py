"""Python access to the test oracle (TEST INFRASTRUCTURE ONLY).

* ``Oracle``      - ctypes binding of liboracle.so (pt_oracle.c, the strict
                    CPU restatement of the reference hot path).
* ``Reference``   - runs the reference renderer built from its own sources
                    (oracle/_ref/<mode>_<W>x<H>_s<SPP>_b<B>/ref_pt) through the
                    harness commands of ref_harness.cc.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
this module; the product never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

ARRAY_KEYS = ["subframes", "instances", "nodes", "links", "indices", "pos", "normal", "albedo", "material"]


class _Scene(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ARRAY_KEYS]


class _Config(C.Structure):
    _fields_ = [(k, C.c_uint32) for k in ["width", "height", "samples_per_pixel", "max_bounces", "student_id",
                                         "samples_per_motion_blur_step"]]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise OSError("oracle not built: %s (run make -C oracle oracle)" % LIB)
        L = C.CDLL(LIB)
        P, U32, I32 = C.c_void_p, C.c_uint32, C.c_int32
        L.orc_path_trace_pixel.argtypes = [P, P, U32, U32, I32, P, P]
        L.orc_tonemap_pixel.argtypes = [P, P]
        L.orc_pcg4d.argtypes = [P]
        L.orc_uniform4.argtypes = [P, P]
        L.orc_trace_ray.argtypes = [P, U32, P, P]
        L.orc_render_rect.argtypes = [P, P, U32, U32, U32, U32, U32, U32, P, P, P]
        for f in (L.orc_path_trace_pixel, L.orc_tonemap_pixel, L.orc_pcg4d, L.orc_uniform4, L.orc_trace_ray,
                  L.orc_render_rect):
            f.restype = None
        _lib = L
    return _lib


class Oracle:
    """The CPU restatement bound to one frame's arrays (numpy, reference layout)."""

    def __init__(self, arrays: dict, cfg):
        self._keep = {k: np.ascontiguousarray(arrays[k]) for k in ARRAY_KEYS}
        self._scene = _Scene(*[self._keep[k].ctypes.data for k in ARRAY_KEYS])
        c = cfg if isinstance(cfg, dict) else {k: getattr(cfg, k) for k, _ in _Config._fields_}
        self._cfg = _Config(*[int(c[k]) for k, _ in _Config._fields_])
        self.cfg = c

    def sample(self, x, y, j, counters=None):
        out = np.zeros(4, np.float32)
        lib().orc_path_trace_pixel(C.byref(self._scene), C.byref(self._cfg), x, y, j, out.ctypes.data,
                                   counters.ctypes.data if counters is not None else None)
        return out

    def samples(self, xy: np.ndarray, js: np.ndarray, counters=None) -> np.ndarray:
        xy = np.asarray(xy, dtype=np.uint32).reshape(-1, 2)
        js = np.asarray(js, dtype=np.int32).reshape(-1)
        out = np.zeros((len(js), 4), np.float32)
        L = lib()
        cp = counters.ctypes.data if counters is not None else None
        for i in range(len(js)):
            L.orc_path_trace_pixel(C.byref(self._scene), C.byref(self._cfg), int(xy[i, 0]), int(xy[i, 1]),
                                   int(js[i]), out[i].ctypes.data, cp)
        return out

    def render_rect(self, x0, y0, w, h, j0=0, j1=None, threads=None, counters=None):
        """baseline_render over a rectangle; rows split over threads (ctypes releases the GIL)."""
        j1 = self.cfg["samples_per_pixel"] if j1 is None else j1
        accum = np.zeros((h, w, 4), np.float32)
        bgra = np.zeros((h, w, 4), np.uint8)
        threads = threads or min(os.cpu_count() or 1, 16)
        per_thread = [np.zeros(8, np.uint64) for _ in range(threads)]

        def rows(t):
            for r in range(t, h, threads):
                lib().orc_render_rect(C.byref(self._scene), C.byref(self._cfg), x0, y0 + r, w, 1, j0, j1,
                                      accum[r].ctypes.data, bgra[r].ctypes.data, per_thread[t].ctypes.data)

        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(rows, range(threads)))
        if counters is not None:
            counters += sum(per_thread)
        return accum, bgra

    def trace_rays(self, subframe, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        out = np.zeros((len(rays), 8), np.uint32)
        L = lib()
        for i in range(len(rays)):
            L.orc_trace_ray(C.byref(self._scene), subframe, rays[i].ctypes.data, out[i].ctypes.data)
        return out


def tonemap(colors: np.ndarray) -> np.ndarray:
    colors = np.ascontiguousarray(colors, dtype=np.float32).reshape(-1, colors.shape[-1])
    out = np.zeros((len(colors), 4), np.uint8)
    L = lib()
    for i in range(len(colors)):
        c = np.ascontiguousarray(colors[i, :3])
        L.orc_tonemap_pixel(c.ctypes.data, out[i].ctypes.data)
    return out


def pcg(seeds: np.ndarray):
    """-> (pcg4d(seed), generate_uniform_random4 on the advanced seed) per row."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32).reshape(-1, 4)
    a = np.zeros_like(seeds)
    u = np.zeros((len(seeds), 4), np.float32)
    L = lib()
    for i in range(len(seeds)):
        s = seeds[i].copy()
        L.orc_pcg4d(s.ctypes.data)
        a[i] = s
        L.orc_uniform4(s.ctypes.data, u[i].ctypes.data)
    return a, u


class Reference:
    """The reference renderer built from /root/reference sources (oracle/Makefile)."""

    def __init__(self, mode="strict", w=640, h=360, spp=32, bounces=4):
        self.mode, self.w, self.h, self.spp, self.bounces = mode, w, h, spp, bounces
        self.exe = os.path.join(HERE, "_ref", "%s_%dx%d_s%d_b%d" % (mode, w, h, spp, bounces), "ref_pt")

    def available(self):
        return os.path.exists(self.exe)

    def run(self, assets, *args, env=None, timeout=3600, cpus=None):
        """Run the harness; `cpus` pins it to those host CPUs (taskset)."""
        if not self.available():
            raise FileNotFoundError(self.exe)
        e = dict(os.environ)
        if env:
            e.update(env)
        pin = ["taskset", "-c", ",".join(str(c) for c in cpus)] if cpus else []
        r = subprocess.run(pin + [self.exe, assets] + [str(a) for a in args], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True, env=e, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError("ref_pt %s failed (%d): %s" % (args, r.returncode, r.stderr[-2000:]))
        return r.stdout

    def samples(self, assets, frame, x0, y0, w, h, j0, j1, timeout=3600):
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "s.f32")
            self.run(assets, "samples", frame, x0, y0, w, h, j0, j1, p, timeout=timeout)
            return np.fromfile(p, np.float32).reshape(h, w, j1 - j0, 4)

    def render(self, assets, frame, timeout=3600):
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "r")
            self.run(assets, "render", frame, p, timeout=timeout)
            acc = np.fromfile(p + ".f32", np.float32).reshape(self.h, self.w, 4)
            bgra = np.fromfile(p + ".bgra", np.uint8).reshape(self.h, self.w, 4)
            return acc, bgra

    def rays(self, assets, frame, subframe, rays):
        with tempfile.TemporaryDirectory() as d:
            i, o = os.path.join(d, "in.f32"), os.path.join(d, "out.u32")
            np.ascontiguousarray(rays, dtype=np.float32).tofile(i)
            self.run(assets, "rays", frame, subframe, i, o)
            return np.fromfile(o, np.uint32).reshape(-1, 8)

    def dump(self, assets, frame, outdir):
        self.run(assets, "dump", frame, outdir)

    def baseline(self, assets, frame, threads=None, timeout=3600, cpus=None, bind=None):
        """Times the reference's own baseline_render (main.cc:12) on this host.
        threads -> OMP_NUM_THREADS; cpus -> taskset pinning; bind -> OMP_PROC_BIND
        (with OMP_PLACES=cores)."""
        import json
        with tempfile.TemporaryDirectory() as d:
            env = {"OMP_NUM_THREADS": str(threads)} if threads else {}
            if bind:
                env.update(OMP_PROC_BIND=bind, OMP_PLACES="cores")
            out = self.run(assets, "baseline", frame, os.path.join(d, "img.bgra"), env=env or None, timeout=timeout,
                           cpus=cpus)
            return json.loads(out.strip().splitlines()[-1])
