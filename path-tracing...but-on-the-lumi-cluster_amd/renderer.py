"""GPU renderer: the MI355X replacement of the reference's baseline_render.

``GpuRenderer`` owns one ``ptg_context`` (one GPU).  The reference drives its
hot path as

    load_scene(); setup_animation_frame(s, f); baseline_render(s, image)
    (main.cc:67, :82, :88)

and the same flow here is

    scene = Scene(assets, cfg); scene.setup_frame(f)
    r = GpuRenderer(device); r.upload(scene); img = r.render(cfg)

Everything below the C ABI runs in HIP kernels; this class only moves
pointers.  Device outputs are torch tensors (torch is used for device memory,
streams and torch.distributed only).  There is no CPU fallback: without a
gfx950 device the constructor raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import native as N


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class GpuRenderer:
    def __init__(self, device: int = 0, stream=None):
        import torch  # noqa: F401  (device memory + streams)
        self._ctx = C.c_void_p()
        N.check(N.lib().ptg_context_create(device, C.byref(self._ctx)), "ptg_context_create")
        self.device = device
        self.scene_uploaded = False
        if stream is not None:
            self.set_stream(stream)

    # -- streams ---------------------------------------------------------
    def set_stream(self, stream):
        """Launch on a torch.cuda.Stream (or raw hipStream_t int)."""
        handle = getattr(stream, "cuda_stream", stream)
        N.check(N.lib().ptg_context_set_stream(self._ctx, C.c_void_p(handle)), "ptg_context_set_stream")

    def synchronize(self):
        N.check(N.lib().ptg_synchronize(self._ctx), "ptg_synchronize")

    # -- uploads ---------------------------------------------------------
    def upload(self, scene: N.Scene, include_static=None):
        """upload_scene (once) + upload_frame (every frame) from a host Scene."""
        if include_static is None:
            include_static = not self.scene_uploaded
        N.check(N.lib().ptg_upload_from_scene(self._ctx, scene.handle, 1 if include_static else 0),
                "ptg_upload_from_scene")
        self.scene_uploaded = True

    def upload_arrays(self, arrays: dict, include_static=True, include_frame=True):
        """Upload reference-layout numpy arrays (the keys of Scene.view()):
        ptg_upload_scene (include_static) and/or ptg_upload_frame (include_frame)."""
        L = N.lib()
        a = {k: (np.ascontiguousarray(v) if isinstance(v, np.ndarray) else v) for k, v in arrays.items()}
        sn = int(a["static_node_count"])
        if include_static:
            N.check(L.ptg_upload_scene(self._ctx, a["nodes"].ctypes.data, a["links"].ctypes.data, sn,
                                       a["indices"].ctypes.data, a["indices"].size, a["pos"].ctypes.data,
                                       a["normal"].ctypes.data, a["albedo"].ctypes.data, a["material"].ctypes.data,
                                       a["pos"].shape[0]), "ptg_upload_scene")
        if not include_frame:
            self.scene_uploaded = self.scene_uploaded or include_static
            return
        nodes = a["nodes"][sn:]
        links = a["links"][8 * sn:]
        N.check(L.ptg_upload_frame(self._ctx, a["subframes"].ctypes.data, a["subframes"].size,
                                   a["instances"].ctypes.data, a["instances"].size,
                                   np.ascontiguousarray(nodes).ctypes.data, np.ascontiguousarray(links).ctypes.data,
                                   sn, nodes.size), "ptg_upload_frame")
        self.scene_uploaded = True

    # -- rendering -------------------------------------------------------
    def render(self, cfg: N.RenderConfig, rect=None, samples=None, out_bgra=None, out_accum=None,
               want_accum=False):
        """baseline_render over `rect` = (x0, y0, w, h) (default: the whole
        image) and sample range `samples` = (begin, end) (default: all).
        Returns (bgra uint8 [h, w, 4], accum float32 [h, w, 4] or None) as
        torch tensors on this GPU.  Asynchronous on the context stream."""
        import torch
        x0, y0, w, h = rect if rect is not None else (0, 0, cfg.width, cfg.height)
        j0, j1 = samples if samples is not None else (0, cfg.samples_per_pixel)
        dev = torch.device("cuda", self.device)
        if out_bgra is None:
            out_bgra = torch.empty((h, w, 4), dtype=torch.uint8, device=dev)
        if out_accum is None and want_accum:
            out_accum = torch.empty((h, w, 4), dtype=torch.float32, device=dev)
        N.check(N.lib().ptg_render(self._ctx, C.byref(cfg), x0, y0, w, h, j0, j1, _ptr(out_accum), _ptr(out_bgra)),
                "ptg_render")
        return out_bgra, out_accum

    def render_tiles(self, cfg: N.RenderConfig, tile_w, tile_h, first, stride, count, out_bgra=None,
                     out_accum=None):
        """Render an interleaved tile set densely (multi-GPU sharding unit)."""
        import torch
        dev = torch.device("cuda", self.device)
        n = count * tile_w * tile_h
        if out_bgra is None:
            out_bgra = torch.empty((n, 4), dtype=torch.uint8, device=dev)
        N.check(N.lib().ptg_render_tiles(self._ctx, C.byref(cfg), tile_w, tile_h, first, stride, count,
                                         _ptr(out_accum), _ptr(out_bgra)), "ptg_render_tiles")
        return out_bgra, out_accum

    def scatter_tiles(self, cfg, tile_w, tile_h, first, stride, count, tiles_bgra, image_bgra):
        N.check(N.lib().ptg_scatter_tiles(self._ctx, C.byref(cfg), tile_w, tile_h, first, stride, count,
                                          _ptr(tiles_bgra), _ptr(image_bgra)), "ptg_scatter_tiles")

    # -- per-sample / per-ray entry points (parity) -------------------------
    def path_trace_samples(self, cfg, xy: np.ndarray, sample_index: np.ndarray) -> np.ndarray:
        xy = np.ascontiguousarray(xy, dtype=np.uint32).reshape(-1, 2)
        js = np.ascontiguousarray(sample_index, dtype=np.int32).reshape(-1)
        out = np.zeros((len(js), 4), np.float32)
        N.check(N.lib().ptg_path_trace_samples(self._ctx, C.byref(cfg), len(js), xy.ctypes.data, js.ctypes.data,
                                               out.ctypes.data), "ptg_path_trace_samples")
        return out

    def trace_rays(self, subframe: int, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros((len(rays), 8), np.uint32)
        N.check(N.lib().ptg_trace_rays(self._ctx, subframe, len(rays), rays.ctypes.data, hits.ctypes.data),
                "ptg_trace_rays")
        return hits

    def tonemap_device(self, colors, out_bgra):
        """tonemap_pixel over a device float32 [..., 4] tensor into a device
        uint8 [..., 4] tensor (ptg_tonemap_device; asynchronous)."""
        n = colors.numel() // 4
        assert out_bgra.numel() == 4 * n
        N.check(N.lib().ptg_tonemap_device(self._ctx, n, _ptr(colors), _ptr(out_bgra)), "ptg_tonemap_device")
        return out_bgra

    def tonemap(self, colors: np.ndarray) -> np.ndarray:
        c = np.zeros((colors.shape[0], 4), np.float32)
        c[:, :colors.shape[1]] = colors[:, :4] if colors.shape[1] >= 4 else colors
        c = np.ascontiguousarray(c)
        out = np.zeros((len(c), 4), np.uint8)
        N.check(N.lib().ptg_tonemap(self._ctx, len(c), c.ctypes.data, out.ctypes.data), "ptg_tonemap")
        return out

    def enable_timing(self, on=True):
        N.check(N.lib().ptg_timing_enable(self._ctx, 1 if on else 0), "ptg_timing_enable")

    def last_timing(self):
        """(summed path-kernel device ms, launch count) since timing was enabled or last read."""
        ms, n = C.c_double(), C.c_uint32()
        N.check(N.lib().ptg_last_timing(self._ctx, C.byref(ms), C.byref(n)), "ptg_last_timing")
        return ms.value, n.value

    KINDS = ("megakernel", "extend", "shadow", "shade", "camera", "accumulate", "sky", "classify")

    def kernel_times(self):
        """{kind: (device ms, launches)} summed over the launches recorded since
        timing was enabled or last read (waits for them; clears the record)."""
        ms = np.zeros(8, np.float64)
        n = np.zeros(8, np.uint32)
        N.check(N.lib().ptg_last_kernel_times(self._ctx, ms.ctypes.data, n.ctypes.data), "ptg_last_kernel_times")
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.KINDS)}

    def kernel_busy(self):
        """{kind: (busy ms, summed ms, launches)}: busy = the union of the
        recorded launches' device intervals (overlapping launches of one kind
        counted once); waits for them and clears the record."""
        busy = np.zeros(8, np.float64)
        ms = np.zeros(8, np.float64)
        n = np.zeros(8, np.uint32)
        N.check(N.lib().ptg_last_kernel_busy(self._ctx, busy.ctypes.data, ms.ctypes.data, n.ctypes.data),
                "ptg_last_kernel_busy")
        return {k: (float(busy[i]), float(ms[i]), int(n[i])) for i, k in enumerate(self.KINDS)}

    def kernel_counters(self):
        """{kind: counters[8]} of the last render call (counting enabled)."""
        out = np.zeros((6, 8), np.uint64)
        N.check(N.lib().ptg_last_kernel_counters(self._ctx, out.ctypes.data), "ptg_last_kernel_counters")
        return {k: out[i] for i, k in enumerate(self.KINDS[:6])}

    WALK_STATS = ("node_phases", "node_lanes", "leaf_phases", "leaf_lanes", "refills", "refill_lanes", "iterations",
                  "active_lanes")

    def walk_stats(self):
        """{"extend"|"shadow": {stat: count}} of the last counted render: the
        walks' phases that loaded records and the lanes they served
        (ptg_last_walk_stats)."""
        out = np.zeros((2, 8), np.uint64)
        N.check(N.lib().ptg_last_walk_stats(self._ctx, out.ctypes.data), "ptg_last_walk_stats")
        return {k: {s: int(out[i, j]) for j, s in enumerate(self.WALK_STATS)} for i, k in enumerate(("extend", "shadow"))}

    def set_hbm_share(self, percent):
        """Cap the wavefront path state at `percent` of HBM per chunk pipeline
        (default 35); identical bits at any share."""
        N.check(N.lib().ptg_set_hbm_share(self._ctx, int(percent)), "ptg_set_hbm_share")

    def set_chunk_paths(self, log2_paths):
        """At most 2^log2_paths live paths per sample chunk and pipeline
        (16-28, default 27); identical bits at any size."""
        N.check(N.lib().ptg_set_chunk_paths(self._ctx, int(log2_paths)), "ptg_set_chunk_paths")

    def set_pipeline(self, name):
        """'wavefront' (default) or 'megakernel' - bit-identical results."""
        N.check(N.lib().ptg_set_pipeline(self._ctx, {"wavefront": 0, "megakernel": 1}[name]), "ptg_set_pipeline")

    def redo_stats(self):
        """Counting renders: paths the certified shading passes handed to the
        exact (glibc-algorithm) pass - {"surface", "sky", "sites": {site: n}}
        (ptg_last_redo_stats)."""
        out = np.zeros(9, np.uint64)
        N.check(N.lib().ptg_last_redo_stats(self._ctx, out.ctypes.data), "ptg_last_redo_stats")
        names = ("acc_exp", "exp_times", "add_mul_pow", "div_mul_pow", "times_cos", "times_sin",
                 "times_one_minus_div_pow")
        return {"surface": int(out[0]), "sky": int(out[1]), "sites": {n: int(out[2 + k]) for k, n in enumerate(names)}}

    def selftest(self):
        """ptg_arith_selftest: mask of the failed arithmetic known-answer checks (0 = all
        passed) of the library's own build on this device against this host's libm."""
        m = N.lib().ptg_arith_selftest(self._ctx)
        if m < 0:
            N.check(m, "ptg_arith_selftest")
        return int(m)

    def set_concurrency(self, level):
        """0: one stream; 1: sky/shadow kernels on a second stream; 2 (default):
        also two sample chunks in flight.  Identical bits at every level."""
        N.check(N.lib().ptg_set_concurrency(self._ctx, int(level)), "ptg_set_concurrency")

    def enable_counters(self, on=True):
        N.check(N.lib().ptg_counters_enable(self._ctx, 1 if on else 0), "ptg_counters_enable")

    def counters(self):
        out = np.zeros(8, np.uint64)
        N.check(N.lib().ptg_last_counters(self._ctx, out.ctypes.data), "ptg_last_counters")
        return out

    def close(self):
        if self._ctx:
            N.lib().ptg_context_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
