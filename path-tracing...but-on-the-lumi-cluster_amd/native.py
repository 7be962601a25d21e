"""ctypes binding of the C ABI in include/ptg.h (libptg.so).

This is the Python host mirror of the reference's interfaces: the scene
functions of scene.hh (load_scene / setup_animation_frame /
get_animation_frame_count), write_bmp (bmp.hh) and the GPU replacement of
baseline_render / path_trace_pixel / tonemap_pixel.  numpy views expose the
reference-layout arrays without copies.

The library is built in-tree (``csrc/Makefile``, driven by
``__graft_entry__.build()``); importing this module never falls back to
anything else - a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PTG_LIB") or os.path.join(HERE, "_build", "libptg.so")

PTG_OK = 0


class RenderConfig(C.Structure):
    """ptg_render_config: the reference's config.hh macros as runtime values."""
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("samples_per_pixel", C.c_uint32),
                ("max_bounces", C.c_uint32), ("student_id", C.c_uint32),
                ("samples_per_motion_blur_step", C.c_uint32)]

    @classmethod
    def make(cls, width=640, height=360, spp=256, bounces=4, student_id=152121358, blur_step=8):
        return cls(width, height, spp, bounces, student_id, blur_step)

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SceneView(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("node_count", C.c_size_t), ("links", C.c_void_p),
                ("static_node_count", C.c_size_t), ("indices", C.c_void_p), ("index_count", C.c_size_t),
                ("pos", C.c_void_p), ("normal", C.c_void_p), ("albedo", C.c_void_p), ("material", C.c_void_p),
                ("vertex_count", C.c_size_t), ("instances", C.c_void_p), ("instance_count", C.c_size_t),
                ("static_instance_count", C.c_size_t), ("subframes", C.c_void_p), ("subframe_count", C.c_size_t)]


class Mesh(C.Structure):
    _fields_ = [("vertex_count", C.c_uint32), ("triangle_count", C.c_uint32), ("index_offset", C.c_uint32),
                ("base_vertex_offset", C.c_uint32)]


class Bvh(C.Structure):
    _fields_ = [("node_count", C.c_uint32), ("node_offset", C.c_uint32)]


# numpy dtypes with the reference byte layout (padding made explicit)
NODE_DTYPE = np.dtype([("min", "<f4", 3), ("max", "<f4", 3)])                      # bvh.hh:45-49, 24 B
LINK_DTYPE = np.dtype([("accept", "<u4"), ("cancel", "<u4")])                       # bvh.hh:57-67
INSTANCE_DTYPE = np.dtype([("blas", "<u4", 2), ("mesh", "<u4", 4), ("_pad", "<u4", 2),
                           ("transform", "<f4", (4, 4)), ("inv_transform", "<f4", (4, 4))])   # 160 B
CAMERA_DTYPE = np.dtype([("orientation", "<f4", (3, 4)), ("position", "<f4", 4), ("aspect_ratio", "<f4"),
                         ("inv_focal_length", "<f4"), ("focal_distance", "<f4"), ("aperture_angle", "<f4"),
                         ("aperture_polygon", "<i4"), ("aperture_radius", "<f4"), ("_pad", "<u4", 2)])  # 96 B
LIGHT_DTYPE = np.dtype([("direction", "<f4", 4), ("color", "<f4", 4), ("cos_solid_angle", "<f4"),
                        ("_pad", "<u4", 3)])                                          # 48 B
SUBFRAME_DTYPE = np.dtype([("tlas", "<u4", 2), ("_pad", "<u4", 2), ("cam", CAMERA_DTYPE), ("light", LIGHT_DTYPE)])
assert NODE_DTYPE.itemsize == 24 and INSTANCE_DTYPE.itemsize == 160
assert CAMERA_DTYPE.itemsize == 96 and LIGHT_DTYPE.itemsize == 48 and SUBFRAME_DTYPE.itemsize == 160

_lib = None


def lib():
    """Load libptg.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError("libptg.so not built at %s - run __graft_entry__.build()" % LIB_PATH)
    # One HIP runtime per process: PyTorch bundles its own libamdhip64.so.7 and
    # loads it under a different DT_NEEDED name, so a libptg loaded first would
    # bring in ROCm's copy beside it, and whichever runtime opens the GPU
    # second finds no device (hipErrorNoDevice; tools/probe_libs.py).  With
    # torch imported first, libptg's libamdhip64.so.7 resolves to torch's.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P, U32, SZ, I = C.c_void_p, C.c_uint32, C.c_size_t, C.c_int
    sig = {
        "ptg_abi_version": (I, []),
        "ptg_arith_selftest": (I, [P]),
        "ptg_last_error": (C.c_char_p, []),
        "ptg_set_host_threads": (I, [I]),
        "ptg_render_config_default": (None, [P]),
        "ptg_scene_load": (I, [C.c_char_p, P, C.POINTER(P)]),
        "ptg_scene_setup_frame": (I, [P, U32]),
        "ptg_scene_view_get": (I, [P, P]),
        "ptg_scene_frame_count": (U32, [P]),
        "ptg_scene_mesh": (I, [P, C.c_char_p, P, P]),
        "ptg_scene_destroy": (None, [P]),
        "ptg_write_bmp": (I, [C.c_char_p, U32, U32, U32, U32, P]),
        "ptg_context_create": (I, [I, C.POINTER(P)]),
        "ptg_context_destroy": (None, [P]),
        "ptg_context_set_stream": (I, [P, P]),
        "ptg_context_get_stream": (I, [P, C.POINTER(P)]),
        "ptg_context_device": (I, [P, C.POINTER(I)]),
        "ptg_upload_scene": (I, [P, P, P, SZ, P, SZ, P, P, P, P, SZ]),
        "ptg_upload_frame": (I, [P, P, SZ, P, SZ, P, P, SZ, SZ]),
        "ptg_upload_from_scene": (I, [P, P, I]),
        "ptg_render": (I, [P, P, U32, U32, U32, U32, U32, U32, P, P]),
        "ptg_render_tiles": (I, [P, P, U32, U32, U32, U32, U32, P, P]),
        "ptg_scatter_tiles": (I, [P, P, U32, U32, U32, U32, U32, P, P]),
        "ptg_path_trace_samples": (I, [P, P, SZ, P, P, P]),
        "ptg_tonemap": (I, [P, SZ, P, P]),
        "ptg_tonemap_device": (I, [P, SZ, P, P]),
        "ptg_trace_rays": (I, [P, U32, SZ, P, P]),
        "ptg_counters_enable": (I, [P, I]),
        "ptg_last_counters": (I, [P, P]),
        "ptg_timing_enable": (I, [P, I]),
        "ptg_last_timing": (I, [P, C.POINTER(C.c_double), C.POINTER(U32)]),
        "ptg_last_kernel_times": (I, [P, P, P]),
        "ptg_last_kernel_busy": (I, [P, P, P, P]),
        "ptg_last_kernel_counters": (I, [P, P]),
        "ptg_last_walk_stats": (I, [P, P]),
        "ptg_last_redo_stats": (I, [P, P]),
        "ptg_set_hbm_share": (I, [P, I]),
        "ptg_set_chunk_paths": (I, [P, I]),
        "ptg_set_pipeline": (I, [P, I]),
        "ptg_set_concurrency": (I, [P, I]),
        "ptg_synchronize": (I, [P]),
        "ptg_device_alloc": (I, [P, SZ, C.POINTER(P)]),
        "ptg_device_free": (I, [P, P]),
        "ptg_memcpy_d2h": (I, [P, P, P, SZ]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):
            raise OSError("%s does not export %s" % (LIB_PATH, name))
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


EXPORTED_SYMBOLS = None  # filled lazily by exported_symbols()


def exported_symbols():
    """Names of the functions the C ABI declares (parsed from include/ptg.h)."""
    import re
    hdr = os.path.join(os.path.dirname(HERE), "include", "ptg.h")
    with open(hdr) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(ptg_[a-z0-9_]+)\s*\(", text)))


class PtgError(RuntimeError):
    pass


def check(code, what=""):
    if code != PTG_OK:
        msg = lib().ptg_last_error()
        raise PtgError("%s failed (%d): %s" % (what, code, msg.decode() if msg else ""))


def _arr(ptr, dtype, count):
    if count == 0:
        return np.zeros(0, dtype=dtype)
    buf = (C.c_char * (np.dtype(dtype).itemsize * count)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=count)


class Scene:
    """Host scene: load_scene() + setup_animation_frame() (scene.cc:135, :271)."""

    def __init__(self, assets_dir, cfg: RenderConfig):
        self.cfg = cfg
        self._h = C.c_void_p()
        check(lib().ptg_scene_load(assets_dir.encode(), C.byref(cfg), C.byref(self._h)), "ptg_scene_load")
        self.frame = None

    def setup_frame(self, frame_index: int):
        check(lib().ptg_scene_setup_frame(self._h, frame_index), "ptg_scene_setup_frame")
        self.frame = frame_index

    def frame_count(self) -> int:
        return lib().ptg_scene_frame_count(self._h)

    def mesh(self, name):
        m, b = Mesh(), Bvh()
        check(lib().ptg_scene_mesh(self._h, name.encode(), C.byref(m), C.byref(b)), "ptg_scene_mesh")
        return m, b

    def view(self):
        """Zero-copy numpy views of the reference-layout arrays (valid until
        the next setup_frame)."""
        v = SceneView()
        check(lib().ptg_scene_view_get(self._h, C.byref(v)), "ptg_scene_view_get")
        return {
            "nodes": _arr(v.nodes, NODE_DTYPE, v.node_count),
            "links": _arr(v.links, LINK_DTYPE, 8 * v.node_count),
            "static_node_count": v.static_node_count,
            "indices": _arr(v.indices, np.uint32, v.index_count),
            "pos": _arr(v.pos, np.float32, 4 * v.vertex_count).reshape(-1, 4),
            "normal": _arr(v.normal, np.float32, 4 * v.vertex_count).reshape(-1, 4),
            "albedo": _arr(v.albedo, np.float32, 4 * v.vertex_count).reshape(-1, 4),
            "material": _arr(v.material, np.float32, 4 * v.vertex_count).reshape(-1, 4),
            "instances": _arr(v.instances, INSTANCE_DTYPE, v.instance_count),
            "static_instance_count": v.static_instance_count,
            "subframes": _arr(v.subframes, SUBFRAME_DTYPE, v.subframe_count),
        }

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().ptg_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_bmp(path, bgra: np.ndarray):
    """write_bmp (bmp.cc:7) of an [H][W][4] uint8 BGRA image."""
    bgra = np.ascontiguousarray(bgra, dtype=np.uint8)
    h, w = bgra.shape[:2]
    check(lib().ptg_write_bmp(str(path).encode(), w, h, 4, w * 4, bgra.ctypes.data), "ptg_write_bmp")
