"""MI355X-native path tracer (gfx950) - drop-in for the per-pixel hot path of
Kalache-abdesattar/Path-Tracing...but-on-the-LUMI-cluster.

Registered as ``ptlumi`` by ``ptlumi_loader`` (the directory name is not a
Python identifier).  Layout:

  csrc/            HIP kernels (csrc/pt_kernels.hip, csrc/device/) and the
                   host C++ scene restatement (csrc/host/) -> _build/libptg.so
  native.py        ctypes binding of include/ptg.h
  renderer.py      GpuRenderer: upload + render through the C ABI
  distributed.py   one process per GPU: tile / frame sharding, RCCL gather
  validator.py     validator.py-equivalent PSNR check (numpy)
  assets.py        scene asset preparation (reference OBJs + substitutes)
  build.py         in-tree build of libptg.so for gfx950
"""
from . import assets, native, validator  # noqa: F401
from .native import RenderConfig, Scene, write_bmp  # noqa: F401

__all__ = ["assets", "native", "validator", "RenderConfig", "Scene", "write_bmp", "GpuRenderer"]


def __getattr__(name):
    if name == "GpuRenderer":
        from .renderer import GpuRenderer
        return GpuRenderer
    raise AttributeError(name)
