"""The C-ABI library (include/ptg.h): loads, exports every declared entry
point, fails loudly and with the documented codes.  No GPU compute here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT, N

HEADER = os.path.join(ROOT, "include", "ptg.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ptg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(native_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], stdout=subprocess.PIPE, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, "declared in ptg.h but not exported: %s" % missing
    assert len(declared_functions()) >= 30


def test_binding_covers_every_declared_symbol(native_lib):
    for f in declared_functions():
        assert getattr(native_lib, f).argtypes is not None or f in ("ptg_abi_version",), f


def test_abi_version(native_lib):
    assert native_lib.ptg_abi_version() == 1


def test_default_config_is_the_reference_testing_preset(native_lib):
    cfg = N.RenderConfig()
    native_lib.ptg_render_config_default(C.byref(cfg))
    # config.hh:5 (STUDENT_ID), :14-18 (TESTING preset), :29 (motion-blur step)
    assert cfg.as_dict() == {"width": 640, "height": 360, "samples_per_pixel": 256, "max_bounces": 4,
                             "student_id": 152121358, "samples_per_motion_blur_step": 8}


def test_scene_load_errors_are_codes_not_exits(native_lib, tmp_path):
    h = C.c_void_p()
    cfg = N.RenderConfig.make()
    assert native_lib.ptg_scene_load(None, C.byref(cfg), C.byref(h)) == -1          # PTG_E_INVALID
    rc = native_lib.ptg_scene_load(str(tmp_path).encode(), C.byref(cfg), C.byref(h))
    assert rc == -2                                                                 # PTG_E_IO
    assert b"Unable to open" in native_lib.ptg_last_error()
    bad = N.RenderConfig.make(0, 360)
    assert native_lib.ptg_scene_load(str(tmp_path).encode(), C.byref(bad), C.byref(h)) == -1


def test_gpu_entry_points_reject_null_context(native_lib):
    cfg = N.RenderConfig.make()
    assert native_lib.ptg_render(None, C.byref(cfg), 0, 0, 1, 1, 0, 1, None, None) == -1
    assert native_lib.ptg_upload_frame(None, None, 0, None, 0, None, None, 0, 0) == -1
    assert native_lib.ptg_synchronize(None) == -1


def test_context_create_without_gpu_fails_loudly(native_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    rc = native_lib.ptg_context_create(0, C.byref(h))
    assert rc in (-5, -4)          # PTG_E_NODEVICE (or PTG_E_HIP from the runtime)
    assert native_lib.ptg_last_error()


def test_write_bmp_error(native_lib, tmp_path):
    import numpy as np
    img = np.zeros((2, 2, 4), np.uint8)
    assert native_lib.ptg_write_bmp(str(tmp_path / "no" / "x.bmp").encode(), 2, 2, 4, 8, img.ctypes.data) == -2


RCCL_HEADER = os.path.join(ROOT, "include", "ptg_rccl.h")
RCCL_LIB = os.path.join(os.path.dirname(N.LIB_PATH), "libptg_rccl.so")


def test_rccl_library_exports_its_header_and_keeps_rccl_out_of_libptg(native_lib):
    """include/ptg_rccl.h's entry points live in libptg_rccl.so, which links
    librccl; libptg.so itself never needs an RCCL (torch loads its own)."""
    text = re.sub(r"/\*.*?\*/", "", open(RCCL_HEADER).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(ptg_[a-z0-9_]+)\s*\(", text)))
    assert declared == ["ptg_rccl_comm_destroy", "ptg_rccl_comm_init_env", "ptg_rccl_last_error", "ptg_render_gather"]
    out = subprocess.run(["nm", "-D", "--defined-only", RCCL_LIB], stdout=subprocess.PIPE, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    assert not [f for f in declared if f not in exported]
    needed = subprocess.run(["readelf", "-d", N.LIB_PATH], stdout=subprocess.PIPE, text=True, check=True).stdout
    assert "rccl" not in needed
    needed = subprocess.run(["readelf", "-d", RCCL_LIB], stdout=subprocess.PIPE, text=True, check=True).stdout
    assert "librccl" in needed and "libptg.so" in needed


def test_rccl_entry_points_reject_bad_arguments():
    lib = C.CDLL(RCCL_LIB)
    lib.ptg_rccl_last_error.restype = C.c_char_p
    cfg = N.RenderConfig.make()
    assert lib.ptg_render_gather(None, C.byref(cfg), 32, 16, None, None) == -1
    assert b"null argument" in lib.ptg_rccl_last_error()
    assert lib.ptg_rccl_comm_init_env(None, None, None, None, 1) == -1
    assert lib.ptg_rccl_comm_destroy(None) == -1
