#!/usr/bin/env python3
"""Diagnostics: does the device drop-in test library work when torch touches
the GPU first / after libptg?  Usage: probe_libs.py <order: torch-first|lib-first|ptg-first>"""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
order = sys.argv[1]
U = os.path.join(ROOT, "tests", "device_dropin", "_build", "libuser_kernel.so")
if order == "torch-first":
    import torch
    x = torch.zeros(4, device="cuda")
    L = C.CDLL(U)
elif order == "ptg-first":
    sys.path.insert(0, ROOT)
    import ptlumi_loader  # noqa
    from ptlumi import native as N
    N.lib()
    import torch
    x = torch.zeros(4, device="cuda")
    L = C.CDLL(U)
else:
    L = C.CDLL(U)
    import torch
    x = torch.zeros(4, device="cuda")
L.user_selftest.restype = C.c_int
print(order, "selftest", L.user_selftest())
