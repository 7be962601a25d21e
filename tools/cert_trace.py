#!/usr/bin/env python3
"""Diagnostics with the cert_trace variant (PTG_LIB=<pkg>/_build/ablate_certtrace/libptg.so):
render frame 0 at 64 spp, print the recorded failing certificate inputs."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], "--spp", "64", "--reps", "1"]
exec(open(os.path.join(ROOT, "tools", "ablate.py")).read())

vals = np.zeros(256, np.float64)
n = C.c_uint(0)
N.lib().ptg_debug_cert_values(vals.ctypes.data_as(C.c_void_p), C.byref(n))
print("failures recorded:", n.value)
for k in range(min(64, n.value)):
    r, x, q, v = vals[4 * k:4 * k + 4]
    print("r=%r bpdf=%r q=%r v=%r" % (r, x, q, v))
