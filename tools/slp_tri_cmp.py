#!/usr/bin/env python3
"""Compare tools/slp_tri outputs of the no-SLP and SLP builds (5 words per
case in the closest-hit form, then 1 word per case in the any-hit form)."""
import sys
import numpy as np
a = np.fromfile(sys.argv[1], dtype=np.uint32)
b = np.fromfile(sys.argv[2], dtype=np.uint32)
n = a.size // 6
full_a, full_b = a[:5 * n].reshape(n, 5), b[:5 * n].reshape(n, 5)
any_a, any_b = a[5 * n:], b[5 * n:]
fd = np.nonzero((full_a != full_b).any(1))[0]
ad = np.nonzero(any_a != any_b)[0]
print("cases", n, "closest-hit form differing:", fd.size, "any-hit form differing:", ad.size)
print("any-hit vs closest-hit verdict (no SLP) differing:", int((any_a != full_a[:, 0]).sum()))
for i in fd[:8]:
    print(" full", int(i), full_a[i].tolist(), full_b[i].tolist())
for i in ad[:8]:
    print(" any", int(i), int(any_a[i]), int(any_b[i]), "closest", full_a[i].tolist())
