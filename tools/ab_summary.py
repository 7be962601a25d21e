#!/usr/bin/env python3
"""Table of an A/B run (tools/gpu_round.sh STEPS=ab): per library and frame the
best wall time of tools/ablate.py and the per-kernel device times.
Usage: ab_summary.py [dir (default gpurun_out)]"""
import glob
import json
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
rows = []
for p in sorted(glob.glob(os.path.join(d, "ab_*_f*.txt"))):
    m = re.match(r"ab_(\d+)_(.+)_f(\d+)\.txt", os.path.basename(p))
    if not m:
        continue
    line = None
    for l in open(p):
        if l.startswith("{"):
            line = json.loads(l)
    if line:
        rows.append((int(m.group(1)), m.group(2), int(m.group(3)), line))
kinds = ["extend", "shadow", "shade", "sky", "camera", "classify", "accumulate"]
print("%-3s %-10s %6s %10s  %s" % ("run", "lib", "frame", "wall ms", "  ".join("%9s" % k for k in kinds)))
for k, lib, f, line in sorted(rows, key=lambda r: (r[2], r[0])):
    km = line["kernels_ms"]
    print("%-3d %-10s %6d %10.1f  %s" % (k, lib, f, line["wall_ms"], "  ".join("%9.1f" % km.get(x, 0) for x in kinds)))
