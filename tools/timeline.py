#!/usr/bin/env python3
"""Concurrency of the last frame in a rocprofv3 kernel trace (tools/timeline.sh):
time with 0 / 1 / 2 / 3+ kernels running, each kind's busy time (union of its
launch intervals), and a coarse strip chart of the frame.
Usage: tools/timeline.py <run_kernel_trace.csv> [bucket_ms]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
bucket = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0


def kind(name):
    m = re.search(r"k_wf_(\w+)<(\w+)", name)
    if m:
        base = m.group(1)
        if base == "walk":
            return "shadow" if m.group(2) == "true" else "extend"
        return base
    m = re.search(r"k_(\w+)\(", name)
    return m.group(1) if m else name[:20]


ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"])) for r in rows]
ev.sort()
cams = [e for e in ev if e[2] == "camera"]
import os
t0 = cams[-int(os.environ.get("TL_CHUNKS", "8"))][0]   # the last frame: its chunks' camera launches (8 at 2^27 paths, 4 at 2^28)
frame = [e for e in ev if e[0] >= t0 and e[2] not in ("fillBufferAligned", "copyBuffer")]
t1 = max(e[1] for e in frame)
wall = (t1 - t0) / 1e6
pts = sorted([(s, 1) for s, _, _ in frame] + [(e, -1) for _, e, _ in frame])
level, last, hist = 0, t0, {}
for t, d in pts:
    hist[min(level, 3)] = hist.get(min(level, 3), 0) + (t - last)
    level += d
    last = t
print("frame wall %.1f ms; time with 0/1/2/3+ kernels: %s" % (
    wall, " / ".join("%.1f" % (hist.get(k, 0) / 1e6) for k in range(4))))
busy = {}
for k in sorted(set(e[2] for e in frame)):
    iv = sorted((s, e) for s, e, kk in frame if kk == k)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    busy[k] = tot / 1e6
print("busy (union) ms: " + ", ".join("%s %.1f" % kv for kv in sorted(busy.items(), key=lambda kv: -kv[1])))
nb = int(wall / bucket) + 1
print("strip chart, %.0f ms buckets: share of each bucket each kind ran" % bucket)
kinds = ["extend", "shadow", "shade", "sky", "classify", "camera", "accumulate"]
print("%8s " % "ms" + " ".join("%9s" % k[:9] for k in kinds))
for b in range(nb):
    bs, be = t0 + int(b * bucket * 1e6), t0 + int((b + 1) * bucket * 1e6)
    line = []
    for k in kinds:
        cov = 0
        for s, e, kk in frame:
            if kk == k:
                cov += max(0, min(e, be) - max(s, bs))
        line.append("%9.2f" % (cov / (be - bs)))
    print("%8.0f " % (b * bucket) + " ".join(line))
