#!/usr/bin/env python3
"""Per-dispatch averages of the walk kernels' counters from tools/profile_walk.sh.
Usage: walk_counters.py gpurun_out/pw_<tag>"""
import csv, glob, json, os, sys, collections

def rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)

base = sys.argv[1]
out = {}
for lib in sorted(os.listdir(base)):
    d = os.path.join(base, lib)
    res = {}
    for k in ("k_wf_walk<false, false>", "k_wf_walk<true, false>"):
        acc = collections.defaultdict(list)
        for fn in glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            for r in rows(fn):
                if k in r.get("Kernel_Name", ""):
                    per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            by = collections.defaultdict(list)
            for (disp, name), v in per.items():
                by[name].append(v)
            for name, vs in by.items():
                acc[name].append(sum(vs) / len(vs))
        tr = []
        for fn in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
            for r in rows(fn):
                if k in r.get("Kernel_Name", ""):
                    tr.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        res[k] = {"ms_total": round(sum(tr), 3), "launches": len(tr), **{n: sum(v) / len(v) for n, v in acc.items()}}
    out[lib] = res
print(json.dumps(out, indent=1))
