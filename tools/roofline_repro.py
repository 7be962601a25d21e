#!/usr/bin/env python3
"""Recompute a bench line's roofline from the committed profiles alone.

bench.py reports, for the closest-hit walk (the dominant kernel), the time
floor of one launch at every level of the memory / issue hierarchy: the
launch's count at that level (per dispatch, from the rocprofv3 PMC passes of
the same workload: profiles/<tag>/pmc_summary.json) over the ceiling measured
on MI355X for the walk's access shape (profiles/r02_probe/ceilings.json).  The
largest floor names the bound; frac = floor / launch time.  This script
redoes that arithmetic from the files the bench line cites, with the launch
time taken two ways:

  * isolated: the bench line's own HIP-event time of the kernel alone;
  * rocprof:  the kernel-trace average of the same profile (kernel_stats.csv),

and checks that its numbers equal the bench line's (1e-3 relative) and that
the two launch times agree (15%, the bench's own acceptance rule).

Usage: roofline_repro.py [bench_line.json]   (default: the newest profiles/*/bench_line.json with a profile-backed roofline)
"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK = 8000e9


def natural(p):
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", p)]


def levels_of(ent, ceil):
    pmc, d = ent["per_dispatch_avg"], ent["derived"]
    clock = d.get("clock_GHz") or 2.4
    lv = {
        "vmem_issue": (pmc["SQ_INSTS_VMEM"], ceil["vmem_issue_per_s"]),
        "l2": (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"], ceil["l2_lines_per_s"]),
        "fabric": (pmc["TCC_MISS_sum"], ceil["ic_lines_per_s"]),
        "hbm": (d["hbm_side_bytes"], HBM_PEAK),
    }
    if "SQ_INSTS_VALU" in pmc:
        lv["valu_issue"] = (pmc["SQ_INSTS_VALU"] * 2.0, 1024 * clock * 1e9)
    if "SQ_INSTS_SALU" in pmc:
        lv["salu_issue"] = (pmc["SQ_INSTS_SALU"], 256 * clock * 1e9)
    return lv


TRACE_NAME = {"extend": "k_wf_walk<false, false>", "shadow": "k_wf_walk<true, false>"}


def trace_ms_of(prof_path, kind):
    stats = os.path.join(os.path.dirname(prof_path), "kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        if TRACE_NAME[kind] in r["Name"]:
            return float(r["AverageNs"]) / 1e6
    return None


def check_levels(ent, ceil, iso_ms, trace_ms, want_levels, label):
    """Recompute every level's floor; compare frac_isolated (and, where the line
    has them, the count and ceiling) with the line.  Returns (ok, floors)."""
    ok = True
    floors = {}
    print("%-11s %16s %16s %12s %10s %10s" % ("level", "count/launch", "ceiling/s", "floor ms", "frac_iso", "frac_rocprof"))
    for name, (count, rate) in levels_of(ent, ceil).items():
        t = count / rate
        floors[name] = t
        fi, fr = t / (iso_ms / 1e3), t / (trace_ms / 1e3)
        print("%-11s %16.4g %16.4g %12.4f %10.4f %10.4f" % (name, count, rate, t * 1e3, fi, fr))
        want = want_levels[name]
        for k, mine in (("count_per_launch", count), ("ceiling_per_s", rate), ("frac_isolated", fi)):
            if k not in want:
                continue
            if abs(want[k] - mine) > 1e-3 * max(abs(want[k]), 1e-12) + 5e-4 * (k == "frac_isolated"):
                print("  MISMATCH %s %s.%s: bench %r, recomputed %r" % (label, name, k, want[k], mine))
                ok = False
    return ok, floors


def repro_roofline(rf, label):
    """One roofline block of a bench line (the metric frame's or the heavy
    frame's): the closest-hit walk's levels, then each walk's in `walks`."""
    ok = True
    if rf.get("traffic_source"):
        prof_path = os.path.join(ROOT, rf["traffic_source"].split(" ")[0])
        prof = json.load(open(prof_path))
        ceil = json.load(open(os.path.join(ROOT, rf["ceilings_source"])))
        trace_ms = trace_ms_of(prof_path, "extend")
        iso_ms = rf["isolated"]["ms_per_launch"]
        print("== %s: %s, PMC profile %s (workload %r), ceilings %s" % (label, rf.get("kernel"), os.path.relpath(prof_path, ROOT),
                                                                     prof.get("_workload"), rf["ceilings_source"]))
        print("launch time: isolated (HIP events) %.4f ms, rocprof trace avg %.4f ms" % (iso_ms, trace_ms))
        ok = abs(trace_ms - iso_ms) <= 0.15 * iso_ms
        lok, floors = check_levels(prof["extend"], ceil, iso_ms, trace_ms, rf["levels"], label)
        bound = max(floors, key=floors.get)
        print("bound: %s (bench: %s); frac isolated %.4f (bench %.4f), frac rocprof %.4f" %
              (bound, rf["bound"], floors[bound] / (iso_ms / 1e3), rf["isolated"]["frac"], floors[bound] / (trace_ms / 1e3)))
        ok = ok and lok and bound == rf["bound"] and abs(floors[bound] / (iso_ms / 1e3) - rf["isolated"]["frac"]) < 1e-3
    for kind, wl in (rf.get("walks") or {}).items():
        if not wl.get("source"):
            continue
        prof_path = os.path.join(ROOT, wl["source"])
        prof = json.load(open(prof_path))
        ceil = json.load(open(os.path.join(ROOT, rf.get("ceilings_source") or "profiles/r02_probe/ceilings.json")))
        trace_ms = trace_ms_of(prof_path, kind)
        iso_ms = wl["ms_per_launch_isolated"]
        print("== %s, walk %s: isolated %.4f ms, rocprof trace avg %.4f ms" % (label, kind, iso_ms, trace_ms))
        kok = abs(trace_ms - iso_ms) <= 0.15 * iso_ms
        lok, floors = check_levels(prof[kind], ceil, iso_ms, trace_ms, wl["levels"], "%s/%s" % (label, kind))
        bound = max(floors, key=floors.get)
        print("bound: %s (bench: %s); frac isolated %.4f (bench %.4f)" %
              (bound, wl["bound"], floors[bound] / (iso_ms / 1e3), wl["frac_isolated"]))
        ok = ok and kok and lok and bound == wl["bound"] and abs(floors[bound] / (iso_ms / 1e3) - wl["frac_isolated"]) < 1e-3
    return ok


def main():
    if len(sys.argv) > 1:
        path = sys.argv[1]
    else:   # the newest bench line whose roofline cites a committed PMC profile (config runs without one are skipped)
        path = [p for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "bench_line.json")), key=natural)
                if "traffic_source" in (json.load(open(p)).get("roofline") or {})][-1]
    line = json.load(open(path))
    print("bench line:", os.path.relpath(path, ROOT))
    ok = repro_roofline(line["roofline"], "metric frame")
    heavy = (line.get("heavy_frame") or {}).get("roofline")
    if heavy:
        ok = repro_roofline(heavy, "heavy frame %d" % line["heavy_frame"]["frame"]) and ok
    print("reproduced" if ok else "NOT reproduced")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
