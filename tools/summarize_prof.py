#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh output directory into profiles/<tag>/.

Writes kernel_stats.csv (rocprofv3 --kernel-trace --stats), pmc_summary.json
(per-dispatch averages of every PMC counter for the kernels matching
--kernel) and a short summary.md with the derived numbers:
  * HBM-side bytes per dispatch = FETCH_SIZE x 1024 x 2 (gfx950 reports 1/2 of
    wide streaming reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE x 1024;
  * L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS);
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch time;
  * VALU busy = 2 cycles x SQ_INSTS_VALU / (1024 SIMDs x cycles).
Usage: summarize_prof.py <prof_dir> <tag> [--kernels extend,shadow,shade,...]
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


KERNELS = {"extend": "k_wf_walk<false, false>", "shadow": "k_wf_walk<true, false>",
           "shade": "k_wf_shade<false, ptg::dm::MathFast>", "shade_exact": "k_wf_shade<false, ptg::dm::MathExact>",
           "camera": "k_wf_camera<false>", "accumulate": "k_accumulate", "megakernel": "k_trace<false>",
           "sky": "k_wf_sky<false>", "classify": "k_wf_classify"}


def derive(avg, trace_avg_ns):
    d = {}
    if "FETCH_SIZE" in avg:
        d["fetch_bytes_corrected"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        d["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "fetch_bytes_corrected" in d and "write_bytes" in d:
        d["hbm_side_bytes"] = d["fetch_bytes_corrected"] + d["write_bytes"]
        if trace_avg_ns:
            d["hbm_side_GBps"] = d["hbm_side_bytes"] / trace_avg_ns
    if "TCC_HIT_sum" in avg:
        d["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in avg and trace_avg_ns:
        d["clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / trace_avg_ns
    if "SQ_INSTS_VALU" in avg and trace_avg_ns and "clock_GHz" in d:
        d["valu_busy"] = 2 * avg["SQ_INSTS_VALU"] / (1024 * trace_avg_ns * d["clock_GHz"])
    if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
        d["wait_any_frac"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        d["wait_inst_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        if trace_avg_ns and "clock_GHz" in d:
            d["avg_waves_per_cu"] = 4 * avg["SQ_WAVE_CYCLES"] / (256 * trace_avg_ns * d["clock_GHz"])
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--workload", default="frame 0, 1280x720, 1024 spp, 4 bounces",
                    help="bench workload the profile was taken on (bench.py reads traffic only on a match)")
    ap.add_argument("--kernels", default="extend,shadow,shade,sky,classify,camera,accumulate",
                    help="comma list of " + ",".join(KERNELS))
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(a.prof_dir, "trace", "*kernel_stats.csv"))
    kstats = {}
    if stats:
        shutil.copyfile(stats[0], os.path.join(out, "kernel_stats.csv"))
        for row in csv.DictReader(open(stats[0])):
            kstats[row["Name"]] = row
    rows = []
    for f in glob.glob(os.path.join(a.prof_dir, "pmc_*", "*counter_collection.csv")):
        rows.extend(csv.DictReader(open(f)))
    summary = {"_workload": a.workload}
    lines = ["# %s rocprofv3 summary" % a.tag, ""]
    for kind in a.kernels.split(","):
        pat = KERNELS[kind]
        pmc = collections.defaultdict(list)
        for row in rows:
            if pat in row["Kernel_Name"]:
                pmc[row["Counter_Name"]].append(float(row["Counter_Value"]))
        avg = {k: sum(v) / len(v) for k, v in pmc.items()}
        ent = {"kernel": pat, "dispatches_per_pass": {k: len(v) for k, v in pmc.items()}, "per_dispatch_avg": avg}
        trace_avg_ns = None
        for name, row in kstats.items():
            if pat in name:
                trace_avg_ns = float(row["AverageNs"])
                ent["trace_avg_ms"] = trace_avg_ns / 1e6
                ent["trace_calls"] = int(row["Calls"])
                ent["trace_total_ms"] = float(row["TotalDurationNs"]) / 1e6
        ent["derived"] = derive(avg, trace_avg_ns)
        summary[kind] = ent
        lines += ["## %s (`%s`)" % (kind, pat), "", "| quantity | value |", "|---|---|"]
        if trace_avg_ns:
            lines.append("| rocprofv3 kernel-trace avg duration | %.4f ms (%d calls, %.1f ms total) |"
                         % (trace_avg_ns / 1e6, ent["trace_calls"], ent["trace_total_ms"]))
        for k, v in ent["derived"].items():
            lines.append("| %s | %.4g |" % (k, v))
        for k, v in sorted(avg.items()):
            lines.append("| PMC %s (per dispatch) | %.4g |" % (k, v))
        lines.append("")
    with open(os.path.join(out, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    with open(os.path.join(out, "summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
