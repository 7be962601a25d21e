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
Usage: summarize_prof.py <prof_dir> <tag> [--kernel k_trace]
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_trace<false>")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(a.prof_dir, "trace", "*kernel_stats.csv"))
    kstats = {}
    if stats:
        shutil.copyfile(stats[0], os.path.join(out, "kernel_stats.csv"))
        for row in csv.DictReader(open(stats[0])):
            kstats[row["Name"]] = row
    pmc = collections.defaultdict(list)
    durations = []
    for f in glob.glob(os.path.join(a.prof_dir, "pmc_*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if a.kernel in row["Kernel_Name"]:
                pmc[row["Counter_Name"]].append(float(row["Counter_Value"]))
                durations.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    avg = {k: sum(v) / len(v) for k, v in pmc.items()}
    summary = {"kernel": a.kernel, "dispatches_per_pass": {k: len(v) for k, v in pmc.items()}, "per_dispatch_avg": avg}
    trace_avg_ns = None
    for name, row in kstats.items():
        if a.kernel in name:
            trace_avg_ns = float(row["AverageNs"])
            summary["trace_avg_ms"] = trace_avg_ns / 1e6
            summary["trace_calls"] = int(row["Calls"])
    derived = {}
    if "FETCH_SIZE" in avg:
        derived["fetch_bytes_corrected"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        derived["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "fetch_bytes_corrected" in derived and "write_bytes" in derived:
        derived["hbm_side_bytes"] = derived["fetch_bytes_corrected"] + derived["write_bytes"]
        if trace_avg_ns:
            derived["hbm_side_GBps"] = derived["hbm_side_bytes"] / trace_avg_ns
    if "TCC_HIT_sum" in avg:
        derived["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in avg and trace_avg_ns:
        derived["clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / trace_avg_ns
    if "SQ_INSTS_VALU" in avg and trace_avg_ns and "clock_GHz" in derived:
        cycles = trace_avg_ns * derived["clock_GHz"]
        derived["valu_busy"] = 2 * avg["SQ_INSTS_VALU"] / (1024 * cycles)
    if "SQ_WAVE_CYCLES" in avg:
        derived["wait_any_frac"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        derived["wait_inst_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        if trace_avg_ns and "clock_GHz" in derived:
            derived["avg_waves_per_cu"] = 4 * avg["SQ_WAVE_CYCLES"] / (256 * trace_avg_ns * derived["clock_GHz"])
    summary["derived"] = derived
    with open(os.path.join(out, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    lines = ["# %s profile summary (%s)" % (a.tag, a.kernel), "",
             "| quantity | value |", "|---|---|"]
    if trace_avg_ns:
        lines.append("| rocprofv3 kernel-trace avg duration | %.3f ms (%d calls) |" % (trace_avg_ns / 1e6, summary["trace_calls"]))
    for k, v in derived.items():
        lines.append("| %s | %.4g |" % (k, v))
    for k, v in sorted(avg.items()):
        lines.append("| PMC %s (per dispatch) | %.4g |" % (k, v))
    with open(os.path.join(out, "summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
