#!/usr/bin/env python3
"""Ceilings for the walk's roofline from tools/probe_pmc.sh output.

tools/_bin/ta_probe issues wave-level 16-B-per-lane gathers in the walk's
access shape: every active lane reads its own random 64-B line.  The sweep over
table sizes gives the time per wave-instruction per CU with the lines served
by the L2 (table <= 4 MiB per XCD), the Infinity Cache (16-256 MiB) or HBM
(>= 384 MiB); the PMC passes confirm that each lane-line is one L2 request
(TCC_HIT + TCC_MISS per lane-line ~ 1).  Written to
profiles/r02_probe/ceilings.json for bench.py's hierarchy_roofline():

  vmem_issue_per_s  wave-instructions per second, chip-wide, at the per-CU
                    floor (the fastest instruction measured: one active lane or
                    one address per wave - an instruction that moves almost
                    nothing still occupies the vector memory path this long)
  l2_lines_per_s    random 64-B L2-hit line requests per second (64 per
                    instruction, L2-resident table)
  ic_lines_per_s    random 64-B line requests per second that miss the L2
                    (Infinity Cache / HBM tables: the same rate)
Usage: tools/make_ceilings.py <probe_pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import re
import sys

CUS, WAVES, ITERS = 256, 32, 2048


def main():
    src, out = sys.argv[1], sys.argv[2]
    rows = {}
    for line in open(os.path.join(src, "sizes.txt")):
        m = re.match(r"\s*(\d+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s*$", line)
        if m:
            rows[int(m.group(1))] = [float(m.group(k)) for k in (2, 3, 4)]
    l2 = [rows[s] for s in rows if s <= 4]
    ic = [rows[s] for s in rows if 16 <= s <= 256]
    hbm = [rows[s] for s in rows if s >= 384]
    ns_floor = min(r[2] for r in l2)
    # the first sweep (ta_probe.txt, 64 MiB table, every mode and lane count):
    # its fastest instruction is the issue floor when it is lower
    first = os.path.join(os.path.dirname(out), "ta_probe.txt")
    if os.path.exists(first):
        vals = [float(x) for line in open(first) if re.match(r"\s+\d+\s", line) for x in line.split()[1:]]
        ns_floor = min([ns_floor] + vals)
    ns_l2 = sum(r[0] for r in l2) / len(l2)
    ns_ic = sum(r[0] for r in ic if True) / len(ic)
    ns_hbm = sum(r[0] for r in hbm) / len(hbm)
    # lines per L2 request in the calibration passes
    calib = {}
    for f in glob.glob(os.path.join(src, "*_TCC_HIT_sum_TCC_MISS_sum", "*counter_collection.csv")):
        tag = os.path.basename(os.path.dirname(f)).split("_TCC")[0]
        mib, active, mode, nbytes = (int(x) for x in tag.split("_"))
        vals = {}
        for r in csv.DictReader(open(f)):
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        req = sum(v[-1] for v in vals.values())          # the timed (second) dispatch
        lines = CUS * WAVES * ITERS * (active if mode == 0 else active // 4)
        calib[tag] = {"l2_requests": req, "lane_lines": lines, "requests_per_line": round(req / lines, 4),
                      "hit": vals["TCC_HIT_sum"][-1], "miss": vals["TCC_MISS_sum"][-1]}
    res = {
        "vmem_issue_per_s": CUS / (ns_floor * 1e-9),
        "l2_lines_per_s": CUS * 64 / (ns_l2 * 1e-9),
        "ic_lines_per_s": CUS * 64 / (min(ns_ic, ns_hbm) * 1e-9),
        "ns_per_instruction_per_cu": {"floor_1_lane_l2": ns_floor, "64_lines_l2": ns_l2, "64_lines_ic": ns_ic,
                                      "64_lines_hbm": ns_hbm},
        "calibration": calib,
        "source": "tools/ta_probe.hip via tools/probe_pmc.sh (sizes.txt + rocprofv3 --pmc passes)",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
