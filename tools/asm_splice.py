#!/usr/bin/env python3
"""SLP root-cause bisection: put one kernel's code, descriptor and metadata
entry from a donor device assembly (e.g. the -fno-slp-vectorize build) into a
host assembly (the SLP build).  Both files must come from the same source, so
the kernel has the same function number (.Lfunc_endN, .LBBN_*).
  asm_splice.py <host.s> <donor.s> <out.s> <kernel label>[,<kernel label>...]"""
import re
import sys


def code_block(lines, func):
    s = next(i for i, l in enumerate(lines) if l.startswith(func + ":"))
    e = next(i for i in range(s + 1, len(lines)) if re.match(r"^\.Lfunc_end\d+:", lines[i]))
    return s, e + 1


def meta_block(lines, func):
    m = next(i for i, l in enumerate(lines) if re.match(r"^\s+\.name:\s+" + re.escape(func) + r"$", l))
    s = max(i for i in range(m) if lines[i].startswith("  - .agpr_count:"))
    e = next((i for i in range(m, len(lines)) if lines[i].startswith("  - ") or lines[i].startswith("amdhsa.target")
              or lines[i].strip().startswith(".end_amdgpu_metadata")), len(lines))
    return s, e


def main():
    host, donor, out, funcs = sys.argv[1:5]
    h = open(host).read().split("\n")
    d = open(donor).read().split("\n")
    for f in funcs.split(","):
        for block in (meta_block, code_block):   # metadata first: it lies after the code
            hs, he = block(h, f)
            ds, de = block(d, f)
            h[hs:he] = d[ds:de]
    open(out, "w").write("\n".join(h))


if __name__ == "__main__":
    main()
