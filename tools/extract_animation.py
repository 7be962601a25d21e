#!/usr/bin/env python3
"""Extract the reference's hard-coded keyframe table into a data file.

The reference animates its scene with a literal table of ~300
``animation_stop {start, duration, from, to, &variable}`` entries
(``/root/reference/scene.cc:319-627``), replayed by ``play_animation_track``
(``scene.cc:33-42``).  That table is scene *data*; this script lifts it,
unchanged, into ``<package>/data/animation_track.csv`` so the host-side scene
restatement can replay it.  Each numeric field keeps its source literal text:
the loader reproduces the C++ conversion rules exactly (``1.5f`` -> strtof;
``-90.6`` -> strtod then cast to float; ``camera_start_pos.x`` -> that
constant), so the replayed values are bit-identical to the reference's.

Usage: python tools/extract_animation.py [/root/reference/scene.cc] [out.csv]
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "path-tracing...but-on-the-lumi-cluster_amd")

ENTRY = re.compile(r"^\s*\{\s*([^,]+?)\s*,\s*([^,]+?)\s*,\s*([^,]+?)\s*,\s*([^,]+?)\s*,\s*&([\w.]+)\s*\}\s*,?\s*(//.*)?$")


def extract(src_path):
    with open(src_path) as f:
        lines = f.read().split("\n")
    start = next(i for i, l in enumerate(lines) if "animation_stop anim[]" in l)
    rows = []
    for line in lines[start + 1:]:
        if line.strip().startswith("};"):
            break
        m = ENTRY.match(line)
        if m:
            rows.append(m.groups()[:5])
        elif line.strip() and not line.strip().startswith("//"):
            raise ValueError("unparsed keyframe line: %r" % line)
    return rows


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/scene.cc"
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(PKG, "data", "animation_track.csv")
    rows = extract(src)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        f.write("# keyframes of the reference animation (scene.cc:319-627), source literals kept\n")
        f.write("# start,duration,from,to,variable\n")
        for r in rows:
            f.write(",".join(r) + "\n")
    print("wrote %d keyframes to %s" % (len(rows), out))


if __name__ == "__main__":
    main()
