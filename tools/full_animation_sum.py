#!/usr/bin/env python3
"""Adds up tools/full_animation.py's parts into the whole animation's figure:
every frame 0..1799 rendered exactly once, the parts' wall times summed
(each part is one process on one GPU, run one after another), frames/min =
frames / total wall.  Also the per-frame render times (HIP events) by
frame, their distribution and the slowest frames.

Usage: python tools/full_animation_sum.py OUT.json PART.json [PART.json ...]
"""
import json
import sys


def main():
    out, parts = sys.argv[1], [json.load(open(p)) for p in sys.argv[2:]]
    cfgs = {json.dumps(p["config"], sort_keys=True) for p in parts}
    assert len(cfgs) == 1, cfgs
    ms, sha = {}, {}
    for p in parts:
        for f, t, h in zip(p["frames"], p["frame_ms"], p["bgra_sha"]):
            assert f not in ms, "frame %d rendered twice" % f
            ms[f], sha[f] = t, h
    frames = sorted(ms)
    assert frames == list(range(len(frames))), "frames missing"
    cfg = parts[0]["config"]
    wall = sum(p["wall_s"] for p in parts)
    per = sorted(ms.values())
    res = {"config": cfg, "frames": len(frames), "parts": len(parts),
           "wall_s": round(wall, 2), "full_animation_min": round(wall / 60.0, 2),
           "frames_per_min": round(len(frames) / wall * 60.0, 3),
           "msamples_per_s": round(len(frames) * cfg["width"] * cfg["height"] * cfg["spp"] / wall / 1e6, 2),
           "render_ms": {"sum": round(sum(per), 1), "min": per[0], "median": per[len(per) // 2], "max": per[-1]},
           "slowest_frames_ms": sorted(([f, ms[f]] for f in frames), key=lambda x: -x[1])[:10],
           "frame_ms_by_100": [round(sum(ms[f] for f in frames[i:i + 100]) / 100.0, 1) for i in range(0, len(frames), 100)],
           "parts_frames_per_min": [p["frames_per_min"] for p in parts],
           "bgra_sha": [sha[f] for f in frames]}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "bgra_sha"}, indent=1))


if __name__ == "__main__":
    main()
