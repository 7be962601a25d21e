#!/usr/bin/env python3
"""Parity statistics of the reference AS SHIPPED against the strict build
(SURVEY 8(c) tiers T1-T3, verdict r1 item 7).

The GPU path reproduces the reference's strict-IEEE build bit for bit
(tests/test_gpu_*.py).  The reference's own Makefile builds with -O3
-ffast-math -march=native (Makefile:2), which changes its arithmetic - and
its scene arrays (normals, albedo, the BVH) - so the fair question is how far
the shipped build is from the strict one: these are then exactly the
GPU-vs-shipped numbers.  Both builds are the reference's own sources
(oracle/Makefile, REF_MODE=strict and v3 = the shipped flags with a portable
-march), run at 640x360 x 32 spp.

  T1  fraction of (pixel, sample) radiances within 1e-4 relative (all three
      channels; |a - b| <= 1e-4 max(|a|, |b|))
  T2  fraction of pixels whose averaged radiance (j-ordered float32 sum / SPP,
      main.cc:24-42) is within 1e-4 relative; relative difference of the image
      means per channel
  T3  PSNR of the tonemapped 8-bit images at full resolution (validator.py's
      formula, validator.py:43-54, without its 2x downscale: both images are
      at the same resolution) and the fraction of byte-identical pixels

Usage: python tests/golden/parity_stats.py [--frames 0 450] [--rows y0 y1]
writes tests/golden/parity_stats.json (whole frames by default).

  --metric [--spp N]   the same tiers at the metric configuration's image
      (1280x720, N spp, default 256): T2 / T3 over the
      whole frames (the reference's `render`: baseline_render's semantics),
      T1 over the 16-row band 352-368 (per-sample radiances of both builds),
      plus T3v, validator.py's own acceptance figure (validator.py:43-54:
      each image downscaled 2x by the 2x2 mean + truncation, the shipped
      build's as the reference frame); merged into parity_stats.json under
      "metric_config".
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

W, H, SPP, BOUNCES = 640, 360, 32, 4
REL = 1e-4


def within(a, b, rel=REL):
    return np.abs(a - b) <= rel * np.maximum(np.abs(a), np.abs(b))


def accumulate(samples, spp):
    """baseline_render's per-pixel sum in sample order, float32, then / SPP."""
    acc = np.zeros(samples.shape[:2] + (3,), np.float32)
    for j in range(samples.shape[2]):
        acc = acc + samples[:, :, j, :3]
    return acc / np.float32(spp)


def tonemap(acc):
    from oracle import tonemap as orc_tonemap
    flat = np.concatenate([acc.reshape(-1, 3), np.zeros((acc.shape[0] * acc.shape[1], 1), np.float32)], 1)
    return orc_tonemap(flat).reshape(acc.shape[0], acc.shape[1], 4)


def psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))


def frame_stats(assets, frame, y0, y1):
    from oracle import Reference
    samples = {}
    for mode in ("strict", "v3"):
        ref = Reference(mode, W, H, SPP, BOUNCES)
        if not ref.available():
            raise FileNotFoundError(ref.exe)
        samples[mode] = ref.samples(assets, frame, 0, y0, W, y1 - y0, 0, SPP)[..., :3]
    s, v = samples["strict"], samples["v3"]
    t1 = within(s, v).all(-1)
    acc_s, acc_v = accumulate(s, SPP), accumulate(v, SPP)
    t2 = within(acc_s, acc_v).all(-1)
    mean_s = acc_s.reshape(-1, 3).mean(0, dtype=np.float64)
    mean_v = acc_v.reshape(-1, 3).mean(0, dtype=np.float64)
    img_s, img_v = tonemap(acc_s), tonemap(acc_v)
    return {
        "frame": frame, "rows": [y0, y1], "samples": int(t1.size), "pixels": int(t2.size),
        "T1_samples_within_1e-4": round(float(t1.mean()), 5),
        "T2_pixels_within_1e-4": round(float(t2.mean()), 5),
        "T2_image_mean_rel_diff": [round(float(x), 7) for x in np.abs(mean_v - mean_s) / np.abs(mean_s)],
        "T3_psnr_db": round(psnr(img_s[..., :3], img_v[..., :3]), 3),
        "T3_pixels_byte_exact": round(float((img_s == img_v).all(-1).mean()), 5),
    }


def _cached(cache, name, make):
    """make() -> tuple of arrays, saved under cache/name.npz (None: no cache)."""
    if cache:
        p = os.path.join(cache, name + ".npz")
        if os.path.exists(p):
            z = np.load(p)
            return tuple(z["a%d" % i] for i in range(len(z.files)))
    out = make()
    out = out if isinstance(out, tuple) else (out,)
    if cache:
        os.makedirs(cache, exist_ok=True)
        np.savez(p, **{"a%d" % i: x for i, x in enumerate(out)})
    return out


def metric_stats(assets, frame, w, h, spp, band=(352, 368), cache=None):
    """T1 on a band, T2 / T3 / T3v on the whole frame, strict vs shipped, at w x h x spp.
    `cache`: a directory keeping each build's render and band samples (hours of
    CPU time at 1024 spp) so a rerun only recomputes the statistics."""
    from oracle import Reference
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "ptv", os.path.join(ROOT, "path-tracing...but-on-the-lumi-cluster_amd", "validator.py"))
    V = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(V)
    refs = {m: Reference(m, w, h, spp, BOUNCES) for m in ("strict", "v3")}
    for r in refs.values():
        if not r.available():
            raise FileNotFoundError(r.exe)
    acc, bgra = {}, {}
    tag = "f%d_%dx%d_s%d" % (frame, w, h, spp)
    for m, r in refs.items():   # the strict build at 1024 spp: > 1 h
        acc[m], bgra[m] = _cached(cache, "render_%s_%s" % (m, tag), lambda r=r: r.render(assets, frame, timeout=6 * 3600))
    y0, y1 = band
    smp = {m: _cached(cache, "band_%s_%s_%d_%d" % (m, tag, y0, y1),
                      lambda r=r: r.samples(assets, frame, 0, y0, w, y1 - y0, 0, spp, timeout=6 * 3600)[..., :3])[0]
           for m, r in refs.items()}
    t1 = within(smp["strict"], smp["v3"]).all(-1)
    a_s, a_v = acc["strict"][..., :3], acc["v3"][..., :3]
    t2 = within(a_s, a_v).all(-1)
    # a pixel one of whose paths met a zero BSDF pdf accumulates NaN (in the
    # reference too): counted, and left out of the means and the median
    nan_s, nan_v = np.isnan(a_s).any(-1), np.isnan(a_v).any(-1)
    mean_s = np.nanmean(a_s.reshape(-1, 3).astype(np.float64), 0)
    mean_v = np.nanmean(a_v.reshape(-1, 3).astype(np.float64), 0)
    rel = np.abs(a_s - a_v) / np.maximum(np.maximum(np.abs(a_s), np.abs(a_v)), 1e-30)
    worst = rel.max(-1)
    b_s, b_v = bgra["strict"], bgra["v3"]
    ref_half = V.downscale_half(V.bgra_to_rgb(b_v))          # the shipped build's frame as validator.py's reference
    p_val, good = V.validate_frame(ref_half, b_s)
    return {
        "frame": frame, "band_rows": [y0, y1], "samples_in_band": int(t1.size), "pixels": int(t2.size),
        "T1_samples_within_1e-4": round(float(t1.mean()), 5),
        "T2_pixels_within_1e-4": round(float(t2.mean()), 5),
        "T2_pixels_within_1e-3": round(float((worst <= 1e-3).mean()), 5),
        "T2_pixels_within_1e-2": round(float((worst <= 1e-2).mean()), 5),
        "T2_median_rel_diff": float("%.3g" % np.nanmedian(worst)),
        "nan_pixels_strict": int(nan_s.sum()), "nan_pixels_shipped": int(nan_v.sum()),
        "T2_image_mean_rel_diff": [round(float(x), 7) for x in np.abs(mean_v - mean_s) / np.abs(mean_s)],
        "T3_psnr_db": round(psnr(b_s[..., :3], b_v[..., :3]), 3),
        "T3_pixels_byte_exact": round(float((b_s == b_v).all(-1).mean()), 5),
        "T3v_validator_psnr_db": round(float(p_val), 3), "T3v_validator_good": bool(good),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--metric", action="store_true")
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--frames", type=int, nargs="*", default=[0, 450])
    ap.add_argument("--rows", type=int, nargs=2, default=[0, H])
    ap.add_argument("--out", default=os.path.join(HERE, "parity_stats.json"))
    ap.add_argument("--cache", default=None, help="keep the reference builds' renders here (--metric)")
    a = ap.parse_args()
    assets = os.path.join(ROOT, "assets")
    if a.metric:
        w, h = 1280, 720
        res = json.load(open(a.out)) if os.path.exists(a.out) else {}
        rows = res.setdefault("metric_config", {"width": w, "height": h, "bounces": BOUNCES, "rows": []})["rows"]
        for f in a.frames:
            st = metric_stats(assets, f, w, h, a.spp, cache=a.cache)
            st["spp"] = a.spp
            rows[:] = [r for r in rows if (r["frame"], r["spp"]) != (f, a.spp)] + [st]
            rows.sort(key=lambda r: (r["spp"], r["frame"]))
            with open(a.out, "w") as fh:
                json.dump(res, fh, indent=1)
            print(json.dumps(st, indent=1))
        return
    res = {"config": {"width": W, "height": H, "spp": SPP, "bounces": BOUNCES,
                      "builds": {"strict": "-O2 -ffp-contract=off -fno-fast-math (== the GPU path, bit for bit)",
                                 "v3": "-O3 -ffast-math -march=x86-64-v3 (the reference Makefile's flags, "
                                       "portable -march)"}},
           "frames": [frame_stats(assets, f, *a.rows) for f in a.frames]}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
