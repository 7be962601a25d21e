"""Helper of tests/test_gpu_redo.py, run as its own process so that it loads
the library named by PTG_LIB (libptg_certfail.so: every rounding certificate
of the surface pass fails, so every surface path is shaded by the exact redo
pass).  Renders the listed animation frames at the anim_render_s8.json
configuration through the product path and prints one JSON line: per frame
the image hashes, plus the redo tallies of one counting render."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import ptlumi_loader  # noqa: E402,F401
from ptlumi import native as N  # noqa: E402
from anim_check import image_hashes  # noqa: E402


def main():
    import torch
    from ptlumi.renderer import GpuRenderer
    frames = [int(f) for f in sys.argv[1].split(",")]
    w, h, spp = 160, 90, 8
    cfg = N.RenderConfig.make(w, h, spp, 4)
    s = N.Scene(os.path.join(ROOT, "assets"), cfg)
    r = GpuRenderer(0)
    dev = torch.device("cuda", 0)
    acc = torch.empty((h, w, 4), dtype=torch.float32, device=dev)
    bgra = torch.empty((h, w, 4), dtype=torch.uint8, device=dev)
    out = {"lib": os.path.basename(N.LIB_PATH), "frames": {}}
    for k, f in enumerate(frames):
        s.setup_frame(f)
        r.upload(s, include_static=(k == 0))
        r.render(cfg, out_bgra=bgra, out_accum=acc)
        out["frames"][str(f)] = image_hashes(acc.cpu().numpy(), bgra.cpu().numpy())
    r.enable_counters(True)
    r.render(cfg, out_bgra=bgra, out_accum=acc)
    r.synchronize()
    out["redo"] = r.redo_stats()
    out["shades"] = int(r.counters()[5])
    r.enable_counters(False)
    r.close()
    s.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
