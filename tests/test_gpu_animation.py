"""Every animation frame rendered on the GPU, whole, against the reference
(north_star: "every frame validator-clean").

The reference built from its own sources rendered all 1800 frames of the
animation (scene.cc:720-724) at 160x90 x 8 spp with baseline_render's
semantics (main.cc:12-46) and hashed each whole image: the averaged radiance
(float32 bits) and the tonemapped BGRA bytes (tests/golden/make_anim_golden.py,
anim_render_s8.json).  Here every frame goes through the product's own
per-frame path - host setup_frame (the scene restatement), ptg_upload_frame,
ptg_render - and both hashes must match for every frame: bit-identical images,
so validator.py's PSNR test passes trivially (infinite PSNR).  The frame's
scene arrays are checked against the reference's per-frame hashes on the way.
"""
import json
import os
import time

import numpy as np
import pytest

from anim_check import image_hashes, scene_frame_hashes
from conftest import GOLDEN, ROOT, N

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_every_frame_bit_identical_to_reference(assets_dir):
    import torch
    from ptlumi.renderer import GpuRenderer
    golden = json.load(open(os.path.join(GOLDEN, "anim_render_s8.json")))
    scene_golden = json.load(open(os.path.join(GOLDEN, "anim_scene_s8.json")))["frames"]
    w, h, spp = golden["width"], golden["height"], golden["spp"]
    frames = sorted(golden["frames"], key=int)
    assert len(frames) == 1800
    cfg = N.RenderConfig.make(w, h, spp, 4)
    s = N.Scene(assets_dir, cfg)
    r = GpuRenderer(0)
    dev = torch.device("cuda", 0)
    acc = torch.empty((h, w, 4), dtype=torch.float32, device=dev)
    bgra = torch.empty((h, w, 4), dtype=torch.uint8, device=dev)
    progress = os.path.join(ROOT, "gpurun_out", "anim_progress.txt")
    log = open(progress, "w") if os.path.isdir(os.path.dirname(progress)) else None
    bad_scene, bad_image = [], []
    t0 = time.time()
    try:
        for k, f in enumerate(frames):
            s.setup_frame(int(f))
            sh = scene_frame_hashes(s.view())
            if sh != scene_golden[f]:
                bad_scene.append(int(f))
            r.upload(s, include_static=(k == 0))
            r.render(cfg, out_bgra=bgra, out_accum=acc)
            got = image_hashes(acc.cpu().numpy(), bgra.cpu().numpy())
            if got != golden["frames"][f]:
                bad_image.append(int(f))
            if log and k % 100 == 99:
                log.write("%d frames, %.1f s, %d mismatched\n" % (k + 1, time.time() - t0, len(bad_image)))
                log.flush()
    finally:
        r.close()
        s.close()
        if log:
            log.close()
    print("1800 frames in %.1f s" % (time.time() - t0))
    assert not bad_scene, "%d frames with scene arrays differing from the reference: %s" % (len(bad_scene), bad_scene[:20])
    assert not bad_image, "%d frames not bit-identical to the reference: %s" % (len(bad_image), bad_image[:20])
