"""Per-frame hashes of the animation, computed the way the reference harness
computes them (oracle/ref_harness.cc anim_hashes / anim_render), so that the
product's arrays and images can be compared with the whole-animation
fixtures of tests/golden/make_anim_golden.py.  Helper module of the tests."""
import hashlib
import os
import sys

import numpy as np

DIGITS = 32
# words of the 160-byte records that carry data (padding excluded), as in
# make_golden.py's scene_hashes and ref_harness.cc's kInstKeep / kSubKeep
INST_KEEP = [0, 1, 2, 3, 4, 5] + list(range(8, 40))
SUB_KEEP = [0, 1] + [4 + 4 * r + c for r in range(3) for c in range(3)] + [16, 17, 18] + list(range(20, 26)) + \
           [28, 29, 30, 32, 33, 34, 36]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:DIGITS]


def scene_frame_hashes(v):
    """{counts and hashes} of one frame's per-frame arrays (Scene.view())."""
    sn = int(v["static_node_count"])
    inst = v["instances"].view(np.uint32).reshape(-1, 40)[:, INST_KEEP]
    sub = v["subframes"].view(np.uint32).reshape(-1, 40)[:, SUB_KEEP]
    return {"instances": len(v["instances"]), "subframes": len(v["subframes"]), "tlas_nodes": len(v["nodes"]) - sn,
            "sha_instances": sha(inst), "sha_subframes": sha(sub), "sha_tlas_nodes": sha(v["nodes"][sn:]),
            "sha_tlas_links": sha(v["links"][8 * sn:])}


def image_hashes(acc, bgra):
    """(radiance xyz f32 bits [H][W][3], BGRA [H][W][4]) hashes of a rendered frame."""
    rad = np.ascontiguousarray(np.asarray(acc, np.float32)[..., :3])
    return {"sha_radiance": sha(rad.view(np.uint32)), "sha_bgra": sha(np.asarray(bgra, np.uint8))}


def scene_hash_range(args):
    """Worker: load the scene once, set up frames [f0, f1) in order, hash each."""
    root, w, h, spp, f0, f1 = args
    sys.path.insert(0, root)
    import ptlumi_loader  # noqa: F401
    from ptlumi import native as N
    s = N.Scene(os.path.join(root, "assets"), N.RenderConfig.make(w, h, spp, 4))
    out = {}
    for f in range(f0, f1):
        s.setup_frame(f)
        out[str(f)] = scene_frame_hashes(s.view())
    s.close()
    return out
