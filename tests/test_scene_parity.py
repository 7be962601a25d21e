"""Host scene restatement vs the reference (scene.cc / bvh.cc / mesh.cc).

The arrays that feed the hot path - BVH nodes, the 8 link orders, mesh
indices/positions/normals/albedo/material, TLAS instances and subframes -
must be byte-identical (padding excluded) to what the reference's
load_scene + setup_animation_frame produce, since node order defines the
traversal order and ties between equal hit distances.  Pinned by SHA-256
fixtures generated from the reference built from its sources
(tests/golden/make_golden.py) and, when that build is present, by a direct
array comparison."""
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN, scene_for

from oracle import Reference

FRAMES = [0, 450]


def hashes_of(v):
    raw = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    out = {"nodes": raw(v["nodes"]), "links": raw(v["links"]), "indices": raw(v["indices"]),
           "albedo": raw(v["albedo"]), "material": raw(v["material"]),
           "pos": raw(v["pos"][:, :3]), "normal": raw(v["normal"][:, :3])}
    inst = v["instances"].view(np.uint32).reshape(-1, 40)
    out["instances"] = raw(inst[:, [0, 1, 2, 3, 4, 5] + list(range(8, 40))])
    sf = v["subframes"].view(np.uint32).reshape(-1, 40)
    keep = [0, 1] + [4 + 4 * r + c for r in range(3) for c in range(3)] + [16, 17, 18] + list(range(20, 26)) + \
           [28, 29, 30, 32, 33, 34, 36]
    out["subframes"] = raw(sf[:, keep])
    return out


@pytest.mark.parametrize("frame", FRAMES)
def test_scene_arrays_match_reference_hashes(assets_dir, frame):
    golden = json.load(open(os.path.join(GOLDEN, "scene_hashes.json")))["hashes"][str(frame)]
    v = scene_for(assets_dir, 640, 360, 32, frame=frame).view()
    got = hashes_of(v)
    bad = [k for k in got if got[k] != golden[k]]
    assert not bad, "arrays differing from the reference: %s" % bad
    assert len(v["nodes"]) == golden["counts"]["nodes"]
    assert len(v["instances"]) == golden["counts"]["instances"]
    assert len(v["subframes"]) == golden["counts"]["subframes"]
    assert v["static_instance_count"] == golden["counts"]["static_instance_count"]


def test_scene_structure(assets_dir):
    s = scene_for(assets_dir, 640, 360, 32, frame=0)
    v = s.view()
    assert s.frame_count() == 1800                       # 60 s x 30 fps (scene.cc:720-724)
    assert len(v["links"]) == 8 * len(v["nodes"])       # 8 link orders per node
    assert len(v["subframes"]) == 4                     # ceil(32 / 8) (scene.cc:648-650)
    sn = v["static_node_count"]
    for sf in v["subframes"]:
        count, off = sf["tlas"]
        assert off >= sn and off + count <= len(v["nodes"])
    # every BVH's link targets stay inside the BVH or are the sentinel
    m, b = s.mesh("teapot")
    links = v["links"][8 * b.node_offset: 8 * (b.node_offset + b.node_count)]
    inner = links["accept"][links["accept"] < 0x80000000]
    assert inner.max() < b.node_count
    cancel = links["cancel"]
    assert ((cancel < b.node_count) | (cancel == 0xFFFFFFFF)).all()
    assert ((links["accept"][links["accept"] >= 0x80000000] & 0x7FFFFFFF) < m.triangle_count).all()


def test_frames_reset_state(assets_dir):
    """setup_animation_frame pops the previous frame (scene.cc:274-277): f -> g -> f is stable."""
    s = scene_for(assets_dir, 640, 360, 32, frame=0)
    a = hashes_of(s.view())
    s.setup_frame(1000)
    s.setup_frame(0)
    assert hashes_of(s.view()) == a


@pytest.mark.parametrize("frame", [0, 1400])
def test_scene_arrays_equal_reference_dump(assets_dir, frame):
    ref = Reference("strict", 640, 360, 32, 4)
    if not ref.available():
        pytest.skip("reference build not present (tests/golden hashes cover this)")
    v = scene_for(assets_dir, 640, 360, 32, frame=frame).view()
    with tempfile.TemporaryDirectory() as d:
        ref.dump(assets_dir, frame, d)
        nodes = np.fromfile(os.path.join(d, "nodes.bin"), np.float32).reshape(-1, 6)
        assert np.array_equal(v["nodes"].view(np.float32).reshape(-1, 6).view(np.uint32), nodes.view(np.uint32))
        links = np.fromfile(os.path.join(d, "links.bin"), np.uint32).reshape(-1, 2)
        assert np.array_equal(v["links"].view(np.uint32).reshape(-1, 2), links)
        for name in ["pos", "normal"]:
            a = np.fromfile(os.path.join(d, name + ".bin"), np.uint32).reshape(-1, 4)[:, :3]
            assert np.array_equal(v[name][:, :3].view(np.uint32), a), name
