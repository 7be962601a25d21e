"""Scene assets: deterministic substitutes + byte copies of the reference meshes."""
import hashlib
import os

from conftest import ASSETS
from ptlumi import assets as A


def manifest(assets_dir):
    out = {}
    for line in open(os.path.join(assets_dir, "MANIFEST")):
        h, name = line.split()
        out[name] = h
    return out


def test_substitutes_are_deterministic(assets_dir):
    m = manifest(assets_dir)
    assert hashlib.sha256(A._terrain_obj().encode()).hexdigest() == m["terrain.obj"]
    for name in A.MISSING:
        assert name in m
    # 17 meshes of load_scene (scene.cc:139-182) + their materials
    assert sum(1 for n in m if n.endswith(".obj")) == 18


def test_every_asset_present_and_hashed(assets_dir):
    for name, h in manifest(assets_dir).items():
        with open(os.path.join(assets_dir, "data", name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == h, name
