"""Scene asset preparation.

The reference renders an OBJ/MTL scene loaded from ``data/`` relative to the
working directory (``scene.cc:139-182``).  Three of its meshes are absent from
the reference tree (``.MISSING_LARGE_BLOBS:1-3``: terrain, bunny, pine_tree),
so ``load_scene`` would exit at ``mesh.cc:25-29``.  This module assembles a
self-contained asset directory ``<dest>/data`` that both the reference build
(the test oracle's checker) and this framework load:

* every OBJ/MTL the reference ships is copied byte-for-byte;
* the three missing meshes are replaced by deterministic substitutes
  (SURVEY.md §8c recipe):
    - ``terrain.obj``: 129x129 heightfield over x,z in [-110, 110],
      ``y = 10 + 14 sin(0.05 x) cos(0.04 z)``, analytic normals,
      ``usemtl Material.003``, plus a 2-triangle water quad at y = 0.5 with
      ``usemtl Material.001`` (its ``Tf`` makes it transmissive, which also
      excludes it from object placement, ``scene.cc:118-120``);
    - ``bunny.obj``: ``teapot.obj`` with mtllib/usemtl renamed to
      ``bunny.mtl`` / ``Material.024``;
    - ``pine_tree.obj``: ``leaf_tree.obj`` renamed to ``pine_tree.mtl`` /
      ``Material.010`` / ``Material.011``.

The generator is pure Python with fixed ``%.6f`` formatting, so the bytes are
identical on every machine.  The GPU box receives the prepared directory with
the repository snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import hashlib
import math
import os
import shutil

REFERENCE_DATA = "/root/reference/data"
MISSING = ("terrain.obj", "bunny.obj", "pine_tree.obj")

TERRAIN_N = 129
TERRAIN_EXTENT = 110.0
WATER_Y = 0.5


def _terrain_obj() -> str:
    n = TERRAIN_N
    out = ["# substitute terrain (SURVEY.md 8c): y = 10 + 14 sin(0.05x) cos(0.04z)",
           "mtllib terrain.mtl", "o Terrain"]
    coords = [(-TERRAIN_EXTENT + 2.0 * TERRAIN_EXTENT * i / (n - 1)) for i in range(n)]
    # vertices: index (i, j) -> 1 + i*n + j, x = coords[i], z = coords[j]
    for x in coords:
        for z in coords:
            y = 10.0 + 14.0 * math.sin(0.05 * x) * math.cos(0.04 * z)
            out.append("v %.6f %.6f %.6f" % (x, y, z))
    for x in coords:
        for z in coords:
            dydx = 0.7 * math.cos(0.05 * x) * math.cos(0.04 * z)
            dydz = -0.56 * math.sin(0.05 * x) * math.sin(0.04 * z)
            nx, ny, nz = -dydx, 1.0, -dydz
            inv = 1.0 / math.sqrt(nx * nx + ny * ny + nz * nz)
            out.append("vn %.6f %.6f %.6f" % (nx * inv, ny * inv, nz * inv))
    # water quad vertices / normal
    wbase = n * n
    e = TERRAIN_EXTENT
    for (x, z) in ((-e, -e), (-e, e), (e, -e), (e, e)):
        out.append("v %.6f %.6f %.6f" % (x, WATER_Y, z))
    out.append("vn 0.000000 1.000000 0.000000")
    out.append("usemtl Material.003")
    out.append("s 1")

    def vid(i, j):
        return 1 + i * n + j

    # counter-clockwise seen from +y: (i,j) -> (i,j+1) -> (i+1,j)
    for i in range(n - 1):
        for j in range(n - 1):
            a, b, c, d = vid(i, j), vid(i, j + 1), vid(i + 1, j), vid(i + 1, j + 1)
            out.append("f %d//%d %d//%d %d//%d" % (a, a, b, b, c, c))
            out.append("f %d//%d %d//%d %d//%d" % (c, c, b, b, d, d))
    out.append("usemtl Material.001")
    out.append("s 0")
    w0, w1, w2, w3 = wbase + 1, wbase + 2, wbase + 3, wbase + 4
    wn = n * n + 1
    out.append("f %d//%d %d//%d %d//%d" % (w0, wn, w1, wn, w2, wn))
    out.append("f %d//%d %d//%d %d//%d" % (w2, wn, w1, wn, w3, wn))
    return "\n".join(out) + "\n"


def _renamed(src_text: str, renames: dict) -> str:
    lines = []
    for line in src_text.split("\n"):
        parts = line.split(" ", 1)
        if len(parts) == 2 and parts[0] in ("mtllib", "usemtl") and parts[1] in renames:
            line = parts[0] + " " + renames[parts[1]]
        lines.append(line)
    return "\n".join(lines)


def prepare(dest: str, reference_data: str = REFERENCE_DATA, force: bool = False) -> str:
    """Create ``<dest>/data`` with the full scene.  Returns ``dest``.

    If the directory is already complete (a ``MANIFEST`` file is present) and
    ``force`` is false, nothing is rewritten, so this is cheap to call.
    """
    data = os.path.join(dest, "data")
    manifest = os.path.join(dest, "MANIFEST")
    if os.path.exists(manifest) and not force:
        return dest
    if not os.path.isdir(reference_data):
        raise FileNotFoundError(
            "scene assets missing: %s has no MANIFEST and the reference data "
            "directory %s is not available to rebuild it" % (dest, reference_data))
    os.makedirs(data, exist_ok=True)
    for name in sorted(os.listdir(reference_data)):
        if name.endswith((".obj", ".mtl")):
            shutil.copyfile(os.path.join(reference_data, name), os.path.join(data, name))
    with open(os.path.join(data, "terrain.obj"), "w", newline="\n") as f:
        f.write(_terrain_obj())
    with open(os.path.join(reference_data, "teapot.obj")) as f:
        teapot = f.read()
    with open(os.path.join(data, "bunny.obj"), "w", newline="\n") as f:
        f.write(_renamed(teapot, {"teapot.mtl": "bunny.mtl", "Material.005": "Material.024"}))
    with open(os.path.join(reference_data, "leaf_tree.obj")) as f:
        leaf = f.read()
    with open(os.path.join(data, "pine_tree.obj"), "w", newline="\n") as f:
        f.write(_renamed(leaf, {"leaf_tree.mtl": "pine_tree.mtl", "Material.006": "Material.010",
                                "Material.007": "Material.011"}))
    lines = []
    for name in sorted(os.listdir(data)):
        with open(os.path.join(data, name), "rb") as f:
            lines.append("%s  %s" % (hashlib.sha256(f.read()).hexdigest(), name))
    with open(manifest, "w") as f:
        f.write("\n".join(lines) + "\n")
    return dest


def default_dir(repo_root: str) -> str:
    return os.path.join(repo_root, "assets")
