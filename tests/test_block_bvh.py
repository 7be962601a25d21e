"""Block BVH records (csrc/device/block_format.h) on the CPU.

tools/walk_sim runs the host half of ptg_upload_frame (BlockCache::pack_frame,
host/block_bvh.cpp) on the real scene - a first frame committed, then the
frame under test, so BLAS blocks are also packed at a nonzero block base -
and walks a path-tracing query mix (camera rays, random bounces, sun shadow
rays) twice: with the reference's stackless link walk (ray_query.hh:184-278)
and with the device's block-walk algorithm over those blocks.  Every query
must return the same hit bits (thit, barycentrics, instance, primitive,
back face / occlusion).  The GPU kernels run the same algorithm and are
checked bit for bit against the oracle by the -m gpu tests.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

TOOL = os.path.join(ROOT, "tools", "_bin", "walk_sim")


@pytest.fixture(scope="module")
def walk_sim(native_lib):
    subprocess.run(["make", "-s", "walk_sim"], cwd=os.path.join(ROOT, "tools"), check=True)
    return TOOL


@pytest.mark.parametrize("frame", [0, 450, 1400])
def test_block_walk_matches_link_walk(walk_sim, assets_dir, frame):
    r = subprocess.run([walk_sim, assets_dir, str(frame), "3000", "16"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"(\d+) queries, (\d+) mismatches", r.stdout)
    assert m and int(m.group(1)) > 5000 and int(m.group(2)) == 0, r.stdout
    # the any-hit candidates' requirement (a candidate's leaf box is tested from its vertices)
    lb = re.search(r"instances whose BLAS leaf boxes are not their vertex bounds: (\d+) of (\d+)", r.stdout)
    assert lb and int(lb.group(1)) == 0 and int(lb.group(2)) > 100, r.stdout
    assert "leaf-box check rejects a perturbed box: yes" in r.stdout, r.stdout
    # the block walk takes about half the dependent steps of the link walk
    steps = [float(x) for x in re.findall(r"steps ([0-9.]+)", r.stdout)]
    link_closest, block_closest = steps[0], steps[1]
    assert block_closest < 0.6 * link_closest, r.stdout
    # the subframes' TLASes share their identical subtrees (pack_frame's
    # deduplication): ~50 MB of per-subframe blocks become 1-2 MB
    t = re.search(r"TLAS (\d+) copies \(([0-9.]+) MB\)", r.stdout)
    assert t and float(t.group(2)) < 5.0, r.stdout


def test_lockstep_schedule_model_exact(walk_sim, assets_dir):
    """The model of the kernel's lockstep schedule (tools/walk_sim LOCKSTEP,
    DESIGN.md section 4.2) walks every query to the reference's result and
    reports the lanes each load serves."""
    env = dict(os.environ, LOCKSTEP="2 1 1 24")
    r = subprocess.run([walk_sim, assets_dir, "450", "1500", "16"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert len(re.findall(r"; 0 mismatches vs the link walk", r.stdout)) == 2, r.stdout
    lanes = [float(x) for x in re.findall(r"lanes/instr node ([0-9.]+)", r.stdout)]
    assert len(lanes) == 2 and all(20 < x < 64 for x in lanes), r.stdout


def test_eight_wide_blocks_exact(native_lib, assets_dir):
    """8-wide blocks (measured slower on the GPU) meet
    every leaf in the reference's order too: the packer and the walk are
    generic in the block width."""
    subprocess.run(["make", "-s", "walk_sim8"], cwd=os.path.join(ROOT, "tools"), check=True)
    r = subprocess.run([os.path.join(ROOT, "tools", "_bin", "walk_sim8"), assets_dir, "450", "1500", "16"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"(\d+) queries, (\d+) mismatches", r.stdout)
    assert m and int(m.group(2)) == 0, r.stdout


def test_zero_and_nan_direction_components(walk_sim, assets_dir):
    """A ray with a zero direction component (1/dir infinite) takes the
    walk's min/max form of the slab test (BlockWalker::node_block).  Bounces
    with one or two zero components, the sun's exact direction (which has one
    in this scene) and NaN directions return the reference's hits, with about
    as many steps as the other rays."""
    env = dict(os.environ, AXIS="1")
    r = subprocess.run([walk_sim, assets_dir, "450", "3000", "16"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    z = re.search(r"queries with a zero direction component: (\d+) of (\d+)", r.stdout)
    assert z and int(z.group(1)) > int(z.group(2)) // 10, r.stdout
    m = re.search(r"(\d+) queries, (\d+) mismatches", r.stdout)
    assert m and int(m.group(2)) == 0, r.stdout
    steps = [float(x) for x in re.findall(r"steps ([0-9.]+)", r.stdout)]
    assert steps[3] < 0.7 * steps[2], r.stdout   # shadow rays: block walk vs link walk
    # NaN directions (one, two or three components) are in the mix too: a ray
    # with three NaN components passes no box, one with one or two is tested
    # on its other axes as in the reference (which enters more BLASes for
    # them), so no query walks the whole scene (580k nodes)
    mx = re.search(r"most block-walk steps of one query: (\d+)", r.stdout)
    assert mx and int(mx.group(1)) < 10000, r.stdout
