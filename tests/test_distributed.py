"""Multi-GPU sharding logic on CPU: tile partition, frame partition, and the
product's render_and_gather (distributed.py) over real world-size 2 and 3
process groups (gloo) with a stub renderer in place of the GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import N
from ptlumi import distributed as D


@pytest.mark.parametrize("w,h,tw,th,world", [(1280, 720, 32, 16, 8), (640, 360, 48, 40, 3), (160, 90, 64, 64, 2),
                                             (37, 11, 8, 8, 5)])
def test_tiles_cover_every_pixel_once(w, h, tw, th, world):
    cfg = N.RenderConfig.make(w, h, 8)
    seen = np.zeros((h, w), np.int32)
    counts = []
    for r in range(world):
        s = D.TileShard(cfg, tw, th, r, world)
        x, y = s.pixels()
        ok = x >= 0
        np.add.at(seen, (y[ok], x[ok]), 1)
        counts.append(s.count)
        assert len(x) == s.count * tw * th
    assert (seen == 1).all()
    assert max(counts) - min(counts) <= 1          # round-robin deal


def test_frames_partition():
    parts = [D.frames_for_rank(1800, r, 8) for r in range(8)]
    assert sorted(sum(parts, [])) == list(range(1800))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class StubRenderer:
    """Stands in for GpuRenderer on CPU: render_tiles writes each pixel slot's
    own coordinates (and the rank), scatter_tiles places a dense tile buffer
    into the image exactly as ptg_scatter_tiles does (through TileShard.pixels)."""

    def __init__(self, rank):
        self.rank = rank
        self.calls = []

    def render_tiles(self, cfg, tw, th, first, stride, count, out_bgra=None):
        self.calls.append(("render_tiles", first, stride, count))
        sh = D.TileShard(cfg, tw, th, first, stride)
        x, y = sh.pixels()
        n = count * tw * th
        buf = out_bgra.view(-1, 4)
        assert buf.shape[0] == n == len(x)
        buf[:, 0] = torch.from_numpy(np.where(x >= 0, x % 251, 0).astype(np.uint8))
        buf[:, 1] = torch.from_numpy(np.where(y >= 0, y % 241, 0).astype(np.uint8))
        buf[:, 2] = self.rank
        buf[:, 3] = 255
        return out_bgra, None

    def scatter_tiles(self, cfg, tw, th, first, stride, count, tiles_bgra, image_bgra):
        self.calls.append(("scatter_tiles", first, stride, count))
        sh = D.TileShard(cfg, tw, th, first, stride)
        x, y = sh.pixels()
        ok = x >= 0
        t = tiles_bgra.view(-1, 4)[:len(x)].numpy()
        img = image_bgra.numpy()
        img[y[ok], x[ok]] = t[ok]


def _worker(rank, world, port, w, h, tw, th, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = N.RenderConfig.make(w, h, 8)
    shard = D.TileShard(cfg, tw, th, rank, world)
    image = torch.zeros((h, w, 4), dtype=torch.uint8)
    stub = StubRenderer(rank)
    D.render_and_gather(stub, cfg, shard, image)          # the product function, collective included
    if rank == 0:
        np.save(out, image.numpy())
        # rank 0 rendered its own tiles and scattered every rank's part
        assert stub.calls[0] == ("render_tiles", 0, world, shard.count)
        assert [c[1] for c in stub.calls[1:]] == list(range(world))
    else:
        assert stub.calls == [("render_tiles", rank, world, shard.count)]
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_framebuffer_gloo(tmp_path, world):
    w, h, tw, th = 100, 60, 16, 8
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), w, h, tw, th, out), nprocs=world, join=True)
    img = np.load(out)
    yy, xx = np.mgrid[0:h, 0:w]
    assert np.array_equal(img[..., 0], xx % 251) and np.array_equal(img[..., 1], yy % 241)
    tiles_x = (w + tw - 1) // tw
    owner = ((yy // th) * tiles_x + xx // tw) % world
    assert np.array_equal(img[..., 2], owner)
    assert (img[..., 3] == 255).all()


def test_render_and_gather_without_group_is_local():
    cfg = N.RenderConfig.make(40, 20, 8)
    shard = D.TileShard(cfg, 16, 8, 0, 1)
    image = torch.zeros((20, 40, 4), dtype=torch.uint8)
    D.render_and_gather(StubRenderer(0), cfg, shard, image)
    yy, xx = np.mgrid[0:20, 0:40]
    assert np.array_equal(image[..., 0].numpy(), xx % 251) and np.array_equal(image[..., 1].numpy(), yy % 241)
    with pytest.raises(RuntimeError, match="no process group"):
        D.render_and_gather(StubRenderer(0), cfg, D.TileShard(cfg, 16, 8, 0, 2), image)


def _mismatch_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = N.RenderConfig.make(40, 20, 8)
    image = torch.zeros((20, 40, 4), dtype=torch.uint8)
    # a one-rank shard inside a 2-rank job: rendered locally by each rank, no collective
    D.render_and_gather(StubRenderer(rank), cfg, D.TileShard(cfg, 16, 8, 0, 1), image)
    yy, xx = np.mgrid[0:20, 0:40]
    ok = np.array_equal(image[..., 0].numpy(), xx % 251) and (image[..., 2].numpy() == rank).all()
    # a shard that is not this process's place in the group: refused up front on every rank
    try:
        D.render_and_gather(StubRenderer(rank), cfg, D.TileShard(cfg, 16, 8, rank, world + 1), image)
        refused = False
    except RuntimeError as e:
        refused = isinstance(e, D.ShardMismatch) and "not their place in the process group" in str(e)
    np.save(out % rank, np.array([ok, refused]))
    dist.barrier()
    dist.destroy_process_group()


def test_render_and_gather_shard_group_mismatch(tmp_path):
    """distributed.py render_and_gather: a local one-rank shard in a larger job
    takes the local path (no collective for the other ranks to miss), and a
    shard that does not describe the process group raises on every rank
    before anything is rendered."""
    out = str(tmp_path / "r%d.npy")
    mp.spawn(_mismatch_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert np.load(out % r).tolist() == [True, True]


# ---- sample-range shard ------------------------------------

@pytest.mark.parametrize("spp,world", [(1024, 8), (1024, 3), (8, 2), (40, 3), (12, 2)])
def test_sample_ranges_partition_whole_groups(spp, world):
    """Every sample index lands on exactly one rank, in consecutive ranges of
    whole motion-blur groups (8 samples, one subframe each)."""
    cfg = N.RenderConfig.make(64, 32, spp)
    seen = []
    for r in range(world):
        s = D.SampleShard(cfg, r, world)
        assert s.j0 <= s.j1 and (s.j0 % 8 == 0) and (s.j1 % 8 == 0 or s.j1 == spp)
        seen.extend(range(s.j0, s.j1))
    assert seen == list(range(spp))


class StubSampleRenderer:
    """Stands in for GpuRenderer on CPU: render over a sample range writes the
    range's sum of f(x, y, j) / SPP (float32), tonemap_device a byte function
    of the radiance."""

    def __init__(self):
        self.calls = []

    @staticmethod
    def f(x, y, j):
        return np.float32(1e-3) * np.float32((x * 7 + y * 13 + j * 3) % 97)

    def render(self, cfg, samples=None, out_accum=None, **_):
        j0, j1 = samples
        self.calls.append(("render", j0, j1))
        h, w = out_accum.shape[:2]
        yy, xx = np.mgrid[0:h, 0:w]
        acc = np.zeros((h, w), np.float32)
        for j in range(j0, j1):
            acc += self.f(xx, yy, j)
        acc /= np.float32(cfg.samples_per_pixel)
        out_accum[..., 0] = torch.from_numpy(acc)
        out_accum[..., 1] = torch.from_numpy(acc * 2)
        out_accum[..., 2] = torch.from_numpy(acc * 3)
        return None, out_accum

    def tonemap_device(self, colors, out_bgra):
        self.calls.append(("tonemap",))
        out_bgra[..., 0] = (colors[..., 0] * 1000).to(torch.uint8)
        out_bgra[..., 3] = 255
        return out_bgra


def _reduce_worker(rank, world, port, spp, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = N.RenderConfig.make(30, 20, spp)
    shard = D.SampleShard(cfg, rank, world)
    image = torch.zeros((20, 30, 4), dtype=torch.uint8)
    accum = torch.zeros((20, 30, 4), dtype=torch.float32)
    stub = StubSampleRenderer()
    D.render_and_reduce(stub, cfg, shard, image, accum=accum)   # the product function, collective included
    if rank == 0:
        np.save(out, accum.numpy())
        assert stub.calls == [("render", shard.j0, shard.j1), ("tonemap",)]
        assert (image[..., 3] == 255).all()
    else:
        assert stub.calls == [("render", shard.j0, shard.j1)]
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_reduce_assembles_radiance_gloo(tmp_path, world):
    """render_and_reduce over a real gloo group: rank 0 holds the sum of every
    rank's range, which equals the whole-range sum within float32 rounding."""
    spp = 48
    out = str(tmp_path / "acc.npy")
    mp.spawn(_reduce_worker, args=(world, _free_port(), spp, out), nprocs=world, join=True)
    acc = np.load(out)
    yy, xx = np.mgrid[0:20, 0:30]
    want = np.zeros((20, 30), np.float64)
    for j in range(spp):
        want += StubSampleRenderer.f(xx, yy, j).astype(np.float64)
    want /= spp
    assert np.allclose(acc[..., 0], want, rtol=1e-5, atol=1e-7)
    assert np.allclose(acc[..., 2], 3 * want, rtol=1e-5, atol=1e-7)


# ---- ranks that disagree on the call fail together ------

def _disagree_worker(rank, world, port, case, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time
    t0 = time.monotonic()
    msg, rendered = "", False
    try:
        if case == "tile":        # only rank 1 cuts other tiles
            cfg = N.RenderConfig.make(40, 20, 8)
            stub = StubRenderer(rank)
            D.render_and_gather(stub, cfg, D.TileShard(cfg, 16 if rank == 0 else 8, 8, rank, world),
                                torch.zeros((20, 40, 4), dtype=torch.uint8))
            rendered = bool(stub.calls)
        elif case == "spp":       # only rank 1 renders another SPP
            cfg = N.RenderConfig.make(30, 20, 48 if rank == 0 else 56)
            stub = StubSampleRenderer()
            D.render_and_reduce(stub, cfg, D.SampleShard(cfg, rank, world), torch.zeros((20, 30, 4), dtype=torch.uint8))
            rendered = bool(stub.calls)
        elif case == "world":     # only rank 1's shard is not its place in the group
            cfg = N.RenderConfig.make(40, 20, 8)
            stub = StubRenderer(rank)
            D.render_and_gather(stub, cfg, D.TileShard(cfg, 16, 8, rank, world if rank == 0 else world + 1),
                                torch.zeros((20, 40, 4), dtype=torch.uint8))
            rendered = bool(stub.calls)
        elif case == "world1":    # only rank 1 holds a one-rank shard (it used to skip the agreement)
            cfg = N.RenderConfig.make(40, 20, 8)
            stub = StubRenderer(rank)
            D.render_and_gather(stub, cfg, D.TileShard(cfg, 16, 8, rank, world) if rank == 0 else
                                D.TileShard(cfg, 16, 8, 0, 1), torch.zeros((20, 40, 4), dtype=torch.uint8))
            rendered = bool(stub.calls)
        elif case == "replicas":  # every rank holds a one-rank shard: they agree and render locally
            cfg = N.RenderConfig.make(40, 20, 8)
            stub = StubRenderer(rank)
            D.render_and_gather(stub, cfg, D.TileShard(cfg, 16, 8, 0, 1), torch.zeros((20, 40, 4), dtype=torch.uint8))
            rendered = bool(stub.calls)
    except D.ShardMismatch as e:
        msg = str(e)
    np.save(out % rank, np.array([msg, str(rendered), str(time.monotonic() - t0)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,field", [("tile", "disagree on tile_w"), ("spp", "disagree on spp"), ("world", "not their place"),
                                        ("world1", "disagree on world")])
def test_disagreeing_rank_fails_every_rank(tmp_path, case, field):
    """render_and_gather / render_and_reduce: when ONE rank's call differs
    (tile size, SPP, or a shard that is not its place in the group), every
    rank raises ShardMismatch within seconds and nothing is rendered - the
    others do not wait in a gather or reduce of other buffer sizes."""
    out = str(tmp_path / "r%d.npy")
    mp.spawn(_disagree_worker, args=(2, _free_port(), case, out), nprocs=2, join=True)
    for r in range(2):
        msg, rendered, secs = np.load(out % r).tolist()
        assert field in msg, (r, msg)
        assert rendered == "False"
        assert float(secs) < 30


def test_one_rank_shards_in_a_group_render_locally(tmp_path):
    """Replicas: every rank of a 2-rank group holds a one-rank shard; the
    agreement passes and each rank renders its whole frame locally."""
    out = str(tmp_path / "r%d.npy")
    mp.spawn(_disagree_worker, args=(2, _free_port(), "replicas", out), nprocs=2, join=True)
    for r in range(2):
        msg, rendered, secs = np.load(out % r).tolist()
        assert msg == "" and rendered == "True", (r, msg)
