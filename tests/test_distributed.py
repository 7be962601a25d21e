"""Multi-GPU sharding logic on CPU: tile partition, frame partition and the
framebuffer gather over a real world_size-2 process group (gloo)."""
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


def _worker(rank, world, port, w, h, tw, th, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = N.RenderConfig.make(w, h, 8)
    shard = D.TileShard(cfg, tw, th, rank, world)
    x, y = shard.pixels()
    # stand-in for ptg_render_tiles: each pixel slot holds its own coordinates
    buf = np.zeros((shard.max_count * tw * th, 4), np.uint8)
    n = len(x)
    buf[:n, 0] = np.where(x >= 0, x % 251, 0)
    buf[:n, 1] = np.where(y >= 0, y % 241, 0)
    buf[:n, 2] = rank
    buf[:n, 3] = 255
    t = torch.from_numpy(buf)
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0)
    if rank == 0:
        img = np.zeros((h, w, 4), np.uint8)
        D.assemble_numpy(shard, [p.numpy() for p in parts], img)
        np.save(out, img)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_assembles_framebuffer_gloo(tmp_path):
    w, h, tw, th, world = 100, 60, 16, 8, 2
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), w, h, tw, th, out), nprocs=world, join=True)
    img = np.load(out)
    yy, xx = np.mgrid[0:h, 0:w]
    assert np.array_equal(img[..., 0], xx % 251) and np.array_equal(img[..., 1], yy % 241)
    tiles_x = (w + tw - 1) // tw
    owner = ((yy // th) * tiles_x + xx // tw) % world
    assert np.array_equal(img[..., 2], owner)
    assert (img[..., 3] == 255).all()
