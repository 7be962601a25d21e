"""Tile sharding on the GPU: every rank's tile set, rendered densely through
ptg_render_tiles and assembled (ptg_scatter_tiles / assemble_numpy), must be
bit-identical to the single-GPU frame - the partition never changes a pixel.

The ranks are simulated one after the other on the one GPU of the test box;
the real collective (dist.gather over RCCL) is the same code path that
tests/test_distributed.py runs over gloo, and bench.py --shard tiles on N>1.
"""
import numpy as np
import pytest

from conftest import arrays_copy, scene_for
from ptlumi import distributed as D

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tw,th,world", [(32, 16, 8), (48, 40, 3), (64, 64, 5)])
def test_tiles_assemble_to_single_gpu_frame(gpu, assets_dir, tw, th, world):
    import torch
    s = scene_for(assets_dir, 640, 360, 32, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    cfg = s.cfg
    full, _ = gpu.render(cfg)
    dev_img = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
    parts = []
    for r in range(world):
        sh = D.TileShard(cfg, tw, th, r, world)
        if sh.count == 0:
            parts.append(np.zeros((0, 4), np.uint8))
            continue
        tiles, _ = gpu.render_tiles(cfg, tw, th, sh.first, sh.stride, sh.count)
        gpu.scatter_tiles(cfg, tw, th, sh.first, sh.stride, sh.count, tiles, dev_img)
        parts.append(tiles.cpu().numpy())
    gpu.synchronize()
    full = full.cpu().numpy()
    assert np.array_equal(dev_img.cpu().numpy(), full)
    host_img = np.zeros_like(full)
    pad = D.TileShard(cfg, tw, th, 0, world).max_count * tw * th
    parts = [np.concatenate([p, np.zeros((pad - len(p), 4), np.uint8)]) for p in parts]
    D.assemble_numpy(D.TileShard(cfg, tw, th, 0, world), parts, host_img)
    assert np.array_equal(host_img, full)
