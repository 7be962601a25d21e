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


def test_metric_config_eight_shards_match_frame(gpu, assets_dir):
    """BASELINE configs[2]: the metric frame (frame 0, 1280x720, 1024 spp) cut
    into interleaved 32x16 tiles for 8 ranks, each shard rendered through
    ptg_render_tiles and scattered: the assembled frame equals the single-GPU
    render byte for byte, and so does the averaged radiance of every shard."""
    import torch
    s = scene_for(assets_dir, 1280, 720, 1024, frame=0)
    gpu.upload_arrays(arrays_copy(s))
    cfg = s.cfg
    full, acc_full = gpu.render(cfg, want_accum=True)
    img = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
    acc_full = acc_full.cpu().numpy()
    for r in range(8):
        sh = D.TileShard(cfg, 32, 16, r, 8)
        n = sh.count * 32 * 16
        acc_t = torch.empty((n, 4), dtype=torch.float32, device="cuda:0")
        tiles, _ = gpu.render_tiles(cfg, 32, 16, sh.first, sh.stride, sh.count, out_accum=acc_t)
        gpu.scatter_tiles(cfg, 32, 16, sh.first, sh.stride, sh.count, tiles, img)
        gpu.synchronize()
        x, y = sh.pixels()
        ok = x >= 0
        got = acc_t.cpu().numpy()[ok, :3].view(np.uint32)
        assert np.array_equal(got, acc_full[y[ok], x[ok], :3].view(np.uint32)), r
    gpu.synchronize()
    assert np.array_equal(img.cpu().numpy(), full.cpu().numpy())


def test_render_and_gather_over_rccl(gpu, assets_dir):
    """The product's render_and_gather with its collective executed over RCCL
    (torch.distributed 'nccl'): a world-size-1 process group on this GPU, so
    dist.gather runs on the device stream exactly as on 8 GPUs (RCCL cannot
    put two ranks on one GPU).  The gathered, scattered frame equals the
    single-GPU render."""
    import socket

    import torch
    import torch.distributed as dist
    s = scene_for(assets_dir, 640, 360, 32, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    cfg = s.cfg
    full, _ = gpu.render(cfg)
    gpu.synchronize()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    stream = torch.cuda.Stream()
    gpu.set_stream(stream)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        img = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
        D.render_and_gather(gpu, cfg, D.TileShard(cfg, 32, 16, 0, 1), img, stream=stream)
        stream.synchronize()
        assert np.array_equal(img.cpu().numpy(), full.cpu().numpy())
    finally:
        dist.destroy_process_group()
        gpu.set_stream(torch.cuda.default_stream())


def test_sample_shards_sum_to_frame(gpu, assets_dir):
    """The sample-range shard: the metric frame's 1024
    samples split into whole motion-blur groups for 8 ranks, each range
    rendered over every pixel and the partial radiances summed (what the
    reduce does).  Not bit-identical to the single-GPU frame - the reference
    sums a pixel's samples in index order in float32 - so it is held to the
    north star's tolerance: accumulated radiance within 1e-4 relative (plus a
    1e-7 absolute floor for near-black pixels), tonemapped bytes within 1."""
    import torch
    s = scene_for(assets_dir, 1280, 720, 1024, frame=0)
    gpu.upload_arrays(arrays_copy(s))
    cfg = s.cfg
    full, acc_full = gpu.render(cfg, want_accum=True)
    total = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.float32, device="cuda:0")
    part = torch.empty_like(total)
    for r in range(8):
        sh = D.SampleShard(cfg, r, 8)
        assert sh.j1 - sh.j0 == 128
        gpu.render(cfg, samples=(sh.j0, sh.j1), out_accum=part)
        total += part
    img = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
    gpu.tonemap_device(total, img)
    gpu.synchronize()
    a, b = total.cpu().numpy()[..., :3], acc_full.cpu().numpy()[..., :3]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
    bad = (np.abs(a - b) > 1e-4 * np.abs(b) + 1e-7).sum()
    print("sample shards vs frame: max rel %.3g, median rel %.3g, exact %.1f%%" %
          (rel.max(), np.median(rel), 100 * (a == b).mean()))
    assert bad == 0
    d = np.abs(img.cpu().numpy().astype(int) - full.cpu().numpy().astype(int))
    assert d.max() <= 1


def test_render_and_reduce_over_rccl(gpu, assets_dir):
    """The product's render_and_reduce with its sum-reduce executed over RCCL
    on a world-size-1 group: one rank owns every sample, so the reduced frame
    equals the single-GPU render bit for bit (radiance and bytes)."""
    import socket

    import torch
    import torch.distributed as dist
    s = scene_for(assets_dir, 640, 360, 32, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    cfg = s.cfg
    full, acc_full = gpu.render(cfg, want_accum=True)
    gpu.synchronize()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    stream = torch.cuda.Stream()
    gpu.set_stream(stream)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        img = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
        acc = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.float32, device="cuda:0")
        D.render_and_reduce(gpu, cfg, D.SampleShard(cfg, 0, 1), img, accum=acc, stream=stream)
        stream.synchronize()
        assert np.array_equal(acc.cpu().numpy()[..., :3].view(np.uint32), acc_full.cpu().numpy()[..., :3].view(np.uint32))
        assert np.array_equal(img.cpu().numpy(), full.cpu().numpy())
    finally:
        dist.destroy_process_group()
        gpu.set_stream(torch.cuda.default_stream())
