"""The wavefront runtime's orderings and knobs on the GPU:

  * asynchronous frame uploads queued behind renders with no host
    synchronisation in between (staging-buffer reuse and device
    buffers that must grow for a new BLAS), bit-identical to synchronised
    renders of the same frames;
  * ptg_set_hbm_share: smaller path-state chunks, identical bits;
  * ptg_set_chunk_paths: larger or smaller sample chunks, identical bits;
  * the counting build's walk statistics (ptg_last_walk_stats) against the
    work counters of the same render;
  * two processes on one GPU, each a real GpuRenderer, rendering their tile
    sets of one frame and gathering them through the product's
    render_and_gather over a gloo group: the assembled
    frame equals the single-process render.
"""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, N, arrays_copy, scene_for

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_async_uploads_between_renders_match_synchronised(gpu, assets_dir):
    """render A, upload B, render B, upload C, render C with no synchronisation:
    B's upload is queued behind A's render, C's reuses A's pinned staging
    buffer (the two alternate), and B (the dragon, frame 690) and C (the end
    card, frame 1799) each bring a BLAS no earlier frame named, so the block
    buffer grows while renders are queued.  Each frame must equal a render
    of it by a fresh context with a synchronisation after every call."""
    import torch
    from ptlumi.renderer import GpuRenderer
    cfg = N.RenderConfig.make(320, 180, 16)
    frames = [0, 690, 1799]
    s = N.Scene(assets_dir, cfg)
    dev = torch.device("cuda", 0)
    outs = []
    r = GpuRenderer(0)
    try:
        for k, f in enumerate(frames):
            s.setup_frame(f)
            r.upload(s, include_static=(k == 0))
            acc = torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device=dev)
            bgra, _ = r.render(cfg, out_accum=acc)
            outs.append((acc, bgra))
        r.synchronize()
        got = [(a.cpu().numpy(), b.cpu().numpy()) for a, b in outs]
    finally:
        r.close()
    for k, f in enumerate(frames):
        q = GpuRenderer(0)
        try:
            s.setup_frame(f)
            q.upload(s, include_static=True)
            q.synchronize()
            bgra, acc = q.render(cfg, want_accum=True)
            q.synchronize()
            assert np.array_equal(_bits(got[k][0][..., :3]), _bits(acc.cpu().numpy()[..., :3])), f
            assert np.array_equal(got[k][1], bgra.cpu().numpy()), f
        finally:
            q.close()
    s.close()


def test_hbm_share_changes_chunks_not_bits(assets_dir):
    """ptg_set_hbm_share(5): the 1280x720 x 256 spp frame (236 M paths) runs
    in ~4x as many sample chunks as at the default share; same bits."""
    from ptlumi.renderer import GpuRenderer
    s = scene_for(assets_dir, 1280, 720, 256, frame=0)
    arr = arrays_copy(s)
    out = []
    for share in (35, 5):
        r = GpuRenderer(0)
        try:
            r.set_hbm_share(share)
            r.upload_arrays(arr)
            r.enable_timing(True)
            _, acc = r.render(s.cfg, want_accum=True)
            r.synchronize()
            launches = r.kernel_times()["camera"][1]      # one camera launch per chunk
            out.append((_bits(acc.cpu().numpy()[..., :3]), launches))
        finally:
            r.close()
    assert out[1][1] > out[0][1], "a smaller share must cut the frame into more chunks: %s" % [o[1] for o in out]
    assert np.array_equal(out[0][0], out[1][0])
    with pytest.raises(N.PtgError, match=r"\(-1\)"):
        GpuRenderer(0).set_hbm_share(2)


def test_chunk_paths_change_chunks_not_bits(assets_dir):
    """ptg_set_chunk_paths: the 1280x720 x 256 spp frame (236 M paths) in
    chunks of at most 2^28 paths with a 40% share (what a renderer that owns
    the GPU takes, bench.py's default) and of at most 2^24 paths: more
    chunks for the smaller size, the same bits."""
    from ptlumi.renderer import GpuRenderer
    s = scene_for(assets_dir, 1280, 720, 256, frame=0)
    arr = arrays_copy(s)
    out = []
    for log2, share in ((28, 40), (24, 35)):
        r = GpuRenderer(0)
        try:
            r.set_hbm_share(share)
            r.set_chunk_paths(log2)
            r.upload_arrays(arr)
            r.enable_timing(True)
            _, acc = r.render(s.cfg, want_accum=True)
            r.synchronize()
            launches = r.kernel_times()["camera"][1]      # one camera launch per chunk
            out.append((_bits(acc.cpu().numpy()[..., :3]), launches))
        finally:
            r.close()
    assert out[1][1] > out[0][1], "smaller chunks must mean more of them: %s" % [o[1] for o in out]
    assert np.array_equal(out[0][0], out[1][0])
    with pytest.raises(N.PtgError, match=r"\(-1\)"):
        GpuRenderer(0).set_chunk_paths(29)


def test_walk_stats_consistent_with_counters(gpu, assets_dir):
    s = scene_for(assets_dir, 640, 360, 32, frame=450)
    gpu.upload_arrays(arrays_copy(s))
    gpu.enable_counters(True)
    try:
        gpu.render(s.cfg)
        gpu.synchronize()
        kc = gpu.kernel_counters()
        ws = gpu.walk_stats()
    finally:
        gpu.enable_counters(False)
    for kind in ("extend", "shadow"):
        w = ws[kind]
        queries = int(kc[kind][4])
        assert w["refill_lanes"] == queries > 0, (kind, w, queries)   # every ray is started once
        for ph, ln in (("node_phases", "node_lanes"), ("leaf_phases", "leaf_lanes"), ("refills", "refill_lanes"),
                       ("iterations", "active_lanes")):
            assert 0 < w[ph] <= w[ln] <= 64 * w[ph], (kind, ph, w)
        # a node phase loads a block for each lane that steps one: at least one
        # block per BLAS entry and per query that reaches a block
        assert w["node_lanes"] >= int(kc[kind][3]), (kind, w)
    print({k: {"node lanes/instr": round(v["node_lanes"] / v["node_phases"], 1),
               "leaf lanes/instr": round(v["leaf_lanes"] / v["leaf_phases"], 1),
               "active lanes/iter": round(v["active_lanes"] / v["iterations"], 1)} for k, v in ws.items()})


def _tile_rank(rank, world, port, out, w, h, spp, frame):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import ptlumi_loader  # noqa: F401
    from ptlumi import native as Nn
    from ptlumi import distributed as D
    from ptlumi.renderer import GpuRenderer
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = Nn.RenderConfig.make(w, h, spp)
        s = Nn.Scene(os.path.join(ROOT, "assets"), cfg)
        s.setup_frame(frame)
        r = GpuRenderer(0)
        stream = torch.cuda.Stream(0)
        r.set_stream(stream)
        r.upload(s)
        image = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda:0")
        D.render_and_gather(r, cfg, D.TileShard(cfg, 32, 16, rank, world), image, stream=stream)
        stream.synchronize()
        if rank == 0:
            np.save(out, image.cpu().numpy())
        r.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_processes_render_and_gather_on_gpu(gpu, assets_dir):
    import torch.multiprocessing as mp
    w, h, spp, frame = 1280, 720, 32, 0
    s = scene_for(assets_dir, w, h, spp, frame=frame)
    gpu.upload_arrays(arrays_copy(s))
    full, _ = gpu.render(s.cfg)
    gpu.synchronize()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "img.npy")
        mp.start_processes(_tile_rank, args=(2, port, out, w, h, spp, frame), nprocs=2, join=True,
                           start_method="spawn")
        img = np.load(out)
    assert np.array_equal(img, full.cpu().numpy())
