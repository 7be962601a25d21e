"""Multi-GPU sharding: one process per GPU, torch.distributed over RCCL.

The hot path is embarrassingly parallel (path_trace_pixel is pure,
path_tracer.hh:637; frames reset their state, scene.cc:274-277), so work is
partitioned, never exchanged, except for one real step:

* frames  - rank r renders its own frames (config 4: the animation,
            one frame per GPU).  No collective at all.
* samples - one frame's sample range split into whole motion-blur groups
            (8 samples, one subframe each) dealt to the ranks in order; each
            rank renders every pixel over its range (ptg_render's
            [sample_begin, sample_end)) and ONE sum-reduce of the float32
            radiance to rank 0 assembles the frame (SURVEY 8(e)(ii),
            `render_and_reduce`).  Not bit-identical: the reference sums the
            samples of a pixel in index order in float32 (main.cc:24-39), and
            a sum of per-range partial sums rounds differently (~1e-7
            relative; tests/test_gpu_distributed.py measures it).
* tiles   - one frame split into tile_w x tile_h tiles dealt round-robin to
            the ranks (tile t -> rank t % world; interleaving balances the
            up-to-7x per-pixel cost differences of a frame).  Each rank
            renders its tiles densely (ptg_render_tiles), then ONE gather of
            the uchar4 tiles to rank 0 over xGMI assembles the framebuffer
            (3.7 MB at 720p: each peer sends ~0.46 MB over its own link, a
            point-to-point shape - no ring all-reduce).

Per-pixel results do not depend on the partition: every pixel's samples are
summed in index order on one GPU, so a sharded frame is bit-identical to a
single-GPU render (tests/test_gpu_distributed.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class TileShard:
    """The interleaved tile set of one rank."""
    width: int
    height: int
    tile_w: int
    tile_h: int
    rank: int
    world: int

    def __init__(self, cfg, tile_w, tile_h, rank, world):
        self.width, self.height = int(cfg.width), int(cfg.height)
        self.tile_w, self.tile_h, self.rank, self.world = int(tile_w), int(tile_h), int(rank), int(world)

    @property
    def tiles_x(self):
        return math.ceil(self.width / self.tile_w)

    @property
    def tiles_y(self):
        return math.ceil(self.height / self.tile_h)

    @property
    def total(self):
        return self.tiles_x * self.tiles_y

    @property
    def first(self):
        return self.rank

    @property
    def stride(self):
        return self.world

    def count_for(self, rank):
        return max(0, (self.total - rank + self.world - 1) // self.world)

    @property
    def count(self):
        return self.count_for(self.rank)

    @property
    def max_count(self):
        return self.count_for(0)

    def pixels(self, rank=None):
        """(x, y) of every pixel slot of `rank`'s dense tile buffer (-1 outside the image)."""
        rank = self.rank if rank is None else rank
        n = self.count_for(rank)
        t = rank + np.arange(n) * self.world
        q = np.arange(self.tile_w * self.tile_h)
        tx, ty = (t % self.tiles_x)[:, None], (t // self.tiles_x)[:, None]
        x = tx * self.tile_w + q[None, :] % self.tile_w
        y = ty * self.tile_h + q[None, :] // self.tile_w
        inside = (x < self.width) & (y < self.height)
        return np.where(inside, x, -1).reshape(-1), np.where(inside, y, -1).reshape(-1)


def assemble_numpy(shard: TileShard, gathered, image):
    """CPU twin of ptg_scatter_tiles: place each rank's dense tiles into `image` ([H, W, C])."""
    for rank, buf in enumerate(gathered):
        x, y = shard.pixels(rank)
        n = len(x)
        ok = x >= 0
        image[y[ok], x[ok]] = np.asarray(buf).reshape(-1, image.shape[-1])[:n][ok]
    return image


class ShardMismatch(RuntimeError):
    """The ranks of one collective render disagree on its shape (raised on every rank)."""


_FIELDS = ("kind", "width", "height", "spp", "bounces", "student_id", "blur_step", "a", "b", "world", "rank", "group_ok")


def _agree(kind, cfg, a, b, shard_rank, shard_world, group_ok, dev, what):
    """Before any rank renders or enters the data collective, every rank of
    the default group all-gathers one small record of the call: the kind of
    shard, the config (config.hh's macros), the shard's two size parameters
    (tile size, or image size), its world size and rank, and whether it
    describes this process's place in the group.  Every rank then checks every
    record and raises ShardMismatch on any disagreement, so a rank with
    another tile size, SPP or world size makes ALL ranks fail within one
    small collective, instead of the others waiting in a gather of different
    buffer sizes until the group's timeout (status, no
    hang).  On RCCL the record is a device tensor on the current stream; the
    host reads it back (one small synchronisation per call)."""
    import torch
    import torch.distributed as dist
    mine = [kind, int(cfg.width), int(cfg.height), int(cfg.samples_per_pixel), int(cfg.max_bounces),
            int(cfg.student_id), int(cfg.samples_per_motion_blur_step), int(a), int(b), int(shard_world),
            int(shard_rank), 1 if group_ok else 0]
    on = dev if (dist.get_backend() != "gloo" and dev.type == "cuda") else torch.device("cpu")
    t = torch.tensor(mine, dtype=torch.int64, device=on)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    recs = torch.stack(parts).cpu().tolist()
    bad = [r for r, rec in enumerate(recs) if not rec[11]]
    if bad:
        raise ShardMismatch("%s: rank(s) %s hold a shard that is not their place in the process group (%s)"
                            % (what, bad, ", ".join("rank %d: shard %d of %d" % (r, recs[r][10], recs[r][9]) for r in bad)))
    keys = [tuple(rec[:10]) for rec in recs]
    if any(k != keys[0] for k in keys):
        names = list(_FIELDS)
        names[7:9] = ("tile_w", "tile_h") if kind == 1 else ("image_h", "image_w")
        diff = [i for i in range(10) if len({k[i] for k in keys}) > 1]
        raise ShardMismatch("%s: the ranks disagree on %s (%s)" % (what, ", ".join(names[i] for i in diff), "; ".join(
            "rank %d: %s" % (r, {names[i]: rec[i] for i in diff}) for r, rec in enumerate(recs))))
    return recs


def _collective_mode(shard, force_collective, what):
    """(agree, collective): whether the ranks agree on the call first
    (_agree) and whether the data collective runs.  A shard of more than one
    rank needs the default process group and does both.  A one-rank shard is
    rendered locally, unless it is the whole group of one and
    `force_collective` asks for the collective anyway; inside a larger group
    it still joins the agreement, so a rank holding a one-rank shard while
    the others hold shards of the group fails with them instead of leaving
    them waiting (every rank holding a one-rank shard - replicas - agrees and
    renders locally)."""
    import torch.distributed as dist
    grouped = dist.is_available() and dist.is_initialized()
    if shard.world == 1:
        if not grouped:
            return False, False
        if dist.get_world_size() == 1:
            return bool(force_collective), bool(force_collective)
        return True, False
    if not grouped:
        raise RuntimeError("%s: world size %d but no process group" % (what, shard.world))
    return True, True


def _place_ok(shard):
    """Whether `shard` is a legitimate place for this process: its own rank of
    the whole group, or a one-rank (replica) shard."""
    import torch.distributed as dist
    return shard.world == 1 and shard.rank == 0 or \
        (dist.get_world_size() == shard.world and dist.get_rank() == shard.rank)


def render_and_gather(renderer, cfg, shard: TileShard, image, stream=None, force_collective=True):
    """Render this rank's tiles and gather them into `image` on rank 0.

    `renderer` provides render_tiles / scatter_tiles (GpuRenderer, or any
    object with the same two methods).  Everything - the render, the gather
    and the scatter - is issued on `stream` (a torch.cuda.Stream; default:
    the current stream), which must be the stream the renderer launches on:
    RCCL then orders the collective after the tiles were written, and the
    scatter after the collective, with no host synchronisation.

    A shard of more than one rank runs the collectives of the default process
    group (and a one-rank shard at world size 1 too, with `force_collective`);
    a one-rank shard in a larger job, or with no group, is rendered locally
    (in a larger job after the agreement: replicas agree, a rank whose
    one-rank shard meets the others' group shards fails with them).
    Before anything is rendered the ranks agree on the call (_agree): if any
    rank's config, tile size or world size differs, or its shard is not its
    place in the group, EVERY rank raises ShardMismatch (no rank waits in a
    gather of other sizes).  Over gloo (CPU groups: tests, rehearsals) the
    tiles go through host memory.
    """
    import contextlib

    import torch
    import torch.distributed as dist
    dev = image.device
    per_tile = shard.tile_w * shard.tile_h
    agree, collective = _collective_mode(shard, force_collective, "render_and_gather")
    ctx = torch.cuda.stream(stream) if (stream is not None and dev.type == "cuda") else contextlib.nullcontext()
    with ctx:
        if agree:
            _agree(1, cfg, shard.tile_w, shard.tile_h, shard.rank, shard.world, _place_ok(shard), dev,
                   "render_and_gather")
        buf = torch.zeros((shard.max_count * per_tile, 4), dtype=torch.uint8, device=dev)
        if shard.count:
            renderer.render_tiles(cfg, shard.tile_w, shard.tile_h, shard.first, shard.stride, shard.count,
                                  out_bgra=buf[:shard.count * per_tile])
        if not collective:
            parts = [buf]
        elif dist.get_backend() == "gloo":   # CPU process groups: gather through host memory
            host = buf.cpu()
            hparts = [torch.empty_like(host) for _ in range(shard.world)] if shard.rank == 0 else None
            dist.gather(host, hparts, dst=0)
            parts = [p.to(dev) for p in hparts] if shard.rank == 0 else None
        else:                                # RCCL over xGMI: one gather of the uchar4 tiles to rank 0
            parts = [torch.empty_like(buf) for _ in range(shard.world)] if shard.rank == 0 else None
            dist.gather(buf, parts, dst=0)
        if shard.rank == 0:
            for r, part in enumerate(parts):
                n = shard.count_for(r)
                if n:
                    renderer.scatter_tiles(cfg, shard.tile_w, shard.tile_h, r, shard.world, n, part, image)
    return image


@dataclass
class SampleShard:
    """The sample range [j0, j1) of one rank: whole groups of `group` samples
    (SAMPLES_PER_MOTION_BLUR_STEP, one subframe each), consecutive groups per
    rank, as even as the group count allows."""
    spp: int
    rank: int
    world: int
    group: int

    def __init__(self, cfg, rank, world, group=None):
        self.spp = int(cfg.samples_per_pixel)
        self.rank, self.world = int(rank), int(world)
        self.group = int(group or getattr(cfg, "samples_per_motion_blur_step", 8) or 8)

    def range_for(self, rank):
        groups = -(-self.spp // self.group)
        g0, g1 = rank * groups // self.world, (rank + 1) * groups // self.world
        return min(self.spp, g0 * self.group), min(self.spp, g1 * self.group)

    @property
    def j0(self):
        return self.range_for(self.rank)[0]

    @property
    def j1(self):
        return self.range_for(self.rank)[1]


def render_and_reduce(renderer, cfg, shard: SampleShard, image, accum=None, stream=None, force_collective=True):
    """Render this rank's sample range of every pixel and sum-reduce the
    radiance to rank 0, which tonemaps it into `image` (and copies the reduced
    radiance into `accum` if given).  Each rank's partial is its range's
    j-ordered float32 sum / SPP (ptg_render over [j0, j1)); rank 0 gets the
    sum of the partials, so the frame is within float32 rounding of the
    single-GPU render, not bit-identical to it (module docstring).

    Like render_and_gather: everything is issued on `stream`, which must be
    the stream the renderer launches on (GpuRenderer.set_stream(stream)), so
    that RCCL orders the reduce after the partial was written and
    tonemap_device after the reduce; the ranks agree on the call first
    (config, image size, world size and place in the group: any disagreement
    raises ShardMismatch on every rank before anything is rendered).  RCCL reduces the device tensors over xGMI; gloo
    (CPU groups: tests, rehearsals) reduces through host memory."""
    import contextlib

    import torch
    import torch.distributed as dist
    dev = image.device
    agree, collective = _collective_mode(shard, force_collective, "render_and_reduce")
    ctx = torch.cuda.stream(stream) if (stream is not None and dev.type == "cuda") else contextlib.nullcontext()
    with ctx:
        h, w = image.shape[0], image.shape[1]
        if agree:
            _agree(2, cfg, h, w, shard.rank, shard.world, _place_ok(shard), dev, "render_and_reduce")
        part = torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
        if shard.j1 > shard.j0:
            renderer.render(cfg, samples=(shard.j0, shard.j1), out_accum=part)
        if collective:
            if dist.get_backend() == "gloo":   # CPU process groups: reduce through host memory
                host = part.cpu()
                dist.reduce(host, dst=0, op=dist.ReduceOp.SUM)
                if shard.rank == 0:
                    part.copy_(host)
            else:                              # RCCL over xGMI: one sum-reduce of the radiance to rank 0
                dist.reduce(part, dst=0, op=dist.ReduceOp.SUM)
        if shard.rank == 0:
            renderer.tonemap_device(part, image)
            if accum is not None:
                accum.copy_(part)
    return image


def frames_for_rank(frame_count, rank, world):
    """Frame-parallel animation (config 4): rank r renders frames r, r + world, ..."""
    return list(range(rank, frame_count, world))
