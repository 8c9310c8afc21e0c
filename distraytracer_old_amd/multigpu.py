"""Image partition across GPUs and the single exchange step.

Rank r of N renders row bands r, r+N, r+2N, ... of BAND rows each (interleaved
bands balance the expensive bunny/glass regions; bands keep a wave's 2-row pixel
tiles on adjacent image rows, which single-row interleaving at large N would not).
Every rank's tile is padded to the same row count (a multiple of the band) so one
`gather` (RCCL point-to-point over xGMI; gloo in CPU tests) brings all float-RGB
tiles to rank 0, and `assemble` re-interleaves them.

Cost-balanced tiles (the default of bench.py's N-GPU step): the frame's wave tiles are dealt
to ranks from their measured wave times (`balanced_tiles`: rank 0 calibrates the whole frame,
rt_tile_costs, and broadcasts the costs, so every rank derives the same partition); each rank
renders its tile list into a whole-frame device buffer (rt_render_tiles_device), packs its pixels
into a compact tile buffer (`tile_pixels` order) for the gather, and rank 0 scatters them back.

Pixels, their RNG keys and their per-pixel sample order do not depend on N,
so the assembled image is bit-identical to the 1-GPU image.
"""
from __future__ import annotations

BAND = 8  # rows per band (a multiple of every wave-tile height)


def rows_of(rank: int, world: int, H: int, band: int = BAND) -> tuple[int, int, int, int]:
    """(row0, row1, row_step, row_band) of a rank's tile (rt_render_params)."""
    return rank * band, H, world, band


def image_rows(rank: int, world: int, H: int, band: int = BAND) -> list[int]:
    """Image rows of a rank's tile, in tile order."""
    return [r for r in range(H) if (r // band) % world == rank]


def tile_rows(rank: int, world: int, H: int, band: int = BAND) -> int:
    return len(image_rows(rank, world, H, band))


def max_tile_rows(world: int, H: int, band: int = BAND) -> int:
    """Padded per-rank tile height: whole bands, the same for every rank."""
    return -(-H // (world * band)) * band


def cost_bucket(costs):
    """Quarter-octave cost buckets (the dispatch sort key, rt_internal.h cost_bucket): 0 for 0, else
    1 + floor(4 log2 c) by exact compares of c / 2^floor(log2 c) against 2^(1/4), 2^(1/2), 2^(3/4)."""
    import numpy as np

    c = np.asarray(costs, dtype=np.float64)
    oct_ = np.floor(np.log2(np.maximum(c, 1.0)))
    # the octave from the float log2 can be off by one at exact powers of two: fix it exactly
    oct_ = np.where(np.exp2(oct_) > c, oct_ - 1, oct_)
    oct_ = np.where(np.exp2(oct_ + 1) <= c, oct_ + 1, oct_)
    f = c / np.exp2(oct_)
    k = 1 + 4 * oct_ + (f >= 1.6817928305074290) + (f >= 1.4142135623730951) + (f >= 1.1892071150027210)
    return np.where(c > 0, k, 0.0)


def contiguous_tiles(costs, world: int, weights=None) -> list:
    """Cut the tiles in row-major order into `world` contiguous runs of (nearly) equal measured
    cost (prefix sums; rank r takes the tiles whose cumulative cost midpoint lies in
    [r T / N, (r + 1) T / N)): every rank renders a compact region of the image, so the waves
    running together share BVH and texture cache lines. Each rank's list is in dispatch order
    (longest first by quarter-octave bucket, row-major inside a bucket). Deterministic."""
    import numpy as np

    c = np.asarray(costs, dtype=np.float64)
    cw = c if weights is None else c * np.asarray(weights, dtype=np.float64)  # the cut's costs
    cum = np.cumsum(cw)
    total = cum[-1] if len(cum) else 0.0
    mid = cum - 0.5 * cw
    owner = np.minimum((mid * world / max(total, 1e-300)).astype(np.int64), world - 1) if total > 0 else \
        (np.arange(len(c)) * world // max(1, len(c)))
    bucket = cost_bucket(c)
    idx = np.arange(len(c), dtype=np.int64)
    out = []
    for r in range(world):
        t = idx[owner == r]
        t = t[np.lexsort((t, -bucket[t]))]
        out.append(t.astype(np.int32))
    return out


def balanced_tiles(costs, world: int) -> list:
    """Deal the tiles of a layout to `world` ranks by their measured costs: tiles sorted by cost
    (descending, ties by index) are dealt serpentine (0..N-1, N-1..0, ...), so the ranks' cost sums
    differ by less than one tile's cost. Each rank's list is in dispatch order: longest first by
    quarter-octave bucket, row-major inside a bucket (waves running together stay close in the
    image). Deterministic: equal costs give equal partitions on every rank."""
    import numpy as np

    c = np.asarray(costs, dtype=np.int64)
    n = len(c)
    idx = np.arange(n, dtype=np.int64)
    order = np.lexsort((idx, -c))
    pos = np.arange(n, dtype=np.int64)
    blk, w = pos // world, pos % world
    owner = np.empty(n, dtype=np.int64)
    owner[order] = np.where(blk % 2 == 0, w, world - 1 - w)
    bucket = cost_bucket(c)
    out = []
    for r in range(world):
        t = idx[owner == r]
        t = t[np.lexsort((t, -bucket[t]))]
        out.append(t.astype(np.int32))
    return out


def tile_pixels(tiles, tiles_x: int, tw: int, th: int, W: int, nrows: int):
    """Flat pixel indices (row * W + col of the layout's output) of the tiles' pixels, tile by tile
    (row-major inside a tile), clipped to the image."""
    import numpy as np

    t = np.asarray(tiles, dtype=np.int64)
    tx, ty = t % tiles_x, t // tiles_x
    dy, dx = np.divmod(np.arange(tw * th, dtype=np.int64), tw)
    rows = ty[:, None] * th + dy[None, :]
    cols = tx[:, None] * tw + dx[None, :]
    ok = (rows < nrows) & (cols < W)
    return (rows * W + cols)[ok]


WAVE_SLOTS = 4096  # waves in flight on one MI355X at the render kernel's occupancy: 256 CUs x 4 SIMDs x 4
# rank_plans' split threshold, in units of a rank's ideal per-slot share. Chosen on the MI355X by
# tools/band_timing.py (profiles/r04q_plan_*.log, N=8 emulated): C3 0.71 (1.0) / 0.81 (1.25) /
# 0.68 (1.5) with one sample per wave, 0.74 with one pixel per wave; C5 0.96 (1.0) / 0.85 (0.75).
HEAVY = 1.25


class RankPlan:
    """One rank's share of a whole-frame layout: wave tiles (rt_render_tiles_device, in dispatch
    order) and the pixels of its heaviest tiles, rendered beside them on a second stream -- one sample
    per wave (rt_render_pixels_device, mode "sample") or one pixel per wave (RT_RENDER_PIXEL_WAVES,
    mode "pixel": a 2 x 2-pixel tile's four pixels in four waves)."""

    def __init__(self, tiles, pixels, mode="sample", split=()):
        import numpy as np

        self.tiles = np.ascontiguousarray(tiles, dtype=np.int32)
        self.pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        self.split = np.ascontiguousarray(split, dtype=np.int32)  # the tiles whose pixels `pixels` are
        self.mode = mode

    def pixel_list(self, tiles_x: int, tw: int, th: int, W: int, H: int):
        """Every pixel the plan writes: its tiles' pixels (tile order), then the split pixels."""
        import numpy as np

        return np.concatenate([tile_pixels(self.tiles, tiles_x, tw, th, W, H), self.pixels.astype(np.int64)])


def rank_plans(costs, world: int, tiles_x: int, tw: int, th: int, W: int, H: int, mode: str = "cut",
               heavy: float = HEAVY, slots: int = WAVE_SLOTS, split: str = "sample", weights=None) -> list:
    """Partition a layout's tiles over `world` ranks by their measured wave times (`contiguous_tiles`
    for mode "cut", `balanced_tiles` for "deal"), then take out of every rank's list the tiles whose
    own wave would last more than `heavy` x a rank's ideal share (total wave time / (slots x world)):
    a launch cannot end before its longest wave, so their pixels are rendered one sample per wave
    (RankPlan.pixels) instead: one sample per wave (split "sample", the measured best), one pixel per wave
    (RT_RENDER_PIXEL_WAVES, "pixel"), or "auto" (pixel when a tile holds several pixels). world == 1: one plan of every tile, nothing split.
    weights: per-tile factors of the cut (rt_group_rebalance's measured rank speeds)."""
    import numpy as np

    c = np.asarray(costs, dtype=np.float64)
    parts = contiguous_tiles(c, world, weights) if mode == "cut" else balanced_tiles(c, world)
    if world == 1:
        return [RankPlan(parts[0], [])]
    thr = heavy * c.sum() / (slots * world)
    mode = split if split != "auto" else ("sample" if tw * th == 1 else "pixel")
    out = []
    for t in parts:
        hv = c[t] > thr
        out.append(RankPlan(t[~hv], tile_pixels(t[hv], tiles_x, tw, th, W, H), mode, t[hv]))
    return out


def render_plan(scene, p, plan: RankPlan, rgb_ptr: int, argb_ptr: int, stream, side_stream):
    """Launch a RankPlan: the split pixels on side_stream (after stream's prior work), the tiles on
    stream, and stream then waits for side_stream: both run at once, the long sample waves first."""
    if len(plan.pixels):
        side_stream.wait_stream(stream)
        if plan.mode == "sample":
            scene.render_pixels_device(p, plan.pixels, rgb_ptr, argb_ptr, side_stream.cuda_stream)
        else:  # one-pixel tiles of the RT_RENDER_PIXEL_WAVES layout: tile index == pixel index
            from . import rt

            pp = rt.RenderParams(*[getattr(p, f) for f, _ in p._fields_])
            pp.flags = p.flags | rt.RENDER_PIXEL_WAVES
            scene.render_tiles_device(pp, plan.pixels, rgb_ptr, argb_ptr, side_stream.cuda_stream)
    if len(plan.tiles):
        scene.render_tiles_device(p, plan.tiles, rgb_ptr, argb_ptr, stream.cuda_stream)
    if len(plan.pixels):
        stream.wait_stream(side_stream)


def tile_assembler(pix, cap: int, device):
    """Rank 0's reassembly of gathered tile buffers: pix[r] = rank r's pixel indices (tile_pixels),
    its packed pixels in slots [0, len(pix[r])) of its [cap, ...] buffer -> the flat image."""
    import numpy as np
    import torch

    dst = torch.from_numpy(np.concatenate(pix)).to(device)
    src = torch.from_numpy(np.concatenate([np.arange(len(x), dtype=np.int64) + r * cap
                                           for r, x in enumerate(pix)])).to(device)

    def assemble_into(g, img):
        img.index_copy_(0, dst, g.reshape((-1,) + tuple(g.shape[2:])).index_select(0, src))
    return assemble_into


def assemble(gathered, H: int, band: int = BAND):
    """gathered: [world, maxrows, W, C] (torch tensor or numpy array) -> [H, W, C]."""
    world, maxrows = gathered.shape[0], gathered.shape[1]
    rest = tuple(gathered.shape[2:])
    k = maxrows // band
    g = gathered.reshape((world, k, band) + rest)
    full = g.swapaxes(0, 1).reshape((k * world * band,) + rest)  # numpy and torch alike
    return full[:H]


def gather_tiles(tile, dist, group=None, dst: int = 0, out=None):
    """The single exchange: gather equal-size padded tiles (tensor [maxrows, W, C]) to rank
    `dst` -> [world, maxrows, W, C] there, None on the other ranks. Over RCCL this is one
    point-to-point send per rank into dst (dist.gather = grouped ncclSend/ncclRecv): on
    fully connected xGMI each rank's tile crosses its own link to dst once, instead of the
    world-1 ring steps an all-gather pays for copies nobody but dst needs."""
    import torch

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank == dst and out is None:
        out = torch.empty((world,) + tuple(tile.shape), dtype=tile.dtype, device=tile.device)
    dist.gather(tile.contiguous(), list(out.unbind(0)) if rank == dst else None, dst=dst, group=group)
    return out if rank == dst else None


class FrameExchange:
    """Frames pipelined against their exchange: frame i renders into one of two tile buffers
    while frame i-1's tile is still being gathered to rank 0 (an async `dist.gather`, which
    RCCL runs on its own stream), so the xGMI transfer and rank 0's re-interleave overlap the
    next frame's kernel instead of adding to it. Every frame is still gathered and assembled;
    `finish()` drains the last one.

      ex = FrameExchange(dist, H, (maxrows, W, 3), device)
      for each frame: ex.step(lambda tile: render into tile)
      ex.finish()                      # ex.image: the last assembled frame (rank 0)

    `step` is `tile()` (this frame's buffer), the render, then `post()` (complete the previous
    frame, start this one's gather): several exchanges (e.g. float RGB and ARGB planes) can share
    one render that way.
    """

    def __init__(self, dist, H: int, tile_shape, device, dtype=None, band: int = BAND, assemble_into=None):
        """assemble_into(gathered, image): rank 0's reassembly of [world, *tile_shape] into the image
        [H, *tile_shape[1:]] (default: the interleaved row bands, `assemble`)."""
        import torch

        dtype = dtype or torch.float32
        self.dist, self.H, self.band = dist, H, band
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.assemble_into = assemble_into
        self.tiles = [torch.zeros(tuple(tile_shape), dtype=dtype, device=device) for _ in range(2)]
        root = self.rank == 0
        self.gathered = torch.empty((self.world,) + tuple(tile_shape), dtype=dtype, device=device) if root else None
        self.image = torch.empty((H,) + tuple(tile_shape[1:]), dtype=dtype, device=device) if root else None
        self.frame = 0
        self._pending = None

    def _complete(self):
        if self._pending is not None:
            self._pending.wait()  # NCCL: the current stream waits for the gather; gloo: the host does
            self._pending = None
            if self.rank == 0:
                if self.assemble_into is not None:
                    self.assemble_into(self.gathered, self.image)
                else:
                    self.image.copy_(assemble(self.gathered, self.H, self.band))

    def tile(self):
        """This frame's tile buffer (render into it, then post())."""
        return self.tiles[self.frame % 2]

    def post(self):
        """Complete frame-1 (gathered + assembled; its buffer is free again) and start this
        frame's gather. The render was enqueued before the wait: the two overlap."""
        tile = self.tile()
        self._complete()
        self._pending = self._gather(tile)
        self.frame += 1

    def step(self, render):
        render(self.tile())
        self.post()

    def _gather(self, tile):
        if not getattr(self, "_use_allgather", False):
            try:
                outs = list(self.gathered.unbind(0)) if self.rank == 0 else None
                return self.dist.gather(tile, outs, dst=0, async_op=True)
            except (RuntimeError, ValueError, NotImplementedError):
                # a backend without gather: the same exchange as an all-gather (every rank
                # receives every tile; only rank 0 assembles them)
                self._use_allgather = True
        if getattr(self, "_ag", None) is None:
            import torch
            self._ag = torch.empty((self.world,) + tuple(tile.shape), dtype=tile.dtype, device=tile.device)
            if self.rank == 0:
                self.gathered = self._ag
        return self.dist.all_gather_into_tensor(self._ag.view(-1), tile.view(-1), async_op=True)

    def finish(self):
        self._complete()
        return self.image


def photon_shard(rank: int, world: int, count: int) -> tuple[int, int]:
    """Emitted-photon index range [first, first+n) of a rank (every light)."""
    first = rank * count // world
    return first, (rank + 1) * count // world - first


def merge_photon_shards(shards):
    """shards: per rank (pos [n,3], pwr [n,3], per_light [L]) in rank order -> the full
    photon_list in the reference's insertion order: light-major, then photon index
    (rank shards hold consecutive index ranges), then path order."""
    import numpy as np

    pos, pwr = [], []
    nl = len(shards[0][2])
    offs = [np.concatenate([[0], np.cumsum(s[2])]) for s in shards]
    for light in range(nl):
        for r, (p, w, _) in enumerate(shards):
            a, b = offs[r][light], offs[r][light + 1]
            pos.append(p[a:b]); pwr.append(w[a:b])
    return np.concatenate(pos), np.concatenate(pwr)


def _all_gather_rows(dist, rows, device):
    """All-gather a ragged float64 array [n_r, C] from every rank -> list of [n_r, C] numpy arrays
    in rank order: counts first, then one all_gather of the tiles padded to the largest count
    (on `device`: the GPU under RCCL, the host under gloo)."""
    import numpy as np
    import torch

    world = dist.get_world_size()
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    cap = max(1, max(ns))
    buf = torch.zeros((cap, rows.shape[1]), dtype=torch.float64, device=device)
    buf[: rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows)).to(device)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return [o[:k].cpu().numpy() for o, k in zip(outs, ns)]


def build_photons_sharded(scene, seed: int, count: int, dist=None, device="cuda"):
    """The photon pre-pass split over ranks: each rank shoots its emitted-photon
    index range, the shards (positions, powers, per-light counts) are all-gathered as tensors
    (RCCL on `device`), merged into the reference's photon_list order, and every rank builds
    the same photon map."""
    import numpy as np

    rank = dist.get_rank() if dist else 0
    world = dist.get_world_size() if dist else 1
    first, n = photon_shard(rank, world, count)
    pos, pwr, per = scene.shoot_photons(seed, first, n)
    if dist is None:
        shards = [(pos, pwr, per)]
    else:
        rec = _all_gather_rows(dist, np.concatenate([pos.reshape(-1, 3), pwr.reshape(-1, 3)], 1), device)
        pers = _all_gather_rows(dist, np.asarray(per, dtype=np.float64).reshape(1, -1), device)
        shards = [(r[:, :3], r[:, 3:], pl[0].astype(np.int64)) for r, pl in zip(rec, pers)]
    full_pos, full_pwr = merge_photon_shards(shards)
    scene.set_photons(full_pos, full_pwr)
    return len(full_pos)


class RankRenderer:
    """One rank's share of bench.py's N-GPU step: renders the rank's part of the frame with the HIP
    kernel into device buffers on the current stream (float RGB and the reference's ARGB ints,
    myObjShader.java:671), and with N > 1 hands the planes in `planes` to a FrameExchange each
    (gathered to rank 0 and reassembled there, pipelined against the next frame). The ARGB plane is
    the frame the reference produces (`rndrdImg.pixels`, myScene.java:1171-1177): the kernel packs it
    from the double colour, so rank 0 receives the 1-GPU ints exactly (packing the gathered float RGB
    again could differ by one in a channel whose double value rounds up to the next float).

    partition "tiles" (default): the frame's wave tiles cut into contiguous runs of equal measured
    cost (`rank_plans`: rank 0 calibrates, rt_tile_costs, and broadcasts the costs), the tiles whose
    own wave would outlast a rank's share rendered one sample per wave beside them; rank r renders
    its plan into a whole-frame buffer (rt_render_tiles_device + rt_render_pixels_device) and packs
    its pixels for the gather. "deal": the tiles dealt serpentine by cost instead (`balanced_tiles`).
    partition "bands": the interleaved 8-row bands of `rows_of` (rt_render_device).
    `stage_host`: copy the tiles to host memory before the exchange (the gloo backend, which cannot
    gather device tensors; used to run this exact path as several processes on one GPU).

      rr = RankRenderer(scene, W, H, spp, seed, dist)
      rr.calibrate()                 # untimed: the layout's tile-schedule calibration renders
      for each frame: rr.step()      # optional (start, end) HIP events around the kernel
      rgb, argb = rr.finish()        # rank 0: the last assembled frame, [H, W, 3] float32 and
                                     # [H, W] int32 (device / host; None for a plane not exchanged)
    """

    def __init__(self, scene, W, H, spp, seed, dist=None, stage_host=False, band=BAND, planes=("rgb", "argb"),
                 partition="tiles"):
        import numpy as np
        import torch

        from . import rt

        assert partition in ("tiles", "deal", "bands")
        assert set(planes) <= {"rgb", "argb"} and planes
        self.scene, self.W, self.H = scene, W, H
        self.dist = dist
        self.rank = dist.get_rank() if dist else 0
        self.world = dist.get_world_size() if dist else 1
        self.partition = ("tiles" if partition == "deal" else partition) if self.world > 1 else "bands"
        self.stream = torch.cuda.current_stream()
        self.stage_host = stage_host
        self.ex = {}
        xdev = "cpu" if stage_host else "cuda"  # where the exchanged tiles (and collectives' tensors) live
        if self.partition == "bands":
            r0, r1, step, b = rows_of(self.rank, self.world, H, band)
            self.p = rt.params(W, H, spp=spp, seed=seed, rows=(r0, r1), row_step=step, row_band=b)
            self.rows = (r0, r1, step, b)
            self.maxrows = max_tile_rows(self.world, H, band)
            assert rt.nrows_of(self.p) <= self.maxrows
            self.rgb = torch.empty((self.maxrows, W, 3), dtype=torch.float32, device="cuda")
            self.argb = torch.empty((self.maxrows, W), dtype=torch.int32, device="cuda")
            if dist is not None and self.world > 1:
                if "rgb" in planes:
                    self.ex["rgb"] = FrameExchange(dist, H, (self.maxrows, W, 3), xdev, band=band)
                if "argb" in planes:
                    self.ex["argb"] = FrameExchange(dist, H, (self.maxrows, W), xdev, dtype=torch.int32, band=band)
            return
        # cost-balanced parts of the whole-frame layout
        self.p = rt.params(W, H, spp=spp, seed=seed)
        self.rows = (0, H, 1, 1)
        ntiles, tiles_x, tw, th = scene.tile_layout(self.p)
        cost = torch.zeros(ntiles, dtype=torch.int64, device=xdev)
        if self.rank == 0:
            cost.copy_(torch.from_numpy(scene.tile_costs(self.p).astype(np.int64)))
        dist.broadcast(cost, 0)
        plans = rank_plans(cost.cpu().numpy(), self.world, tiles_x, tw, th, W, H,
                           mode="cut" if partition == "tiles" else "deal")
        self.plan = plans[self.rank]
        self.tiles = self.plan.tiles
        self.side = torch.cuda.Stream()
        pix = [pl.pixel_list(tiles_x, tw, th, W, H) for pl in plans]
        self.npix = len(pix[self.rank])
        self.pix = torch.from_numpy(pix[self.rank]).to("cuda")
        cap = max(len(x) for x in pix)
        self.rgb = torch.empty((H * W, 3), dtype=torch.float32, device="cuda")
        self.argb = torch.empty((H * W,), dtype=torch.int32, device="cuda")
        assemble_into = tile_assembler(pix, cap, xdev) if self.rank == 0 else None
        if "rgb" in planes:
            self.ex["rgb"] = FrameExchange(dist, H * W, (cap, 3), xdev, assemble_into=assemble_into)
        if "argb" in planes:
            self.ex["argb"] = FrameExchange(dist, H * W, (cap,), xdev, dtype=torch.int32, assemble_into=assemble_into)

    def render(self, rgb=None, argb=None, ev=None):
        if ev:
            ev[0].record(self.stream)
        rgb = self.rgb if rgb is None else rgb
        argb = self.argb if argb is None else argb
        if self.partition == "tiles":
            render_plan(self.scene, self.p, self.plan, rgb.data_ptr(), argb.data_ptr(), self.stream, self.side)
        else:
            self.scene.render_device(self.p, rgb.data_ptr(), argb.data_ptr(), self.stream.cuda_stream)
        if ev:
            ev[1].record(self.stream)

    def calibrate(self, n=2):
        """A row layout's first two renders order its tiles (probe, then measured wave times); a tile
        partition was calibrated at construction (these renders only warm up)."""
        import torch

        for _ in range(n):
            self.render()
        torch.cuda.synchronize()

    def step(self, ev=None):
        if not self.ex:
            self.render(ev=ev)
            return
        tiles = {k: e.tile() for k, e in self.ex.items()}
        if self.partition == "tiles":
            import torch

            self.render(ev=ev)
            for k, t in tiles.items():  # this rank's pixels, packed in tile order (device gather)
                if self.stage_host:  # device -> host (synchronous), then the gloo gather
                    t[: self.npix].copy_(torch.index_select(getattr(self, k), 0, self.pix))
                else:
                    torch.index_select(getattr(self, k), 0, self.pix, out=t[: self.npix])
        elif self.stage_host:
            self.render(ev=ev)
            for k, t in tiles.items():
                t.copy_(getattr(self, k))  # device -> host (synchronous), then the gloo gather
        else:
            self.render(tiles.get("rgb"), tiles.get("argb"), ev)
        for e in self.ex.values():
            e.post()

    def finish(self):
        """Drain the pipelined exchange; rank 0 gets the assembled frame (rgb [H, W, 3], argb
        [H, W]; None for a plane not exchanged), the other ranks (None, None)."""
        if self.ex:
            out = {k: e.finish() for k, e in self.ex.items()}
            if self.rank != 0:
                return None, None
            rgb, argb = out.get("rgb"), out.get("argb")
            if self.partition == "tiles":
                rgb = rgb.reshape(self.H, self.W, 3) if rgb is not None else None
                argb = argb.reshape(self.H, self.W) if argb is not None else None
            return rgb, argb
        if self.rank != 0:
            return None, None
        return self.rgb[: self.H], self.argb[: self.H]
