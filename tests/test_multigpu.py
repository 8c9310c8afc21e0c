"""Multi-GPU partition + exchange (distraytracer_old_amd/multigpu.py) with
world_size-2 gloo on CPU. The per-rank renderer here is the oracle (a CPU
stand-in for the HIP kernel, same row semantics): the gathered, re-interleaved
image must equal the single-process image bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distraytracer_old_amd import multigpu, scenes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, H, W, q):
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from oracle.oracle import OracleScene

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = OracleScene(scenes.SCENE_DIR, "c3shinyBall.cli", scenes.prepare("c3shinyBall.cli"))
    band = 3
    rows = multigpu.image_rows(rank, world, H, band)
    # the oracle renders the rank's bands one by one (the HIP kernel does them in one launch)
    parts = [o.render(W, H, spp=2, seed=11, rows=(b0, min(b0 + band, H)), threads=2)[0]
             for b0 in rows[::band]]
    rgb = np.concatenate(parts)
    assert rgb.shape[0] == len(rows)
    tile = torch.zeros((multigpu.max_tile_rows(world, H, band), W, 3), dtype=torch.float32)
    tile[: rgb.shape[0]] = torch.from_numpy(rgb)
    g = multigpu.gather_tiles(tile, dist)
    if rank == 0:
        q.put(multigpu.assemble(g, H, band).numpy())
    else:
        assert g is None
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_equals_single_image():
    from oracle.oracle import OracleScene

    H, W, world = 37, 24, 2  # odd height: ragged tiles
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, H, W, q)) for r in range(world)]
    for p in ps:
        p.start()
    full = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = OracleScene(scenes.SCENE_DIR, "c3shinyBall.cli", scenes.prepare("c3shinyBall.cli"))
    ref, _, _ = o.render(W, H, spp=2, seed=11)
    assert np.array_equal(full, ref)


def _exchange_worker(rank, world, port, H, W, q, allgather=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    band = 2
    rows = torch.tensor(multigpu.image_rows(rank, world, H, band), dtype=torch.float32)
    maxrows = multigpu.max_tile_rows(world, H, band)
    ex = multigpu.FrameExchange(dist, H, (maxrows, W, 1), "cpu", band=band)
    ex._use_allgather = allgather  # the fallback for backends without gather
    seen = []
    for f in range(4):
        def render(tile, f=f):  # frame f's pixel value: 1000 * f + image row
            tile.zero_()
            tile[: len(rows), :, 0] = (1000 * f + rows)[:, None]
        ex.step(render)
        if rank == 0 and f > 0:
            seen.append(ex.image[:, 0, 0].clone())  # frame f-1, assembled
    last = ex.finish()
    if rank == 0:
        seen.append(last[:, 0, 0].clone())
        q.put(torch.stack(seen).numpy())
    else:
        assert last is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("allgather", [False, True])
def test_gloo_world3_pipelined_exchange_delivers_every_frame(allgather):
    """FrameExchange (bench.py's N-GPU step): frame i's gather overlaps frame i+1's render;
    rank 0 still assembles every frame exactly, and finish() drains the last one (also through
    the all-gather fallback)."""
    H, W, world = 13, 3, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_exchange_worker, args=(r, world, port, H, W, q, allgather)) for r in range(world)]
    for p in ps:
        p.start()
    frames = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.stack([1000 * f + np.arange(H) for f in range(4)]).astype(np.float32)
    assert np.array_equal(frames, expect)


def _planes_worker(rank, world, port, H, W, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = torch.tensor(multigpu.image_rows(rank, world, H), dtype=torch.int64)
    maxrows = multigpu.max_tile_rows(world, H)
    # RankRenderer's pattern: one render fills the float-RGB and ARGB planes, then each is posted
    ex = {"rgb": multigpu.FrameExchange(dist, H, (maxrows, W, 3), "cpu"),
          "argb": multigpu.FrameExchange(dist, H, (maxrows, W), "cpu", dtype=torch.int32)}
    for f in range(3):
        t = {k: e.tile() for k, e in ex.items()}
        t["rgb"].zero_()
        t["rgb"][: len(rows)] = (rows.to(torch.float32) / 7 + f)[:, None, None]
        t["argb"].zero_()
        # ARGB ints as the kernel packs them (alpha 255: negative as int32)
        t["argb"][: len(rows)] = ((0xFF000000 + rows * 65793 + f) - (1 << 32)).to(torch.int32)[:, None]
        for e in ex.values():
            e.post()
    out = {k: e.finish() for k, e in ex.items()}
    if rank == 0:
        q.put((out["rgb"].numpy(), out["argb"].numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_rgb_and_argb_planes():
    """The N-rank frame's two planes (float RGB and the reference's ARGB ints, myObjShader.java:671)
    go through their own exchanges after one shared render; rank 0 assembles both exactly."""
    H, W, world = 40, 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_planes_worker, args=(r, world, port, H, W, q)) for r in range(world)]
    for p in ps:
        p.start()
    rgb, argb = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    r = np.arange(H)
    assert np.array_equal(rgb, np.broadcast_to((r.astype(np.float32) / 7 + 2)[:, None, None], (H, W, 3)))
    expect = ((0xFF000000 + r * 65793 + 2) - (1 << 32)).astype(np.int32)
    assert argb.dtype == np.int32 and np.array_equal(argb, np.broadcast_to(expect[:, None], (H, W)))


def test_assemble_numpy_ragged():
    for H, W, world, band in [(10, 3, 4, 1), (37, 5, 3, 4), (1024, 2, 8, 8), (19, 2, 8, 8)]:
        img = np.arange(H * W).reshape(H, W, 1)
        tiles = np.zeros((world, multigpu.max_tile_rows(world, H, band), W, 1), dtype=img.dtype)
        for r in range(world):
            rows = img[multigpu.image_rows(r, world, H, band)]
            tiles[r, : rows.shape[0]] = rows
            assert rows.shape[0] == multigpu.tile_rows(r, world, H, band)
        assert np.array_equal(multigpu.assemble(tiles, H, band), img)


def test_row_band_params_match_partition():
    """rt_render_params (row0, row_step, row_band) select exactly multigpu.image_rows."""
    from distraytracer_old_amd import rt
    for H, world, band in [(1024, 8, 8), (37, 3, 4), (300, 2, 8), (10, 4, 1)]:
        for rank in range(world):
            r0, r1, step, b = multigpu.rows_of(rank, world, H, band)
            p = rt.params(64, H, rows=(r0, r1), row_step=step, row_band=b)
            rows = [r0 + (i // b) * step * b + i % b for i in range(rt.nrows_of(p))]
            assert rows == multigpu.image_rows(rank, world, H, band)


def test_merge_photon_shards_restores_insertion_order():
    """Shards (rank r holds emitted-photon indices [r*P/N, (r+1)*P/N) of every light, each
    light-major) merge back into the reference's light-major photon_list order."""
    import numpy as np
    from distraytracer_old_amd import multigpu

    # full list: light 0 photons 0..9 (some store 0 or 2 photons), light 1 photons 0..9
    rng = np.random.default_rng(1)
    stored = rng.integers(0, 3, size=(2, 10))
    full = [(l, i, k) for l in range(2) for i in range(10) for k in range(stored[l, i])]
    pos_full = np.array([[l, i, k] for l, i, k in full], dtype=float)
    shards = []
    for r in range(3):
        first, n = multigpu.photon_shard(r, 3, 10)
        rows = [(l, i, k) for l in range(2) for i in range(first, first + n) for k in range(stored[l, i])]
        per = np.array([sum(1 for x in rows if x[0] == l) for l in range(2)])
        p = np.array([[l, i, k] for l, i, k in rows], dtype=float).reshape(-1, 3)
        shards.append((p, p * 2, per))
    mp, mw = multigpu.merge_photon_shards(shards)
    assert np.array_equal(mp, pos_full) and np.array_equal(mw, pos_full * 2)
    assert sum(multigpu.photon_shard(r, 3, 10)[1] for r in range(3)) == 10


def test_balanced_tiles_partition():
    """Cost-balanced tile partition (multigpu.balanced_tiles): every tile exactly once, the same
    partition for the same costs, cost sums within one tile's cost of each other, and each rank's
    list longest-first by quarter-octave bucket (row-major inside a bucket)."""
    rng = np.random.default_rng(7)
    for n, world in [(1000, 2), (262144, 8), (37, 3), (5, 8)]:
        costs = (rng.pareto(1.5, n) * 1000 + 1).astype(np.uint32)
        costs[rng.random(n) < 0.05] = costs[0]  # ties
        parts = multigpu.balanced_tiles(costs, world)
        assert len(parts) == world
        allt = np.concatenate(parts)
        assert np.array_equal(np.sort(allt), np.arange(n))
        again = multigpu.balanced_tiles(costs.copy(), world)
        assert all(np.array_equal(a, b) for a, b in zip(parts, again))
        sums = [int(costs[p].astype(np.int64).sum()) for p in parts]
        assert max(sums) - min(sums) <= int(costs.max())
        b = multigpu.cost_bucket(costs)
        for p in parts:
            kb = b[p]
            assert np.all(np.diff(kb) <= 0)
            same = np.diff(kb) == 0
            assert np.all(np.diff(p)[same] > 0)


def test_tile_pixels_cover_the_image():
    """The tiles of a layout (tw x th pixel wave tiles, clipped at the image edge) cover every
    pixel exactly once, whatever the partition."""
    for W, H, tw, th in [(1024, 1024, 2, 2), (37, 19, 2, 2), (10, 7, 1, 1), (13, 9, 8, 8)]:
        tx = -(-W // tw)
        n = tx * -(-H // th)
        parts = multigpu.balanced_tiles(np.arange(n)[::-1] % 17 + 1, 3)
        pix = np.concatenate([multigpu.tile_pixels(t, tx, tw, th, W, H) for t in parts])
        assert np.array_equal(np.sort(pix), np.arange(W * H))


def _tiles_worker(rank, world, port, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tw, th = 2, 2
    tx = -(-W // tw)
    n = tx * -(-H // th)
    cost = torch.zeros(n, dtype=torch.int64)
    if rank == 0:  # only rank 0 measures (RankRenderer: rt_tile_costs), the others receive them
        cost.copy_(torch.from_numpy((np.arange(n) * 7919 % 1000 + 1).astype(np.int64)))
    dist.broadcast(cost, 0)
    parts = multigpu.balanced_tiles(cost.numpy(), world)
    pix = [multigpu.tile_pixels(t, tx, tw, th, W, H) for t in parts]
    cap = max(len(x) for x in pix)
    mine = torch.from_numpy(pix[rank])
    asm = multigpu.tile_assembler(pix, cap, "cpu") if rank == 0 else None
    ex = multigpu.FrameExchange(dist, H * W, (cap, 3), "cpu", assemble_into=asm)
    frames = []
    for f in range(3):
        # the rank's "render": a whole-frame buffer where only its own tiles' pixels are right
        full = torch.full((H * W, 3), -1.0)
        full[mine] = (torch.arange(H * W, dtype=torch.float32)[mine] + 1000 * f)[:, None]
        t = ex.tile()
        t.zero_()
        torch.index_select(full, 0, mine, out=t[: len(mine)])
        ex.post()
        if rank == 0 and f > 0:
            frames.append(ex.image[:, 0].clone())
    last = ex.finish()
    if rank == 0:
        frames.append(last[:, 0].clone())
        q.put(torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world3_tile_partition_reassembles():
    """The N-rank tile path (RankRenderer partition="tiles"): costs broadcast from rank 0, the same
    partition on every rank, each rank's pixels packed in tile order, gathered and scattered back
    by rank 0 -- every pixel of every frame in place (ragged image, unequal tile counts)."""
    W, H, world = 37, 19, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tiles_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in ps:
        p.start()
    frames = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.stack([np.arange(H * W) + 1000 * f for f in range(3)]).astype(np.float32)
    assert np.array_equal(frames, expect)


def test_rank_plans_cover_the_frame_and_split_only_heavy_tiles():
    """multigpu.rank_plans (bench.py --gpus N's default split): contiguous runs of equal cost, every
    pixel exactly once, and only tiles costlier than heavy x a rank's ideal share (total / (4096 x N))
    become one-sample-per-wave pixels; split "auto" on a multi-pixel layout picks per-pixel waves."""
    rng = np.random.default_rng(3)
    W, H, tw, th = 256, 200, 2, 2
    tx = W // tw
    n = tx * (H // th)
    costs = (rng.pareto(2.0, n) * 20 + 5).astype(np.int64)
    costs[rng.choice(n, 5, replace=False)] = 10 ** 7  # five outliers
    for world in (2, 3, 8):
        plans = multigpu.rank_plans(costs, world, tx, tw, th, W, H)
        pix = np.concatenate([pl.pixel_list(tx, tw, th, W, H) for pl in plans])
        assert np.array_equal(np.sort(pix), np.arange(W * H))
        thr = multigpu.HEAVY * costs.sum() / (multigpu.WAVE_SLOTS * world)
        assert sum(len(pl.pixels) for pl in plans) == 4 * int((costs > thr).sum())
        for pl in plans:
            assert (costs[pl.tiles] <= thr).all()
            assert pl.mode == "sample"
    assert all(pl.mode == "pixel" for pl in multigpu.rank_plans(costs, 8, tx, tw, th, W, H, split="auto"))
    one = multigpu.rank_plans(costs, 1, tx, tw, th, W, H)
    assert len(one) == 1 and len(one[0].pixels) == 0 and len(one[0].tiles) == n
