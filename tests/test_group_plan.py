"""The native multi-GPU plan (rt_rank_plan, csrc/group.hip plan_ranks) against the independent
Python restatement (multigpu.rank_plans): the same run tiles in the same dispatch order and the same
split pixels for every rank, on measured-like and adversarial cost vectors (CPU only)."""
import numpy as np
import pytest

from distraytracer_old_amd import multigpu, rt


def _native_plans(cost, world, tiles_x, tw, th, W, H, heavy=multigpu.HEAVY, slots=multigpu.WAVE_SLOTS, weight=None):
    owner, order = rt.rank_plan(cost, world, heavy, slots, weight)
    o = owner[order]
    out = []
    for r in range(world):
        run, split = order[o == r], order[o == world + r]
        out.append((run, multigpu.tile_pixels(split, tiles_x, tw, th, W, H)))
    return owner, order, out


def _costs(kind, n, seed):
    g = np.random.default_rng(seed)
    if kind == "lognormal":  # wave times of a real frame: heavy right tail
        return np.minimum(g.lognormal(7.0, 1.2, n), 2**32 - 1).astype(np.uint32)
    if kind == "flat":
        return np.full(n, 1000, dtype=np.uint32)
    if kind == "zeros":
        c = g.integers(0, 3000, n).astype(np.uint32)
        c[g.random(n) < 0.3] = 0
        return c
    if kind == "pow2":  # exact bucket boundaries
        return (2 ** g.integers(0, 31, n)).astype(np.uint32)
    if kind == "allzero":
        return np.zeros(n, dtype=np.uint32)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["lognormal", "flat", "zeros", "pow2", "allzero"])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_native_plan_equals_python(kind, world):
    W, H, tw, th = 300, 202, 2, 2  # ragged: the last tile row / column is clipped
    tiles_x = -(-W // tw)
    n = tiles_x * (-(-H // th))
    cost = _costs(kind, n, seed=world * 7 + len(kind))
    owner, order, nat = _native_plans(cost, world, tiles_x, tw, th, W, H, slots=64)
    py = multigpu.rank_plans(cost, world, tiles_x, tw, th, W, H, slots=64)
    assert sorted(order.tolist()) == list(range(n))
    for r in range(world):
        assert np.array_equal(nat[r][0], py[r].tiles), r
        assert np.array_equal(nat[r][1], py[r].pixels), r
    # every pixel of the frame belongs to exactly one rank
    allpix = np.concatenate([np.concatenate([multigpu.tile_pixels(t, tiles_x, tw, th, W, H), p]) for t, p in nat])
    assert np.array_equal(np.sort(allpix), np.arange(W * H))


def test_cost_bucket_matches_dispatch_key():
    c = np.array([0, 1, 2, 3, 4, 5, 6, 7, 8, 1189, 1190, 1414, 1415, 1681, 1682, 2**31, 2**32 - 1], dtype=np.uint32)
    owner, order = rt.rank_plan(c, 1)
    b = multigpu.cost_bucket(c)
    # dispatch order: bucket descending, index ascending inside a bucket
    assert np.array_equal(order, np.lexsort((np.arange(len(c)), -b)))
    assert b[0] == 0 and b[1] == 1 and b[2] == 5 and b[-2] == 1 + 4 * 31


def test_rank_plan_rejects_bad_arguments():
    with pytest.raises(rt.RTError):
        rt.rank_plan(np.ones(4, dtype=np.uint32), 0)


@pytest.mark.parametrize("world", [2, 8])
def test_weighted_cut_equals_python(world):
    """rt_group_rebalance's cut: the runs hold equal sums of cost x weight (per-rank speed factors)."""
    W, H, tw, th = 256, 130, 2, 2
    tiles_x = -(-W // tw)
    n = tiles_x * (-(-H // th))
    cost = _costs("lognormal", n, seed=world)
    g = np.random.default_rng(world)
    weight = np.repeat(g.uniform(0.6, 1.7, world), -(-n // world))[:n]
    owner, order, nat = _native_plans(cost, world, tiles_x, tw, th, W, H, slots=64, weight=weight)
    py = multigpu.rank_plans(cost, world, tiles_x, tw, th, W, H, slots=64, weights=weight)
    for r in range(world):
        assert np.array_equal(nat[r][0], py[r].tiles), r
        assert np.array_equal(nat[r][1], py[r].pixels), r
    # the weights move the cut (and only the cut: the split tiles and the dispatch order are the same)
    o0, d0 = rt.rank_plan(cost, world, 0.0, 64)
    assert np.array_equal(d0, order) and np.array_equal(o0 >= world, owner >= world)
    assert not np.array_equal(o0, owner)
