"""Full-size GPU properties of the SURVEY 8(d) configs C4 and C5 (BASELINE.json configs[3],
configs[4]), which the parity tests otherwise cover only at reduced size:

* deterministic: two renders are bit-equal;
* the N-GPU partitions: the eight cost-balanced tile lists of an 8-rank split (the layout
  bench.py --gpus 8 runs) and the eight row-band tiles (multigpu.rows_of, --partition bands)
  reassemble to the 1-GPU frame bit for bit, float RGB and ARGB alike;
* parity: a row subsample of the full frame against the oracle at the full spp, with the
  decision-exact bar of tests/parity.py (per-channel |d| <= 1e-4 where decisions agree, 0
  decision mismatches, ARGB equal).

C4 = data/plnts3ColsBunnies.cli 2048^2 x 64 spp (~0.6 s per GPU frame); C5 = data/t11.cli
1024^2 x 64 spp at its real photon map (2.68 M photons, k = 200; the oracle gathers over the
GPU's photon_list, which test_c5_full_prepass_and_k200_gather_parity checks is the oracle's
own bit for bit).
"""
import numpy as np
import pytest

from distraytracer_old_amd import multigpu, rt, scenes
from oracle.oracle import OracleScene
from tests.parity import assert_exact_decisions, compare

pytestmark = pytest.mark.gpu


def _split_equals_full(g, W, H, spp, seed, rgb, argb, world=8):
    maxrows = multigpu.max_tile_rows(world, H)
    tr = np.zeros((world, maxrows, W, 3), np.float32)
    ta = np.zeros((world, maxrows, W), np.int32)
    for r in range(world):
        r0, r1, step, band = multigpu.rows_of(r, world, H)
        t, a = g.render(W, H, spp=spp, seed=seed, rows=(r0, r1), row_step=step, row_band=band)
        n = multigpu.tile_rows(r, world, H)
        assert t.shape[0] == n
        tr[r, :n], ta[r, :n] = t, a
    assert np.array_equal(multigpu.assemble(ta, H), argb)
    assert np.array_equal(multigpu.assemble(tr, H).view(np.uint32), rgb.view(np.uint32))


def _plan_split_equals_full(g, W, H, spp, seed, rgb, argb, world=8, expect_split=True):
    """bench.py --gpus 8's default split (multigpu.rank_plans: contiguous cost-balanced runs, the
    heaviest tiles' pixels one sample per wave on a second stream) == the 1-GPU frame."""
    import torch

    p = rt.params(W, H, spp=spp, seed=seed)
    n, tx, tw, th = g.tile_layout(p)
    plans = multigpu.rank_plans(g.tile_costs(p), world, tx, tw, th, W, H)
    if expect_split:  # the one-sample-per-wave path is exercised (C4's tiles are all short: none split)
        assert sum(len(pl.pixels) for pl in plans) > 0
    out_rgb = torch.full((H * W, 3), -1.0, device="cuda")
    out_argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    b_rgb, b_argb = torch.empty_like(out_rgb), torch.empty_like(out_argb)
    st, side = torch.cuda.current_stream(), torch.cuda.Stream()
    for pl in plans:
        b_rgb.fill_(-2.0)
        multigpu.render_plan(g, p, pl, b_rgb.data_ptr(), b_argb.data_ptr(), st, side)
        pix = torch.from_numpy(pl.pixel_list(tx, tw, th, W, H)).cuda()
        out_rgb[pix] = b_rgb[pix]
        out_argb[pix] = b_argb[pix]
    torch.cuda.synchronize()
    assert np.array_equal(out_argb.cpu().numpy().reshape(H, W), argb)
    assert np.array_equal(out_rgb.cpu().numpy().reshape(H, W, 3).view(np.uint32), rgb.view(np.uint32))


def _tiles_split_equals_full(g, W, H, spp, seed, rgb, argb, world=8):
    """The cost-balanced tile partition of bench.py --gpus 8 (measured costs, balanced_tiles,
    rt_render_tiles_device per rank, pixels scattered back by tile_pixels) == the 1-GPU frame."""
    import torch

    p = rt.params(W, H, spp=spp, seed=seed)
    n, tx, tw, th = g.tile_layout(p)
    parts = multigpu.balanced_tiles(g.tile_costs(p), world)
    assert sum(len(t) for t in parts) == n
    out_rgb = torch.full((H * W, 3), -1.0, device="cuda")
    out_argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    b_rgb, b_argb = torch.empty_like(out_rgb), torch.empty_like(out_argb)
    st = torch.cuda.current_stream()
    for t in parts:
        b_rgb.fill_(-2.0)
        g.render_tiles_device(p, t, b_rgb.data_ptr(), b_argb.data_ptr(), st.cuda_stream)
        pix = torch.from_numpy(multigpu.tile_pixels(t, tx, tw, th, W, H)).cuda()
        out_rgb[pix] = b_rgb[pix]
        out_argb[pix] = b_argb[pix]
    torch.cuda.synchronize()
    assert np.array_equal(out_argb.cpu().numpy().reshape(H, W), argb)
    assert np.array_equal(out_rgb.cpu().numpy().reshape(H, W, 3).view(np.uint32), rgb.view(np.uint32))


def _group_equals_full(g, W, H, spp, seed, rgb, argb, world=8):
    """The native N-GPU frame (rt_group_*, VERDICT r04 Next #1) emulated on one GPU: 8 ranks on device
    0 with the device-copy transport -- plans, split pixels, pack, exchange, scatter -- == the 1-GPU
    frame bit for bit."""
    with rt.Group.create([g] * world, W, H, spp=spp, seed=seed, rgb=True, copy=True) as grp:
        c, a = grp.render_host(W, H)
    assert np.array_equal(a, argb)
    assert np.array_equal(c.view(np.uint32), rgb.view(np.uint32))


def test_c4_full_size_properties():
    cli, W, H, spp, seed = scenes.CONFIGS["C4"]
    scenes.ensure_bun69k()
    tex = scenes.prepare(cli)
    g = rt.Scene.load_cli(cli, textures=tex)
    rgb, argb = g.render(W, H, spp=spp, seed=seed)
    rgb2, argb2 = g.render(W, H, spp=spp, seed=seed)
    assert np.array_equal(argb, argb2) and np.array_equal(rgb.view(np.uint32), rgb2.view(np.uint32))
    assert rgb.min() >= 0 and rgb.max() <= 1.0
    _split_equals_full(g, W, H, spp, seed, rgb, argb)
    _tiles_split_equals_full(g, W, H, spp, seed, rgb, argb)
    _plan_split_equals_full(g, W, H, spp, seed, rgb, argb, expect_split=False)
    _group_equals_full(g, W, H, spp, seed, rgb, argb)
    # oracle rows through the glass bunnies, the columns and the sky (the oracle runs ~3 s a row)
    o = OracleScene(scenes.SCENE_DIR, cli, tex)
    for row in (700, 1300, 1900):
        ro, ao, _ = o.render(W, H, spp=spp, seed=seed, rows=(row, row + 1))
        assert_exact_decisions(compare(rgb[row:row + 1], argb[row:row + 1], ro, ao))


def test_c5_full_size_properties():
    cli, W, H, spp, seed = scenes.CONFIGS["C5"]
    g = rt.Scene.load_cli(cli, textures={})
    g.build_photons(seed)
    assert g.info()["photons"] > 2_600_000
    rgb, argb = g.render(W, H, spp=spp, seed=seed)
    rgb2, argb2 = g.render(W, H, spp=spp, seed=seed)
    assert np.array_equal(argb, argb2) and np.array_equal(rgb.view(np.uint32), rgb2.view(np.uint32))
    assert rgb.min() >= 0 and rgb.max() <= 1.0
    _split_equals_full(g, W, H, spp, seed, rgb, argb)
    _tiles_split_equals_full(g, W, H, spp, seed, rgb, argb)
    _plan_split_equals_full(g, W, H, spp, seed, rgb, argb)
    _group_equals_full(g, W, H, spp, seed, rgb, argb)
    o = OracleScene(scenes.SCENE_DIR, cli)
    o.set_photons(*g.photons())
    for row in (100, 400, 640, 900):  # ceiling light, spheres (mirror / glass: caustics), floor
        ro, ao, _ = o.render(W, H, spp=spp, seed=seed, rows=(row, row + 1))
        assert_exact_decisions(compare(rgb[row:row + 1], argb[row:row + 1], ro, ao))


def test_c3_full_size_plan_split():
    """The headline config's 8-rank split (contiguous cost-balanced runs + the heaviest tiles' pixels
    one sample per wave) reassembles to the 1-GPU frame bit for bit."""
    cli, W, H, spp, seed = scenes.CONFIGS["C3"]
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    rgb, argb = g.render(W, H, spp=spp, seed=seed)
    _plan_split_equals_full(g, W, H, spp, seed, rgb, argb)
    _group_equals_full(g, W, H, spp, seed, rgb, argb)
