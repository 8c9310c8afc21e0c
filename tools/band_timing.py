#!/usr/bin/env python3
"""Per-rank kernel time of the multi-GPU partitions, emulated on one GPU: max over ranks vs
full-frame/N (strong-scaling efficiency of the kernel alone).

  tools/band_timing.py [BANDS] [CFG] [--tiles [--cut] [--heavy H] [--split sample|pixel|auto]]
                       [--worlds 2,4,8] [--flags F]

bands: rank r renders the interleaved row bands of multigpu.rows_of (rt_render_device, longest-
first measured tile schedule of its own layout); --tiles: multigpu.rank_plans over the whole
frame's measured wave times -- a serpentine deal by cost, or with --cut the contiguous runs of
equal cost (bench.py --gpus N's default) -- with the tiles above H x a rank's per-slot share split
per sample (or per pixel) on a side stream; every rank's plan timed with HIP events on its stream."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import multigpu, rt, scenes  # noqa: E402

argv = sys.argv[1:]
WORLDS = [2, 4, 8]
if "--worlds" in argv:
    i = argv.index("--worlds")
    WORLDS = [int(x) for x in argv[i + 1].split(",")]
    del argv[i:i + 2]
FLAGS = 0
if "--flags" in argv:
    i = argv.index("--flags")
    FLAGS = int(argv[i + 1])
    del argv[i:i + 2]
HEAVY = 1e30
if "--heavy" in argv:
    i = argv.index("--heavy")
    HEAVY = float(argv[i + 1])
    del argv[i:i + 2]
SPLIT = "sample"
if "--split" in argv:
    i = argv.index("--split")
    SPLIT = argv[i + 1]
    del argv[i:i + 2]
TILES = "--tiles" in argv
CUT = "--cut" in argv
args = [a for a in argv if not a.startswith("--")]
BANDS = [int(x) for x in args[0].split(",")] if args else [multigpu.BAND]
CFG = args[1] if len(args) > 1 else "C3"
ORDERS = ((0, "schedule"), (rt.RENDER_ROWMAJOR, "row-major")) if not args and not TILES else ((FLAGS, "schedule"),)
cli, W, H, spp, seed = scenes.CONFIGS[CFG]
scenes.ensure_bun69k()
s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
s.build_photons(seed)


def time_plan(p, plan, iters=20, warm=3):
    import torch

    rgb = torch.empty((H * W, 3), dtype=torch.float32, device="cuda")
    argb = torch.empty((H * W,), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    for _ in range(warm):
        multigpu.render_plan(s, p, plan, rgb.data_ptr(), argb.data_ptr(), st, side)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        multigpu.render_plan(s, p, plan, rgb.data_ptr(), argb.data_ptr(), st, side)
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for flags, name in ORDERS:
    full = s.time_render(W, H, spp=spp, seed=seed, iters=5, flags=flags)
    print(CFG, name, "full %.3f ms" % full, flush=True)
    if TILES:
        p = rt.params(W, H, spp=spp, seed=seed, flags=flags)
        costs = s.tile_costs(p)
        for world in WORLDS:
            n, tx, tw, th = s.tile_layout(p)
            plans = multigpu.rank_plans(costs, world, tx, tw, th, W, H, mode="cut" if CUT else "deal",
                                        heavy=HEAVY, split=SPLIT)
            ts = [time_plan(p, pl) for pl in plans]
            print(" ", "cut" if CUT else "tiles", "heavy", HEAVY, SPLIT, "split px", sum(len(pl.pixels) for pl in plans), "N", world, "max %.3f mean %.3f ideal %.3f eff %.3f" % (
                max(ts), sum(ts) / len(ts), full / world, full / world / max(ts)),
                "per rank", " ".join("%.3f" % t for t in ts), flush=True)
        continue
    for band, world in [(b, w) for b in BANDS for w in WORLDS]:
        ts = []
        for rank in range(world):
            r0, r1, step, b = multigpu.rows_of(rank, world, H, band)
            ts.append(s.time_render(W, H, spp=spp, seed=seed, rows=(r0, r1), row_step=step, row_band=b,
                                    iters=5, flags=flags))
        print(" ", "band", band, "N", world, "max %.3f mean %.3f ideal %.3f eff %.3f" % (
            max(ts), sum(ts) / len(ts), full / world, full / world / max(ts)),
            "per rank", " ".join("%.3f" % t for t in ts), flush=True)
