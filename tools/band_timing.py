#!/usr/bin/env python3
"""Per-rank kernel time of the multi-GPU row-band partition, emulated on one GPU: max over
ranks vs full-frame/N (strong-scaling efficiency of the kernel alone), with the probed
longest-first tile schedule and with row-major dispatch."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import multigpu, rt, scenes  # noqa: E402

BANDS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [multigpu.BAND]
ORDERS = ((0, "schedule"), (rt.RENDER_ROWMAJOR, "row-major")) if len(sys.argv) <= 1 else ((0, "schedule"),)
CFG = sys.argv[2] if len(sys.argv) > 2 else "C3"  # tools/band_timing.py 8 C4
cli, W, H, spp, seed = scenes.CONFIGS[CFG]
scenes.ensure_bun69k()
s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
s.build_photons(seed)
for flags, name in ORDERS:
    full = s.time_render(W, H, spp=spp, seed=seed, iters=5, flags=flags)
    print(CFG, name, "full %.3f ms" % full)
    for band, world in [(b, w) for b in BANDS for w in (2, 4, 8)]:
        ts = []
        for rank in range(world):
            r0, r1, step, b = multigpu.rows_of(rank, world, H, band)
            ts.append(s.time_render(W, H, spp=spp, seed=seed, rows=(r0, r1), row_step=step, row_band=b,
                                    iters=5, flags=flags))
        print(" ", "band", band, "N", world, "max %.3f mean %.3f ideal %.3f eff %.3f" % (max(ts), sum(ts) / len(ts), full / world,
                                                                       full / world / max(ts)))
