#!/usr/bin/env python3
"""Where the level-synchronous path (RT_RENDER_WAVEFRONT) and the monolithic kernel differ."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

cli = sys.argv[1] if len(sys.argv) > 1 else "plnts3ColsBunnies.cli"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 96
SPPS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 4]
MODES = sys.argv[4].split(",") if len(sys.argv) > 4 else ["default", "nowavecull", "generic", "nocull"]
scenes.ensure_bun69k()
g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
for spp in SPPS:
    for extra, name in ((0, "default"), (rt.RENDER_NOWAVECULL, "nowavecull"), (rt.RENDER_GENERIC, "generic"),
                        (rt.RENDER_NOCULL, "nocull")):
        if name not in MODES:
            continue
        ra, aa = g.render(W, W, spp=spp, seed=0x5EED0001, flags=extra)
        rb, ab = g.render(W, W, spp=spp, seed=0x5EED0001, flags=extra | rt.RENDER_WAVEFRONT)
        d = np.abs(ra.astype(np.float64) - rb).max(-1)
        bad = np.argwhere(d > 0)
        rows = np.unique(bad[:, 0]) if len(bad) else []
        print(f"spp {spp} {name}: {len(bad)} pixels differ, max {d.max():.3g}", [tuple(int(v) for v in x) for x in bad[:8]],
              "rows", list(rows[:20]), flush=True)
