#!/usr/bin/env python3
"""The slowest wave tiles of a config's frame (the multi-GPU tail: a rank's launch cannot end
before its longest wave): measured wave times of the whole-frame layout (rt_tile_costs, 10 ns
ticks of s_memrealtime), their distribution, the slowest tiles' pixels, and each one's counted
work (rt_render_tiles_count on that tile alone).

  python tools/slow_tiles.py C5 [TOP]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

CFG = sys.argv[1] if len(sys.argv) > 1 else "C5"
TOP = int(sys.argv[2]) if len(sys.argv) > 2 else 12
FLAGS = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cli, W, H, spp, seed = scenes.CONFIGS[CFG]
scenes.ensure_bun69k()
s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
s.build_photons(seed)
p = rt.params(W, H, spp=spp, seed=seed, flags=FLAGS)
n, tx, tw, th = s.tile_layout(p)
c = s.tile_costs(p).astype(np.float64) * 0.01  # us
print(f"{CFG}: {n} tiles of {tw}x{th} px; wave time us: mean {c.mean():.1f} p50 {np.median(c):.1f} "
      f"p99 {np.percentile(c, 99):.1f} p99.9 {np.percentile(c, 99.9):.1f} max {c.max():.1f}; sum/1024 slots "
      f"{c.sum() / 1024 / 1e3:.2f} ms")
order = np.argsort(-c, kind="stable")
print("top tiles (us, tile, first pixel (row, col), counters):")
for t in order[:TOP]:
    st = s.render_tiles_count(p, np.array([t], dtype=np.int32))
    keep = {k: v for k, v in st.items() if v}
    print(f"  {c[t]:9.1f} tile {t} px ({(t // tx) * th}, {(t % tx) * tw}) {keep}", flush=True)
med = order[len(order) // 2]
st = s.render_tiles_count(p, np.array([med], dtype=np.int32))
print(f"  median tile {med} ({c[med]:.1f} us):", {k: v for k, v in st.items() if v})
