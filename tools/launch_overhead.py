#!/usr/bin/env python3
"""Kernel time vs image size (fixed per-launch cost vs per-pixel cost) for C3."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

scenes.ensure_bun69k()
s = rt.Scene.load_cli("c3_bun69k.cli", textures=scenes.prepare("c3_bun69k.cli"))
for rows in ((0, 8), (0, 64), (448, 576), (0, 128), (0, 256), (0, 512), (0, 1024)):
    ms = s.time_render(1024, 1024, spp=16, seed=0x5EED0001, rows=rows, iters=5)
    print(rows, "%.3f ms" % ms, "%.2f us/row" % (ms * 1e3 / (rows[1] - rows[0])))
