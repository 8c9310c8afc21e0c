#!/usr/bin/env python3
"""Render a config's frame K times (for a PMC pass that sums every kernel of a frame, e.g. the
level-synchronous path's many launches): python tools/frame_runner.py CFG K FLAGS"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

cfg, k, flags = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cli, W, H, spp, seed = scenes.CONFIGS[cfg]
scenes.ensure_bun69k()
s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
s.build_photons(seed)
for _ in range(k):
    s.render(W, H, spp=spp, seed=seed, flags=flags)
print("rendered", k)
