#!/usr/bin/env python3
"""Instrumented counters + image hash of one config (for A/B checks of kernel builds:
DISTRAYTRACER_LIB=tools/_variants/lib_X.so python tools/count_check.py C3 256)."""
import hashlib
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
cli, W, H, spp, seed = scenes.CONFIGS[cfg]
if len(sys.argv) > 2:
    W = H = int(sys.argv[2])
scenes.ensure_bun69k()
with rt.Scene.load_cli(cli, textures=scenes.prepare(cli)) as s:
    s.build_photons(seed)
    rgb, argb, st = s.render_count(W, H, spp=spp, seed=seed)
    _, argb2 = s.render(W, H, spp=spp, seed=seed)
print(json.dumps({"cfg": cfg, "W": W, "hash": hashlib.sha1(argb.tobytes()).hexdigest()[:12],
                  "hash_plain": hashlib.sha1(argb2.tobytes()).hexdigest()[:12], "counts": st}))
