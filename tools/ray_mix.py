#!/usr/bin/env python3
"""Counted work of a config's frame (instrumented render at a reduced size): rays by kind, per
camera sample, and the record tests -- the shading-tree shape a level-synchronous split would see.
  python tools/ray_mix.py C4 [W]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
cli, W, H, spp, seed = scenes.CONFIGS[cfg]
w = int(sys.argv[2]) if len(sys.argv) > 2 else 512
scenes.ensure_bun69k()
s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
s.build_photons(seed)
_, _, st = s.render_count(w, w * H // W, spp=spp, seed=seed)
cam = st["camera"]
print(cfg, f"{w}x{w * H // W} {spp}spp", {k: v for k, v in st.items() if v and not k.startswith("w_")})
print("per camera sample:", {k: round(st[k] / cam, 3) for k in ("shadow", "refl", "refr", "tri", "quad", "implicit", "light")})
