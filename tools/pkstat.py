#!/usr/bin/env python3
"""Packet-traversal lane utilisation (profiling build -DRT_PROF_PKSTAT, counting kernel):
wave steps of the packet traversals and the lanes that test in them.

  python tools/variant_sweep.py build --names pkstat     # here (CPU)
  DISTRAYTRACER_LIB=tools/_variants/lib_pkstat.so python tools/pkstat.py [C3] [W]
"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
cli, W, H, spp, seed = scenes.CONFIGS[cfg]
if len(sys.argv) > 2:
    W = H = int(sys.argv[2])
scenes.ensure_bun69k()
L = rt.lib()
buf = np.zeros(16, dtype=np.uint64)
with rt.Scene.load_cli(cli, textures=scenes.prepare(cli)) as s:
    s.build_photons(seed)
    L.rt_prof_pkstat_get(ctypes.c_void_p(buf.ctypes.data))  # clear
    _, _, st = s.render_count(W, H, spp=spp, seed=seed)
    assert L.rt_prof_pkstat_get(ctypes.c_void_p(buf.ctypes.data)) == 0
names = ["closest_box", "closest_tri", "any_box", "any_tri", "ray_calls", "shadow_calls",
         "closest_tri_hit", "any_tri_hit"]  # *_hit: wave steps with a hitting lane, the lanes that hit
out = {"cfg": cfg, "W": W, "H": H, "spp": spp, "counts": st}
for i, n in enumerate(names):
    steps, lanes = int(buf[2 * i]), int(buf[2 * i + 1])
    out[n] = {"wave_steps": steps, "lane_tests": lanes, "utilisation": lanes / max(1, 64 * steps)}
print(json.dumps(out))
