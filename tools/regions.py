#!/usr/bin/env python3
"""Where a wave's time goes, by region (profiling build -DRT_PROF_REGIONS: shader-clock cycles
per region instance, summed over waves; the timed production kernel, not the counting one).

  python tools/variant_sweep.py build --names regions                     # here (CPU)
  DISTRAYTRACER_LIB=tools/_variants/lib_regions.so python tools/regions.py [C4] [W]
Shares are of the summed wave time (R_KERNEL); inner regions are subtracted from outer ones.
"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402

R = ["closest", "closest_accel", "shadow", "shadow_accel", "hit", "tex", "light", "shade", "sample", "kernel",
     "bg", "photon", "knn_count", "knn_final", "knn_npass", "knn_ncall"]
cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
cli, W, H, spp, seed = scenes.CONFIGS[cfg]
if len(sys.argv) > 2:
    W = H = int(sys.argv[2])
scenes.ensure_bun69k()
L = rt.lib()
buf = np.zeros(16, dtype=np.uint64)
with rt.Scene.load_cli(cli, textures=scenes.prepare(cli)) as s:
    s.build_photons(seed)
    for _ in range(2):  # tile-order calibration renders
        s.render(W, H, spp=spp, seed=seed)
    assert L.rt_prof_regions_get(ctypes.c_void_p(buf.ctypes.data)) == 0  # clear
    s.render(W, H, spp=spp, seed=seed)
    assert L.rt_prof_regions_get(ctypes.c_void_p(buf.ctypes.data)) == 0
c = {n: float(buf[i]) for i, n in enumerate(R)}
k = max(1.0, c["kernel"])
parts = {
    "camera setup / sums / output": c["kernel"] - c["sample"],
    "closest: top-level loop": c["closest"] - c["closest_accel"],
    "closest: BVH traversal": c["closest_accel"],
    "hit record": c["hit"],
    "texture": c["tex"],
    "photon gather": c["photon"],
    "  of it: kNN counting passes": c["knn_count"],
    "  of it: kNN final pass": c["knn_final"],
    "lights: shading (excl. shadow rays)": c["light"] - c["shadow"],
    "shadow: top-level loop": c["shadow"] - c["shadow_accel"],
    "shadow: BVH traversal": c["shadow_accel"],
    "shade: rest (children, Fresnel)": c["shade"] - c["tex"] - c["light"] - c["photon"],
    "background": c["bg"],
    "trace tree: rest (frames)": c["sample"] - c["closest"] - c["hit"] - c["shade"] - c["bg"],
}
knn = {"passes_per_call": c["knn_npass"] / max(1.0, c["knn_ncall"]), "calls": c["knn_ncall"]}
print(json.dumps({"cfg": cfg, "W": W, "H": H, "spp": spp, "raw": c, "knn_wave": knn,
                  "share": {n: round(v / k, 4) for n, v in parts.items()}}, indent=1))
