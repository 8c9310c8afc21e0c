#!/usr/bin/env python3
"""Time every SURVEY 8(d) config on one GPU (rt_time_render) with exact ray counts.

  python tools/bench_configs.py [C2,C3,C4,C5] [--iters N]
Prints one JSON line per config: ms/frame, Mray/s, bytes/ray (SURVEY 8(d) formula),
achieved GB/s, photon pre-pass time.
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from bench import algorithmic_bytes, traced_rays  # noqa: E402
from distraytracer_old_amd import rt, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="?", default="C2,C3,C4,C5")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    scenes.ensure_bun69k()
    for cfg in a.configs.split(","):
        cli, W, H, spp, seed = scenes.CONFIGS[cfg]
        t0 = time.perf_counter()
        s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
        t_load = time.perf_counter() - t0
        t0 = time.perf_counter()
        s.build_photons(seed)
        t_ph = time.perf_counter() - t0
        _, _, st = s.render_count(W, H, spp=spp, seed=seed)
        ms = s.time_render(W, H, spp=spp, seed=seed, warmup=1, iters=a.iters)
        rays = traced_rays(st)
        b = algorithmic_bytes(st)
        print(json.dumps({"config": cfg, "cli": cli, "W": W, "H": H, "spp": spp, "ms": ms,
                          "mray_s": rays / ms / 1e3, "rays": rays, "bytes_per_ray": b / rays,
                          "achieved_gbps": b / ms / 1e6, "load_s": t_load, "photons_s": t_ph,
                          "photons": s.info().get("photons"), "counts": st}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
