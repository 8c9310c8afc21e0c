#!/usr/bin/env python3
"""Photon-map build time, device (photon_build.hip) vs host (photon.cpp), on C5's photon list
(t11: 1 M diffuse photons per light) and on synthetic lists up to 80 M photons (t08's
caustic_photons count); checks the two structures are identical where the host build is run.

  python tools/photon_build_timing.py [--sizes 2000000,20000000,80000000] [--host-max 20000000]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import rt, scenes  # noqa: E402


def timed_set(cli, pos, pwr, mode):
    if mode == "host":
        os.environ["DISTRAYTRACER_PHOTON_BUILD"] = "host"
    else:
        os.environ.pop("DISTRAYTRACER_PHOTON_BUILD", None)
    s = rt.Scene.load_cli(cli, textures={})
    t0 = time.perf_counter()
    s.set_photons(pos, pwr)
    dt = time.perf_counter() - t0
    return s, dt


def same(a, b):
    return rt.photon_maps_equal(a, b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2000000,20000000,80000000")
    ap.add_argument("--host-max", type=int, default=20000000)
    a = ap.parse_args()
    cli = "t11.cli"
    s = rt.Scene.load_cli(cli, textures={})
    t0 = time.perf_counter()
    s.build_photons(0x5EED0005)
    t_full = time.perf_counter() - t0
    pos, pwr = s.photons()
    s.close()
    lists = [("C5 t11 photon_list", pos, pwr)]
    rng = np.random.default_rng(7)
    for n in [int(x) for x in a.sizes.split(",") if x]:
        lists.append((f"synthetic uniform {n}", rng.random((n, 3)) * 2 - 1, rng.random((n, 3))))
    print(json.dumps({"c5_prepass_s": t_full, "c5_photons": len(pos)}), flush=True)
    for name, p, w in lists:
        g, tg = timed_set(cli, p, w, "gpu")
        g2, tg2 = timed_set(cli, p, w, "gpu")  # warm (first build JITs nothing, but pages in)
        out = {"list": name, "photons": len(p), "gpu_build_s": min(tg, tg2)}
        g2.close()
        if len(p) <= a.host_max:
            h, th = timed_set(cli, p, w, "host")
            out["host_build_s"] = th
            out["identical"] = bool(same(g.photon_map(), h.photon_map()))
            h.close()
        g.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
