#!/usr/bin/env python3
"""Workgroup timeline of the render kernel (profiling build with -DRT_PROF_TIMELINE):
per workgroup start / end (s_memrealtime, 100 MHz), HW_ID and XCC_ID, for the full C3
frame and for each rank's rows of an N-GPU band split (emulated on one GPU).

  python tools/variant_sweep.py build --names tl      # here (CPU)
  DISTRAYTRACER_LIB=tools/_variants/lib_tl.so python tools/timeline.py [--world 8] [--out f.npz]

Prints per launch: span, wave-duration percentiles, the time until the machine is
full, the tail (time from the last dispatch to the end), and busy slots over time.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import multigpu, rt, scenes  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def run(scene, torch, W, H, spp, seed, rows, step, band, flags=0):
    p = rt.params(W, H, spp=spp, seed=seed, rows=rows, row_step=step, row_band=band, flags=flags)
    n = rt.nrows_of(p)
    rgb = torch.empty((n, W, 3), dtype=torch.float32, device="cuda")
    argb = torch.empty((n, W), dtype=torch.int32, device="cuda")
    nblk = W * n + 64  # >= tiles of any wave layout
    buf = torch.zeros((nblk, 4), dtype=torch.int64, device="cuda")
    L = rt.lib()
    L.rt_prof_timeline_set.argtypes = [ctypes.c_void_p]
    scene.render_device(p, rgb.data_ptr(), argb.data_ptr(), 0)  # warm (schedule probe)
    torch.cuda.synchronize()
    assert L.rt_prof_timeline_set(ctypes.c_void_p(buf.data_ptr())) == 0
    scene.render_device(p, rgb.data_ptr(), argb.data_ptr(), 0)
    torch.cuda.synchronize()
    assert L.rt_prof_timeline_set(ctypes.c_void_p(0)) == 0
    b = buf.cpu().numpy()
    b = b[b[:, 1] != 0]
    return b


def summarize(b, name):
    t0, t1 = b[:, 0].astype(np.float64), b[:, 1].astype(np.float64)
    base = t0.min()
    s, e = (t0 - base) * TICK_US, (t1 - base) * TICK_US
    d = e - s
    span = e.max()
    hw = b[:, 2]
    xcc = b[:, 3] & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    slots = len(np.unique(np.stack([xcc, se, cu, simd], 1), axis=0))
    last_start = s.max()
    # busy lanes over time (20 bins)
    edges = np.linspace(0, span, 21)
    busy = [(np.minimum(e, edges[i + 1]) - np.maximum(s, edges[i])).clip(0).sum() / (edges[i + 1] - edges[i])
            for i in range(20)]
    peak = max(busy)
    area = d.sum()
    out = {"launch": name, "blocks": int(len(b)), "span_us": round(span, 1),
           "dur_us": {q: round(float(np.percentile(d, q)), 1) for q in (10, 50, 90, 99, 100)},
           "mean_dur_us": round(float(d.mean()), 1),
           "simd_slots": int(slots), "peak_concurrency": round(peak, 1),
           "fill_us": round(float(np.sort(s)[min(len(s) - 1, int(peak) - 1)]), 1),
           "last_start_us": round(float(last_start), 1), "tail_us": round(float(span - last_start), 1),
           "efficiency": round(float(area / (peak * span)), 3),
           "busy": [round(x / peak, 2) for x in busy],
           "xcc_end_us": [round(float(e[xcc == x].max()), 1) for x in range(8) if (xcc == x).any()]}
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="C3")
    ap.add_argument("--world", default="1,8")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    cli, W, H, spp, seed = scenes.CONFIGS[a.cfg]
    scenes.ensure_bun69k()
    raw = {}
    with rt.Scene.load_cli(cli, textures=scenes.prepare(cli)) as sc:
        for world in [int(x) for x in a.world.split(",")]:
            for rank in range(world if world > 1 else 1):
                r0, r1, step, band = multigpu.rows_of(rank, world, H)
                b = run(sc, torch, W, H, spp, seed, (r0, r1), step, band, a.flags)
                summarize(b, f"N={world} rank {rank}")
                raw[f"w{world}r{rank}"] = b
    if a.out:
        np.savez_compressed(a.out, **raw)


if __name__ == "__main__":
    main()
