#!/usr/bin/env python3
"""Kernel tuning sweep: build the library with different compile-time settings
(here, on CPU) and time each on the GPU box, one subprocess per build.

  python tools/variant_sweep.py build            # -> tools/_variants/*.so
  python tools/variant_sweep.py run [--cfg C3]   # on the GPU: ms/frame + ARGB hash per build

Every build must give the same ARGB hash (the specialisations change speed, not results).
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
OUT = REPO / "tools" / "_variants"
VARIANTS = {  # name -> -D defines; names like "s12w4" are parsed (see defines_of)
    "noshadow": ["RT_PROF_NOSHADOW"],          # profiling only: results differ
    "nosec": ["RT_PROF_NOSECONDARY"],
    "primary": ["RT_PROF_NOSHADOW", "RT_PROF_NOSECONDARY"],
    "nogather": ["RT_PROF_NOGATHER"],
    "knnheap": ["RT_KNN_HEAP"],
    "nophong": ["RT_PROF_NOPHONG"],
    "notex": ["RT_PROF_NOTEX"],                # object textures -> plain diffuse
    "noshade": ["RT_PROF_NOSHADE"],            # camera rays traced, no hit record / shading
    "notrace": ["RT_PROF_NOTRACE"],            # camera rays generated, nothing traced
    "wprio": ["-Xarch_device", "-mllvm=--amdgpu-set-wave-priority"],  # compiler flags (results equal)
    "itsched": ["-Xarch_device", "-mllvm=--amdgpu-sched-strategy=gcn-iterative-max-occupancy-experimental"],
    "bias0": ["-Xarch_device", "-mllvm=--amdgpu-schedule-metric-bias=0"],
    "trk": ["-Xarch_device", "-mllvm=--amdgpu-use-amdgpu-trackers=1"],
    # scheduler of trace.hip only (C4's variant and the others; C3 / C5 are in render_minreg.hip)
    "mrnohrp": ["@render_minreg.hip:-Xarch_device", "@render_minreg.hip:-mllvm=--amdgpu-disable-unclustered-high-rp-reschedule=1"],
    "mrbias0": ["@render_minreg.hip:-Xarch_device", "@render_minreg.hip:-mllvm=--amdgpu-schedule-metric-bias=0"],
    "c4ilp": ["@trace.hip:-Xarch_device", "@trace.hip:-mllvm=--amdgpu-sched-strategy=max-ilp"],
    "c4mmc": ["@trace.hip:-Xarch_device", "@trace.hip:-mllvm=--amdgpu-sched-strategy=max-memory-clause"],
    "c4itilp": ["@trace.hip:-Xarch_device", "@trace.hip:-mllvm=--amdgpu-sched-strategy=iterative-ilp"],
    "minreg": ["-Xarch_device", "-mllvm=--amdgpu-sched-strategy=iterative-minreg"],
    "trkminreg": ["-Xarch_device", "-mllvm=--amdgpu-use-amdgpu-trackers=1", "-Xarch_device",
                  "-mllvm=--amdgpu-sched-strategy=iterative-minreg"],
    "ed8": [],
    "ed16": ["RT_KNN_EDGES=16"],
    "ed32": ["RT_KNN_EDGES=32"],
    "ed16sh12": ["RT_KNN_EDGES=16", "RT_KNN_SHELL=12"],
    "hist0": ["RT_KNN_LDS_HIST=0"],            # kNN counting in registers (results equal)
    "h32b2": ["RT_KNN_EDGES=32", "RT_PH_BATCH=2"],
    "h32sh12": ["RT_KNN_EDGES=32", "RT_KNN_SHELL=12"],
    "sh10": ["RT_KNN_SHELL=10"],               # window list in LDS: up to 10 photons
    "h32": ["RT_KNN_EDGES=32"],
    "h32sh10": ["RT_KNN_EDGES=32", "RT_KNN_SHELL=10"],
    "h64": ["RT_KNN_H16=1"],                   # 64 u16 LDS buckets per counting pass
    "h64s10": ["RT_KNN_H16=1", "RT_KNN_SHELL=10"],
    "vl": ["RT_PH_VLOAD=1"],                   # leaf photons: vector load + v_readlane
    "vl2": ["RT_PH_VLOAD=2"],                  # ... two independent distances per step
    "vl4": ["RT_PH_VLOAD=4"],
    "h64s10reg": ["RT_KNN_H16=1", "RT_KNN_SHELL=10", "RT_PROF_REGIONS"],
    "tl": ["RT_PROF_TIMELINE"],               # workgroup timeline (tools/timeline.py)
    "pkstat": ["RT_PROF_PKSTAT"],             # packet lane utilisation (tools/pkstat.py)
    "shnoquad": ["RT_PROF_SH_NOQUAD"],         # shadow scan without quads / planes
    "shnoimpl": ["RT_PROF_SH_NOIMPL"],         # shadow scan without implicit primitives
    "shnoaccel": ["RT_PROF_SH_NOACCEL"],       # shadow scan without BVHs / lists
    "shinline": ["RT_SHADOW_NOINLINE"],        # shadow scan as a real call (results equal)
    "shscan": ["RT_PROF_SH_SCANONLY"],         # shadow rays: the top-level scan only, no tests
    "shnoacc": ["RT_PROF_SH_NOACCEL"],         # shadow rays: no BVH / list entries
    "regions": ["RT_PROF_REGIONS"],           # wave time per region (tools/regions.py)
    "nf0": ["RT_NEAREST_FIRST=0"],             # closest hit in the reference order only (round 2)
    "nf1": [],                                 # nearest-first closest hit where it applies (default)
    "nopio": ["RT_JF_NPIO2=0"],                # rem_pio2 without e_rem_pio2.c's npio2_hw shortcut
    "an0": ["RT_ANY_NEAR=0"],
    "wc0": ["RT_WAVE_CULL=0"],                 # no wave-level shadow candidates (the r03l kernel)
    "wc1": [],                                 # wave-level shadow candidates per shading step (default)
    "base": [],                                # the default build
    "wp1": [],                                 # the default build (+ quad / plane sides in the wave cull)
    "wtri": ["RT_WC_TRI=1"],                   # the wave cull in the triangles-only variant (C3) too
    "nft": ["RT_NF_TRANS=1"],                  # nearest-first closest hit in C4's transparent variant
    "ant": ["RT_AN_TRANS=1"],                  # nearest-first any-hit order there
    "nftant": ["RT_NF_TRANS=1", "RT_AN_TRANS=1"],
    "nfan0": ["RT_NEAREST_FIRST=0", "RT_ANY_NEAR=0"],
    "ld8": ["RT_LANE_DIV=8"],                  # divergent waves: per-lane BVH traversal (closest hit)
    "ld16": ["RT_LANE_DIV=16"],
    "ld32": ["RT_LANE_DIV=32"],
    "ld16c99": ["RT_LANE_DIV=16", "RT_LANE_DIV_COS=0.99"],
    "kd1": ["RT_KNN_DIV=1"],                   # ... when half of the call's lanes are far apart
    "ld1": ["RT_LANE_DIV=1"],
    "nfcode": ["RT_NF_CODE=1"],
    "kd1f4": ["RT_KNN_DIV=1", "RT_KNN_DIV_FRAC=4"],
    "kd1f1": ["RT_KNN_DIV=1", "RT_KNN_DIV_FRAC=1"],
    "kd1r4": ["RT_KNN_DIV=1", "RT_KNN_DIV_R=4.0"],
    "kd1r1": ["RT_KNN_DIV=1", "RT_KNN_DIV_R=1.0"],
    "kd8": ["RT_KNN_DIV=8"],                   # divergent query points: per-lane photon scans
    "kd16": ["RT_KNN_DIV=16"],
    "kd32": ["RT_KNN_DIV=32"],
    "wf5": ["RT_WF_WAVES=5"],                  # level-synchronous kernels at 5 / 3 waves per SIMD
    "wf3": ["RT_WF_WAVES=3"],
    "head": [],                                # a copy of the in-tree library (the A of an A/B)
    "flate": [],                               # shade_node's local colour stored into the frame only when it pushes
    "reslds": [],                              # a finished sample's colour waits in LDS, not in spilled VGPRs
    "reslds0": ["RT_RES_LDS=0"],
    "inner0": ["RT_KNN_INNER=0"],             # the kNN final pass scans every photon below the window (round 4)
    "sprim0": ["RT_SPRIM=0"],                 # top-level implicit primitives as vector loads (round 4)
    "sprim1": ["RT_SPRIM=1"],                 # ... as scalar loads in the variants without a photon map
    "sprim2": ["RT_SPRIM=2"],                 # ... in every variant
    "uload0": ["RT_ULOAD=0"],                 # leaf transforms / light fields as per-lane loads
    "uload1": ["RT_ULOAD=1"],                 # the leaf member's transform inverse as scalar loads
    "uload2": ["RT_ULOAD=2"],                 # the light's spot / disk fields as scalar loads
    "uload3": ["RT_ULOAD=3"],
    "ex0": ["RT_KNN_EXTRAP=0"],               # kNN start window too small: widen to the node's far corner
    "ex1": ["RT_KNN_EXTRAP=1"],               # ... to the density extrapolation, above the counted photons
    "ex1s115": ["RT_KNN_EXTRAP=1", "RT_KNN_START=1.15"],
    "ex1s10": ["RT_KNN_EXTRAP=1", "RT_KNN_START=1.0"],
    "ex1s11": ["RT_KNN_EXTRAP=1", "RT_KNN_START=1.1"],
    "ex1s12": ["RT_KNN_EXTRAP=1", "RT_KNN_START=1.2"],
    "ex1s125": ["RT_KNN_EXTRAP=1", "RT_KNN_START=1.25"],
    "h8off": ["RT_KNN_H8=0"],                 # kNN counting: 64 u16 LDS buckets (round 2)
    "h8on": ["RT_KNN_H8=1"],                  # 128 u8 buckets, u16 pass on a carry
    "h8s12": ["RT_KNN_H8=1", "RT_KNN_START=1.2"],
    "h8s13": ["RT_KNN_H8=1", "RT_KNN_START=1.3"],
    "slim0": ["RT_FRAME_SLIM=0"],             # shading-tree frames with every field (round 4)
    "slim1": ["RT_FRAME_SLIM=1"],             # ... without the fields derivable at the fold
    "xh0": ["RT_XCD_HASH=0"],                 # longest-first tile order, blocks dealt to XCDs as they come
    "xh2": ["RT_XCD_HASH=2"],                 # 2x2-tile superblocks hashed to one XCD's list
    "xh4": ["RT_XCD_HASH=4"],
    "xh8": ["RT_XCD_HASH=8"],
    "sc0": ["RT_SLAB_CALL=0"],                # exact slab fallback inlined in the traversal loops
    "sc1": ["RT_SLAB_CALL=1"],                # ... as a real call
    "apx0": ["RT_APX2=0"],                    # approximate box test returning a tri-state int
    "apx1": ["RT_APX2=1"],                    # ... as two lane masks (settled, hit)
    "ib0": ["RT_INV_BALLOT=0"],               # a lane's bit of a wave mask by shift and compare
    "ib1": ["RT_INV_BALLOT=1"],               # ... by inverse ballot (the mask as exec)
    "ib1apx1": ["RT_INV_BALLOT=1", "RT_APX2=1"],
    "mo0": ["RT_MASKOPS=0"],                  # packet lane bits by shift, tri-state approximate box tests
    "mo1": ["RT_MASKOPS=1"],                  # inverse ballot + lane-mask box tests in opaque variants (default)
    "tl0": [],                                # (the default build)
    "tlsum": ["RT_SUMS_LDS_TRANS=1"],         # per-pixel sums in LDS in the transparent variants
    "tlres": ["RT_RES_LDS_TRANS=1"],          # finished colours in LDS in the transparent variants
    "tlboth": ["RT_SUMS_LDS_TRANS=1", "RT_RES_LDS_TRANS=1"],
    "fin": [],                                # the final build's settings (A of the last A/Bs)
    "mo2": ["RT_MASKOPS=2"],                  # mask ops in every variant
    "mo2xh4": ["RT_MASKOPS=2", "RT_XCD_HASH=4"],
    "lb0": ["RT_NF_LB=0"],                    # nearest-first: grown-box entry by its own slab computation
    "lb1": ["RT_NF_LB=1"],                    # ... as a lower bound from the exact box's slab values
    "kd0": ["RT_KNN_DIV=0"],                  # kNN scans as packets only
    "uo0": ["RT_UNI_OPAQUE=0"],               # uniform values hoisted (and spilled) out of the sample loop (round 5)
    "uo1": [],                                # ... made opaque where used (uni_here, default)
    "f320": ["RT_F32_BOX=0"],                 # box tests in fp64 only (round 5)
    "f32nf": ["RT_F32_SHADOW=0"],             # fp32 box pre-test in the nearest-first closest hit only
    "f32all": ["RT_F32_SHADOW_OPAQUE=1"],     # ... and in every variant's shadow traversal
    "f32def": [],                             # ... in the transparent variants' shadow traversal (default)
    "f32nt": ["RT_F32_SHADOW_TRANS=0"],       # ... but not in the transparent variants' shadow traversal
    "lz0": ["RT_F32_SH_LAZY=0"],              # shadow fp32 pre-test with the fp32 ray held through the traversal
    "lz": [],                                 # ... rebuilt per node from the fp64 ray (default)
    "lzop": ["RT_F32_SHADOW_OPAQUE=1"],       # ... and in the opaque variants' (C3's) shadow traversal too
    "cpk0": ["RT_F32_CPK=0"],                 # reference-order closest hit (transparent variants): fp64 box tests
    "cpk": [],                                # ... with the fp32 pre-test (default)
    "cpkph0": ["RT_F32_CPK_PHOTON=0"],        # ... but not in the photon-map variant
    "tri0": ["RT_F32_TRI=0"],                 # no fp32 triangle edge pre-test
    "tricpk0": ["RT_F32_TRI_CPK=0"],          # ... none in the reference-order closest hit
    "tph01": ["RT_F32_TRI_PH_ANY=0", "RT_F32_TRI_PH_CPK=1"],  # photon variant: the triangle pre-test in its closest hit
    "tph11": ["RT_F32_TRI_PH_ANY=1", "RT_F32_TRI_PH_CPK=1"],  # ... in both traversals
    "nosample": ["RT_PROF_NOSAMPLE"],         # camera setup, sums and output alone (results differ)
    "pers": ["RT_PERSIST=1"],                 # persistent render launches: resident grid, tiles from a ticket counter
    "c4mr": ["@trace.hip:-Xarch_device", "@trace.hip:-mllvm=--amdgpu-sched-strategy=iterative-minreg",
             "@trace.hip:-Xarch_device", "@trace.hip:-mllvm=--amdgpu-use-amdgpu-trackers=1"],
}
FIELDS = {"w": "RT_RENDER_WAVES", "s": "RT_STACK_LDS", "x": "RT_XCD_CHUNKS", "g": "RT_MAX_G", "p": "RT_PACKET",
          "l": "RT_PK_LDS", "b": "RT_PH_BATCH", "m": "RT_PK_MASKED"}


def defines_of(name: str) -> list[str]:
    import re
    if name in VARIANTS:
        return VARIANTS[name]
    return [f"{FIELDS[k]}={v}" for k, v in re.findall(r"([a-z])(\d+)", name)]


def _build_one(n):
    from distraytracer_old_amd import build
    p = build.build(defines=defines_of(n), out=OUT / f"lib_{n}.so")
    for o in OUT.glob(f"lib_{n}.*.o"):
        o.unlink()
    return p


def do_build(names):
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(max_workers=4) as ex:
        for p in ex.map(_build_one, names):
            print("built", p, flush=True)


def time_one(cfg: str, W: int, H: int, spp: int, iters: int, flags: int, save: str = ""):
    from distraytracer_old_amd import rt, scenes
    cli, W0, H0, spp0, seed = scenes.CONFIGS[cfg]
    scenes.ensure_bun69k()
    with rt.Scene.load_cli(cli, textures=scenes.prepare(cli)) as s:
        W = W or W0; H = H or H0; spp = spp or spp0
        rgb, argb = s.render(W, H, spp=spp, seed=seed, flags=flags)
        if save:  # the frame, to compare builds whose images may differ in the last bits
            import numpy as np
            np.savez_compressed(save, rgb=rgb, argb=argb)
        ms = s.time_render(W, H, spp=spp, seed=seed, warmup=1, iters=iters, flags=flags)
    return {"ms": ms, "hash": hashlib.sha1(argb.tobytes()).hexdigest()[:12], "W": W, "H": H, "spp": spp}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run", "one"])
    ap.add_argument("--cfg", default="C3")
    ap.add_argument("--names", default="w4,w5")
    ap.add_argument("--W", type=int, default=0)
    ap.add_argument("--H", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--dir", default="", help="run: where the built libraries are (default tools/_variants)")
    ap.add_argument("--save", default="", help="directory: each build's frame as <name>_<cfg>.npz")
    a = ap.parse_args()
    names = a.names.split(",")
    if a.mode == "build":
        do_build(names)
    elif a.mode == "one":
        print(json.dumps(time_one(a.cfg, a.W, a.H, a.spp, a.iters, a.flags, a.save)))
    else:
        for n in names:
            lib = (Path(a.dir) if a.dir else OUT) / f"lib_{n}.so"
            env = dict(os.environ, DISTRAYTRACER_LIB=str(lib))
            cmd = [sys.executable, __file__, "one", "--cfg", a.cfg, "--W", str(a.W), "--H", str(a.H), "--spp", str(a.spp),
                   "--iters", str(a.iters), "--flags", str(a.flags)]
            if a.save:
                os.makedirs(a.save, exist_ok=True)
                cmd += ["--save", os.path.join(a.save, f"{n}_{a.cfg}.npz")]
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
            line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-800:]
            print(n, a.cfg, line, flush=True)
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
