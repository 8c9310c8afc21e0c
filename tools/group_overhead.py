#!/usr/bin/env python3
"""Non-kernel cost of the native N-GPU step (rt_group_*, VERDICT r04 Next #1), measured on ONE GPU.

An N-rank RT_GROUP_COPY group with every rank on device 0 runs each rank's step alone
(rt_group_time_rank: its render, pack, copy into rank 0's receive slab and the scatter of its slice;
rank 0: its render and the whole scatter), frames pipelined as rt_group_render pipelines them.
Per rank: wall-clock ms per step and the mean HIP-event time of its render; the line reports
max_r(step) - max_r(kernel), the step's cost beyond its slowest rank's kernel.

  python tools/group_overhead.py [--config C3] [--world 8] [--iters 50] [--out file.json]
"""
import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rebalance", type=int, default=0, help="rt_group_rebalance rounds before timing")
    ap.add_argument("--heavy", type=float, default=0.0, help="plan: split tiles above heavy x a slot's share (0: 1.25)")
    ap.add_argument("--slots", type=int, default=0, help="plan: wave slots per rank (0: 4096)")
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)

    from distraytracer_old_amd import rt, scenes

    cli, W, H, spp, seed = scenes.CONFIGS[a.config]
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    if g.info()["photon_mode"]:
        g.build_photons(seed)
    full = g.time_render(W, H, spp=spp, seed=seed, warmup=2, iters=5)
    rows = []
    with rt.Group.create([g] * a.world, W, H, spp=spp, seed=seed, copy=True, heavy=a.heavy, slots=a.slots) as grp:
        if a.rebalance:
            ms = grp.rebalance(rounds=a.rebalance, iters=10)
            print(json.dumps({"rebalanced_rank_ms": ms.tolist()}), flush=True)
        for r in range(a.world):
            run, split = grp.rank_tiles(r)
            step, kern = grp.time_rank(r, warmup=a.warmup, iters=a.iters)
            rows.append({"rank": r, "tiles": int(len(run)), "split_tiles": int(len(split)),
                         "pixels": int(len(grp.rank_pixels(r))), "step_ms": step, "kernel_ms": kern,
                         "overhead_us": (step - kern) * 1e3})
            print(json.dumps(rows[-1]), flush=True)
    smax = max(x["step_ms"] for x in rows)
    kmax = max(x["kernel_ms"] for x in rows)
    out = {"config": a.config, "workload": f"{cli} {W}x{H} {spp}spp", "world": a.world, "iters": a.iters,
           "rebalance_rounds": a.rebalance, "heavy": a.heavy or 1.25, "slots": a.slots or 4096,
           "full_frame_kernel_ms": full, "max_step_ms": smax, "max_kernel_ms": kmax,
           "step_minus_kernel_us": (smax - kmax) * 1e3,
           "emulated_efficiency": full / a.world / smax, "kernel_efficiency": full / a.world / kmax,
           "build_id": rt.build_id(), "ranks": rows}
    print(json.dumps({k: v for k, v in out.items() if k != "ranks"}), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    g.close()


if __name__ == "__main__":
    main()
