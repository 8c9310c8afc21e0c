#!/usr/bin/env python3
"""bench.py's N-rank step path, run for a check: every rank renders its cost-balanced tiles
(--partition tiles: rt_render_tiles_device) or row bands (bands: rt_render_device) with the HIP
kernel (multigpu.RankRenderer), the photon pre-pass (photon scenes) is
sharded over the ranks (multigpu.build_photons_sharded), the float-RGB and ARGB tiles go through
multigpu.FrameExchange to rank 0, and rank 0 writes the assembled frame to --out (.npz: rgb, argb).

Launched under torch.distributed.run; with --backend gloo the ranks may share one GPU (tiles
staged to host), which is how tests/test_rank_path.py runs it on a one-GPU box. Without
WORLD_SIZE it runs as a single rank (no exchange): the 1-GPU image to compare against.
"""
import argparse
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cli", default="c3_bun69k.cli")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0x5EED0001)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"])
    ap.add_argument("--partition", default="tiles", choices=["tiles", "bands"])
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import numpy as np
    import torch

    from distraytracer_old_amd import multigpu, rt, scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    scenes.ensure_bun69k()
    scene = rt.Scene.load_cli(a.cli, textures=scenes.prepare(a.cli), device=dev)
    info = scene.info()
    if info["photon_mode"]:
        multigpu.build_photons_sharded(scene, a.seed, info["photon_count"], dist,
                                       device="cuda" if a.backend == "nccl" else "cpu")
    rr = multigpu.RankRenderer(scene, a.size, a.size, a.spp, a.seed, dist, stage_host=(a.backend == "gloo"),
                               partition=a.partition)
    rr.calibrate()
    frames = []
    for _ in range(a.frames):
        rr.step()
        ex = rr.ex.get("rgb") if rr.ex else None
        if ex is not None and rr.rank == 0 and ex.frame > 1:  # the previous frame, assembled
            frames.append((ex.image.cpu().numpy().reshape(a.size, a.size, 3).copy(),
                           rr.ex["argb"].image.cpu().numpy().reshape(a.size, a.size).copy()))
    rgb, argb = rr.finish()
    torch.cuda.synchronize()
    if rr.rank == 0:
        rgb, argb = rgb.cpu().numpy(), argb.cpu().numpy()
        for f, fa in frames:  # every pipelined frame was delivered whole (same seed: same image)
            assert np.array_equal(f, rgb) and np.array_equal(fa, argb), "a pipelined frame differs from the last"
        np.savez(a.out, rgb=rgb, argb=argb)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    scene.close()


if __name__ == "__main__":
    main()
