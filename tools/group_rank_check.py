#!/usr/bin/env python3
"""The native one-process-per-GPU group (rt_group_create_comm, csrc/group.hip) run as N real ranks
(VERDICT r05 Next #1): launched under torch.distributed.run, every rank

  * builds the photon map sharded over the ranks (rt_photons_build_comm, photon scenes) -- rank 0
    checks the photon_list and the device map against its own unsharded rt_photons_build;
  * creates its rank of the group over a communicator: --transport host (rt_comm_create_host over
    torch.distributed gloo; ranks may share device 0, which is how a one-GPU box runs it) or rccl
    (rt_comm_create_rccl; one device per rank) -- the cost broadcast, the argument and plan checks;
  * re-cuts the plan from the ranks' measured render times (rt_group_rebalance: the all-gather of
    {status, time} and a plan check after every cut);
  * renders frames: blocking ones into host buffers (rt_group_render_host, the JNI draw() over N
    GPUs) and pipelined ones into device buffers (rt_group_render without a sync between them).

Rank 0 compares every frame with rt_render of the same scene bit for bit (ARGB ints and the float
RGB plane) and writes a JSON report to --out. --mismatch makes the last rank pass a different `heavy`
(the ranks must all fail with RTError, not hang).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cli", default="c3_bun69k.cli")
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0x5EED0001)
    ap.add_argument("--transport", default="host", choices=["host", "rccl"])
    ap.add_argument("--heavy", type=float, default=0.1)
    ap.add_argument("--slots", type=int, default=64)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--rebalance", type=int, default=2)
    ap.add_argument("--mismatch", action="store_true")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    from datetime import timedelta

    import numpy as np
    import torch
    import torch.distributed as dist

    from distraytracer_old_amd import rt, scenes

    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = local if a.transport == "rccl" else 0
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", timeout=timedelta(seconds=90))
    report = {"world": world, "transport": a.transport, "cli": a.cli, "checks": []}
    W, H, spp, seed = a.width, a.height, a.spp, a.seed
    scenes.ensure_bun69k()
    scene = rt.Scene.load_cli(a.cli, textures=scenes.prepare(a.cli), device=dev)
    if a.transport == "host":
        comm = rt.Comm.host(dist)
    else:
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(rt.group_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        comm = rt.Comm.rccl(rank, world, bytes(uid.numpy().tobytes()), dev)
    comm.selftest(4099)
    report["comm"] = comm.info()

    info = scene.info()
    if info["photon_mode"]:
        t = time.perf_counter()
        scene.build_photons_comm(comm, seed)
        report["photon_build_comm_s"] = time.perf_counter() - t
        if rank == 0:
            ref = rt.Scene.load_cli(a.cli, textures=scenes.prepare(a.cli), device=dev)
            ref.build_photons(seed)
            p1, w1 = scene.photons()
            p0, w0 = ref.photons()
            ok = (p0.shape == p1.shape and np.array_equal(p0.view(np.uint64), p1.view(np.uint64))
                  and np.array_equal(w0.view(np.uint64), w1.view(np.uint64))
                  and rt.photon_maps_equal(scene.photon_map(), ref.photon_map()))
            report["checks"].append(["photon_list and map == rt_photons_build", bool(ok), int(len(p0))])
            ref.close()

    heavy = a.heavy * (2.0 if (a.mismatch and rank == world - 1) else 1.0)
    try:
        grp = rt.Group.create_comm(scene, comm, W, H, spp=spp, seed=seed, rgb=True, heavy=heavy, slots=a.slots)
    except rt.RTError as e:
        report["create_error"] = str(e)
        grp = None
    if a.mismatch:
        report["checks"].append(["every rank refused the mismatched frame", grp is None, report.get("create_error")])
        if grp is not None:
            grp.close()
    else:
        gi = grp.info()
        report["group_info"] = gi
        report["checks"].append(["transport", gi["rccl"] == (2 if a.transport == "host" else 1), gi["rccl"]])
        report["checks"].append(["plan checked at creation", gi["plan_checks"] == 1, gi["plan_checks"]])
        owner, order = grp.plan()
        report["split_tiles"] = int((owner >= world).sum())
        report["rank_pixels"] = len(grp.rank_pixels(rank))
        if a.rebalance:
            ms = grp.rebalance(rounds=a.rebalance, iters=2)
            report["rank_ms"] = ms.tolist()
            gi = grp.info()
            report["checks"].append(["plan checked after every cut", gi["plan_checks"] == 1 + a.rebalance,
                                     gi["plan_checks"]])
            o2, d2 = grp.plan()
            report["checks"].append(["rebalance keeps split tiles and order",
                                     bool(np.array_equal(d2, order) and np.array_equal(o2 >= world, owner >= world)), None])
        # every rank's pixels partition the frame (each rank derives every rank's list)
        allpix = np.concatenate([grp.rank_pixels(q) for q in range(world)])
        report["checks"].append(["rank pixel lists partition the frame",
                                 bool(np.array_equal(np.sort(allpix), np.arange(W * H))), None])
        if rank == 0:
            rgb1, argb1 = scene.render(W, H, spp=spp, seed=seed)
        frames = []
        for f in range(a.frames):  # blocking frames into host buffers
            c, argb = grp.render_host(W, H)
            if rank == 0:
                frames.append(bool(np.array_equal(argb, argb1) and np.array_equal(c.view(np.uint32), rgb1.view(np.uint32))))
        # pipelined frames into caller-owned device buffers, no sync between them
        outs = [(torch.full((H, W, 3), -1.0, device=f"cuda:{dev}"), torch.zeros((H, W), dtype=torch.int32,
                                                                                device=f"cuda:{dev}"))
                for _ in range(4)]
        torch.cuda.synchronize()
        for o in outs:
            grp.render(o[0].data_ptr(), o[1].data_ptr())
        grp.sync()
        if rank == 0:
            for c, argb in outs:
                frames.append(bool(np.array_equal(argb.cpu().numpy(), argb1)
                                   and np.array_equal(c.cpu().numpy().view(np.uint32), rgb1.view(np.uint32))))
            report["checks"].append(["every frame == rt_render bit for bit", all(frames), frames])
        report["frames"] = grp.info()["frames"]
        grp.close()
    dist.barrier()
    comm.close()
    scene.close()
    if rank == 0:
        Path(a.out).write_text(json.dumps(report, indent=1) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
