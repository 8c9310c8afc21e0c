#!/usr/bin/env python3
"""Benchmark: the reference's headline workload on MI355X (BASELINE.json).

metric  "Mray/s + achieved HBM GB/s, bun69k.cli 1024^2 16spp, 1/2/4/8 GPU"
workload C3 = scenes/c3_bun69k.cli (data/p3_t09.cli without `wood`) with the
         synthetic bun69k (69,451 triangles), 1024x1024, 16 spp, seed 0x5EED0001.

One step = one full C3 frame through the native N-GPU group (rt_group_*, csrc/group.hip): every
rank renders its part of the frame's wave tiles -- a contiguous cut of rank 0's measured wave times,
re-cut from the ranks' measured render times in setup (rt_group_rebalance), the heaviest tiles
rendered one sample per wave -- into a device buffer; ranks > 0 pack their ARGB pixels (the ints the
reference's rndrdImg.pixels holds) and send them to rank 0 over RCCL (grouped ncclSend / ncclRecv,
each rank's pixels over its own xGMI link), rank 0 scatters them into the frame; frame i's exchange
overlaps frame i+1's render and the last one is drained inside the timed region (--backend gloo:
the same native rank mode over the host transport, ranks sharing GPUs -- a rehearsal, not a scaling
measurement). After timing, rank 0 checks the assembled frame against rt_render bit for bit
(frame_check). Work per step is one frame whatever N is
(strong scaling). value = traced rays of the frame (camera + shadow + reflection + refraction,
counted exactly by an instrumented run before timing) / max-over-ranks step time.

roofline: algorithmic bytes of the render kernel per launch /
its mean duration from HIP events on the launch stream; peak 8000 GB/s (MI355X HBM3E).
The bytes are SURVEY 8(d)'s record sizes x the record loads the instrumented kernel counts
-- once per WAVE step for records a wave loads once for all its lanes (packet traversal
of BVHs and the photon map, wave-uniform top-level entries, lights), per lane otherwise
(texels). The per-lane 8(d) figure (every lane charged for every record it tests) is
reported beside it. traffic: measured HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE)
from the newest committed rocprofv3 --pmc summary of the workload in profiles/ when it is of
this library build (rt_build_id) and its kernel time is within 5 % of this run's, else null
(traffic_missing says why); fp64: the kernel's fp64 FLOP rate (same PMC summary) against the measured fp64
VALU peak (tools/fp64_peak.hip); valu: the share of the SIMDs' VALU issue slots the kernel fills at an
assumed 4 cycles per instruction; valu_measured: the same from MEASURED issue costs per instruction
class (tools/valu_issue.hip x the PMC class counts, tools/valu_model.py) -- the bound this branchy
fp64 traversal runs into.

cpu_baseline: the oracle (CPU restatement of the reference path, fp64) timed on
the box's CPU share (affinity / cgroup quota / OMP_NUM_THREADS; the host's CPU count and model
are recorded beside it) on the same frame (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

METRIC = "Mray/s + achieved HBM GB/s, bun69k.cli 1024² 16spp, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_PEAK_GBPS = 6300.0  # measured float4-copy peak (MI355X_MICROARCH.md)
SIMD_CLOCK_HZ = 2.4e9  # MI355X max engine clock (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 74.07  # measured: tools/fp64_peak.hip on MI355X (profiles/r02_fp64_peak.json)

# Algorithmic bytes per counted event: SURVEY.md 8(d)'s per-ray formula, records at the
# sizes it states and no cache credit:
#   64 node + 48 triangle + 64 quad + 32 sphere/cylinder + 16 light + 32 photon kd-node
#   + 16 texel quad (DESIGN.md "Measurement")
RECORD_BYTES = {
    "node": 64,       # BVH node records fetched (internal-node visits)
    "tri": 48,        # triangle records tested
    "quad": 64,       # quad / plane records tested
    "implicit": 32,   # sphere / cylinder / box records tested
    "light": 16,      # light records read per shaded hit
    "photon": 32,     # photon kd-nodes visited
    "texel": 16,      # bilinear texel quads fetched
}


# the same records counted per wave step where a wave loads a record once for all its lanes
# (RT_ST_W_*); texels are per-lane loads
WAVE_RECORD_BYTES = {"w_node": 64, "w_tri": 48, "w_quad": 64, "w_implicit": 32, "w_light": 16, "w_photon": 32,
                     "texel": 16}


def algorithmic_bytes(st: dict) -> int:
    """SURVEY 8(d) per-lane figure: every lane charged for every record it tests."""
    return int(sum(st.get(k, 0) * b for k, b in RECORD_BYTES.items()))


def wave_bytes(st: dict) -> int:
    """8(d) record sizes x record loads as the kernel issues them (per wave step / per lane)."""
    return int(sum(st.get(k, 0) * b for k, b in WAVE_RECORD_BYTES.items()))


def traced_rays(st: dict) -> int:
    return int(st["camera"] + st["shadow"] + st["refl"] + st["refr"])


def find_pmc(workload: str, build_id: str, kern_ms: float):
    """The newest committed PMC summary (profiles/rNN_*pmc*.json, written by tools/pmc_table.py;
    BENCH_TRAFFIC_JSON names one explicitly) that describes THIS kernel: same workload, same
    library build id (rt_build_id) and a kernel time within 5 % of this run's. Returns (summary,
    file name, why-not): a summary of another build or a stale time is not used."""
    files = sorted(glob.glob(str(REPO / "profiles" / "*pmc*.json")))  # rNN<letter>_...: later runs sort later
    if os.environ.get("BENCH_TRAFFIC_JSON"):
        files = [os.environ["BENCH_TRAFFIC_JSON"]]
    why = "no PMC summary of this workload in profiles/"
    for f in reversed(files):
        try:
            d = json.loads(Path(f).read_text())
        except Exception:
            continue
        if d.get("workload") != workload or not d.get("hbm_bytes_per_launch"):
            continue
        pms = (d.get("derived") or {}).get("kernel_ms")
        if d.get("build_id") != build_id:
            why = f"newest summary {Path(f).name} is of build {d.get('build_id')}, not {build_id}"
        elif not pms or abs(pms - kern_ms) > 0.05 * kern_ms:
            why = f"{Path(f).name}: its kernel time {pms} ms is not within 5 % of this run's {kern_ms:.4f} ms"
        else:
            return d, Path(f).name, None
        break  # only the newest summary of the workload is a candidate
    return None, None, why


# PMC instruction classes of the VALU issue model (tools/valu_model.py cost_ns keys)
VALU_CLASSES = {"add_f64": "SQ_INSTS_VALU_ADD_F64", "mul_f64": "SQ_INSTS_VALU_MUL_F64", "fma_f64": "SQ_INSTS_VALU_FMA_F64",
                "trans_f64": "SQ_INSTS_VALU_TRANS_F64", "add_f32": "SQ_INSTS_VALU_ADD_F32",
                "mul_f32": "SQ_INSTS_VALU_MUL_F32", "fma_f32": "SQ_INSTS_VALU_FMA_F32",
                "trans_f32": "SQ_INSTS_VALU_TRANS_F32", "int32": "SQ_INSTS_VALU_INT32",
                "int64": "SQ_INSTS_VALU_INT64", "cvt": "SQ_INSTS_VALU_CVT"}


def find_valu_model(variant: int):
    """The newest committed VALU issue model (profiles/*valu_model*.json, tools/valu_model.py) of this
    render-kernel variant: measured issue cost per instruction class."""
    for f in sorted(glob.glob(str(REPO / "profiles" / "*valu_model*.json")), reverse=True):
        try:
            d = json.loads(Path(f).read_text())
        except Exception:
            continue
        if d.get("variant_F") == variant and d.get("cost_ns"):
            return d, Path(f).name
    return None, None


def valu_issue(cnt: dict, vm: dict, n_simd: int, kern_ms: float):
    """Share of the SIMDs' VALU issue capacity the kernel's instructions fill: sum over PMC classes of
    count x measured cost (tools/valu_issue.hip: ns per wave instruction per SIMD at saturation), the
    unclassified rest at its static-mix cost, over SIMDs x kernel time. None without the class counts."""
    cost = vm["cost_ns"]
    if not all(c in cnt for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                  "SQ_INSTS_VALU_INT32")):
        return None
    total = float(cnt["SQ_INSTS_VALU"])
    per, known = {}, 0.0
    for k, c in VALU_CLASSES.items():
        if c in cnt:
            per[k] = float(cnt[c]) * cost[k]
            known += float(cnt[c])
    per["rest"] = max(0.0, total - known) * cost["rest"]
    avail = n_simd * kern_ms * 1e6  # SIMD-ns
    return {"issue_frac": sum(per.values()) / avail,
            "by_class": {k: v / avail for k, v in per.items()},
            "classes_counted": sorted(k for k in VALU_CLASSES if VALU_CLASSES[k] in cnt),
            "note": "sum of PMC class counts x measured saturated issue cost per wave instruction "
                    "(tools/valu_issue.hip, 8 waves / SIMD); the unclassified rest (moves, compares, "
                    "selects, lane ops) at the mean cost of its static in-loop mix (tools/valu_model.py)"}


def cpu_share() -> dict:
    """The host CPUs this process may use (the box's share: its affinity mask and cgroup quota --
    os.cpu_count() reports the whole machine's CPUs, which a shared box does not give us),
    plus what the host has (lscpu's model name, nproc)."""
    n_host = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n_aff = n_host
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = n_aff if quota is None else max(1, min(n_aff, int(quota)))
    # the pool's rule for a one-GPU box: worker pools sized to its 16-CPU share (OMP_NUM_THREADS)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(share, cap) if cap > 0 else share
    return {"threads": threads, "host_cpus": n_host, "affinity_cpus": n_aff, "cgroup_cpu_quota": quota,
            "omp_num_threads": cap or None, "cpu_model": model}


def cpu_baseline(cli, W, H, spp, seed, tex, row_step=1):
    from oracle.oracle import OracleScene

    share = cpu_share()
    threads = share["threads"]
    o = OracleScene(REPO / "scenes", cli, tex)
    o.render(W, H, spp=spp, seed=seed, rows=(0, H), row_step=512, threads=threads)  # warm caches
    t0 = time.perf_counter()
    _, _, st = o.render(W, H, spp=spp, seed=seed, rows=(0, H), row_step=row_step, threads=threads)
    dt = time.perf_counter() - t0
    rays = traced_rays(st)
    # single-thread rate (mirrors the single-threaded Java reference) on a smaller sample
    t1 = time.perf_counter()
    _, _, st1 = o.render(W, H, spp=spp, seed=seed, rows=(1, H), row_step=16, threads=1)
    dt1 = time.perf_counter() - t1
    o.close()
    return {
        "value": rays / dt / 1e6,
        "unit": "Mray/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle (fp64 C++ restatement) on rows 0::{row_step} of the {W}x{H}x{spp} frame "
                  f"({rays} rays, {dt:.2f} s on {threads} threads)",
        "host": share,
        "value_1thread": traced_rays(st1) / dt1 / 1e6,
        "sample_1thread": f"rows 1::16 ({traced_rays(st1)} rays, {dt1:.2f} s, 1 thread)",
    }


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising HIP (a process that has initialised
    the GPU must not start the ranks): the *_VISIBLE_DEVICES lists, else the KFD topology's GPU
    nodes (/sys/class/kfd: nodes with a non-zero gpu_id)."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip()])
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            n += int(Path(f).read_text().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    return n


def launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) started directly: start N ranks as ONE child process tree
    (torch.distributed.run, one rank per GPU, 127.0.0.1 rendezvous) and return its exit code.
    Nothing here touches the GPU (visible_gpus reads sysfs / the environment, not HIP)."""
    import socket
    import subprocess

    if args.backend == "nccl":  # gloo rehearsals share devices: no count needed
        have = visible_gpus()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {have}", file=sys.stderr)
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(REPO / "bench.py"), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--partition", default="tiles", choices=["tiles", "bands"],
                    help="N > 1: cost-balanced wave tiles (default) or interleaved 8-row bands")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N-rank step on fewer GPUs (the native group over the host transport "
                         "on gloo, pixels staged through host memory; ranks share devices)")
    ap.add_argument("--impl", default="native", choices=["native", "python"],
                    help="N > 1: the native group (rt_group_create_comm, default) or the Python rank path "
                         "(multigpu.RankRenderer over torch.distributed)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)

    import numpy as np
    import torch

    from distraytracer_old_amd import multigpu, rt, scenes

    cli, W, H, spp, seed = scenes.CONFIGS[args.config]
    ndev = torch.cuda.device_count()
    if ndev < 1:
        print("bench.py: no GPU visible", file=sys.stderr)
        sys.exit(2)
    dev = local if args.backend == "nccl" else local % ndev
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    coll_dev = "cuda" if args.backend == "nccl" else "cpu"  # where collectives' tensors live

    tex = scenes.prepare(cli)
    # host-side parse + flatten + BVH build alone (rt_scene_inspect_cli: no device), then the full
    # scene load (the same host build + upload to HBM); both outside the scaling metric
    t = time.perf_counter()
    rt.inspect_cli(cli, textures=tex)
    host_build_s = time.perf_counter() - t
    t = time.perf_counter()
    scene = rt.Scene.load_cli(cli, textures=tex, device=dev)
    scene_load_s = time.perf_counter() - t
    info = scene.info()
    # the ranks' communicator (N > 1, native): RCCL over xGMI, or the host transport on gloo (rehearsals)
    native = args.impl == "native"
    comm = None
    comm_note = None
    if world > 1 and native:
        if args.backend == "nccl":
            # RCCL communicator of the library (its own, beside torch's); if any rank fails to make it,
            # every rank falls back to the host transport over a gloo group (slower exchange through host
            # memory, same frame) -- decided collectively, so no rank is left waiting
            gloo_pg = dist.new_group(backend="gloo")
            uid = torch.zeros(128, dtype=torch.uint8, device=coll_dev)
            if rank == 0:
                uid.copy_(torch.frombuffer(bytearray(rt.group_unique_id()), dtype=torch.uint8))
            dist.broadcast(uid, 0)
            err = None
            try:
                comm = rt.Comm.rccl(rank, world, bytes(uid.cpu().numpy().tobytes()), dev)
                comm.selftest(1031)
            except rt.RTError as e:
                err = str(e)
            bad = torch.tensor([1 if err else 0], dtype=torch.int32)
            dist.all_reduce(bad, group=gloo_pg)
            if int(bad.item()):
                if comm is not None:
                    comm.close()
                comm = rt.Comm.host(dist, gloo_pg)
                comm_note = f"RCCL communicator failed on {int(bad.item())} rank(s) ({err or 'another rank'}): host transport over gloo"
                print(f"bench.py rank {rank}: {comm_note}", file=sys.stderr)
        else:
            comm = rt.Comm.host(dist)
    photon_s = None
    if info["photon_mode"]:  # photon pre-pass (initRender), outside the timed region; sharded over ranks
        torch.cuda.synchronize()
        t = time.perf_counter()
        if native:  # rt_photons_build_comm: shard, exchange, merge, build -- behind the C ABI
            scene.build_photons_comm(comm, seed)
        else:
            multigpu.build_photons_sharded(scene, seed, info["photon_count"], dist, device=coll_dev)
        torch.cuda.synchronize()
        photon_s = time.perf_counter() - t
    # the exchanged frame is the reference's output, ARGB ints (rndrdImg.pixels): 4 bytes a pixel.
    # The N-rank step is the native group (rt_group_*, csrc/group.hip): rank 0 measures the layout's
    # wave times and broadcasts them, every rank derives the same plan (checked collectively), renders
    # its part, packs it and sends it to rank 0 over RCCL (ncclSend / ncclRecv), rank 0 scatters it
    # into the frame -- one C call per frame. N = 1: a one-rank group (every tile, no exchange).
    # --backend gloo (ranks sharing one GPU, where RCCL cannot run): the same native rank mode over
    # the host transport (pixels staged through host memory); --impl python: multigpu.RankRenderer.
    p_frame = rt.params(W, H, spp=spp, seed=seed)
    if native:
        if world > 1:
            grp = rt.Group.create_comm(scene, comm, W, H, spp=spp, seed=seed)
        else:
            grp = rt.Group.create([scene], W, H, spp=spp, seed=seed)
        rank_ms_rebalanced = None
        if world > 1:  # setup: three re-cuts of the plan from the ranks' measured render times (collective)
            rank_ms_rebalanced = grp.rebalance(rounds=3, iters=10).tolist()
        run_t, split_t = grp.rank_tiles(rank)
        my_tiles = np.concatenate([run_t, split_t]).astype(np.int32)
        parallelism = ("1 GPU" if world == 1 else
                       f"cost-balanced wave tiles over {world} ranks (native rt_group, one process per GPU) + "
                       + ("RCCL send/recv of the ARGB pixels to rank 0" if comm is not None and comm.info()["transport"] == "rccl"
                          else "host-transport (gloo) send/recv of the ARGB pixels to rank 0"))

        def step(ev=None):
            grp.render()

        def drain():
            grp.sync()
    else:
        rr = multigpu.RankRenderer(scene, W, H, spp, seed, dist, stage_host=True, planes=("argb",),
                                   partition=args.partition)
        my_tiles = (np.concatenate([rr.plan.tiles, rr.plan.split]).astype(np.int32)
                    if rr.partition == "tiles" else None)
        parallelism = (f"cost-balanced wave tiles over {world} ranks" if rr.partition == "tiles" else
                       f"{multigpu.BAND}-row bands interleaved over {world} ranks") + " + gloo gather of the ARGB pixels"
        step, drain = rr.step, rr.finish

    # exact per-frame counters (instrumented runs, outside the timed region): the kernel as it
    # runs (top-level culling on: the record loads it issues) and the reference algorithm's work
    # (RT_RENDER_NOCULL: every objList entry tested for every ray, SURVEY 8(d)'s per-ray bytes).
    # A rank's split tiles are counted as tile waves (their samples and rays are the same).
    p_nocull = rt.params(W, H, spp=spp, seed=seed, flags=rt.RENDER_NOCULL)
    if my_tiles is not None:
        zero = dict.fromkeys(rt.ST_NAMES, 0)
        st = scene.render_tiles_count(p_frame, my_tiles) if len(my_tiles) else zero
        sr = scene.render_tiles_count(p_nocull, my_tiles) if len(my_tiles) else zero
    else:
        r0, r1, rstep, band = rr.rows
        _, _, st = scene.render_count(W, H, spp=spp, seed=seed, rows=(r0, r1), row_step=rstep, row_band=band)
        _, _, sr = scene.render_count(W, H, spp=spp, seed=seed, rows=(r0, r1), row_step=rstep, row_band=band,
                                      flags=rt.RENDER_NOCULL)
    counts = torch.tensor([traced_rays(st), algorithmic_bytes(sr), st["camera"], wave_bytes(st), algorithmic_bytes(st)],
                          dtype=torch.float64, device=coll_dev)
    if dist:
        dist.all_reduce(counts)
    rays_frame, bytes_frame, cam_frame, wbytes_frame, xbytes_frame = [float(x) for x in counts.tolist()]
    assert int(cam_frame) == W * H * spp, f"counted {cam_frame} camera samples, the frame has {W * H * spp}"
    my_bytes = float(algorithmic_bytes(sr))
    my_xbytes = float(algorithmic_bytes(st))
    my_wbytes = float(wave_bytes(st))

    # setup (untimed, like the counting run): a layout's calibration renders ran when the group /
    # renderer was made; ~0.2 s of untimed frames next -- the GPU's clocks ramp over the first launches
    # Every frame is collective at N > 1, so the ranks agree on the count (max over ranks of
    # 0.2 s / one frame): a per-rank time bound would leave them on different frames, deadlocked.
    t_warm = time.perf_counter()
    step()
    drain()
    n_warm = torch.tensor([min(200, int(0.2 / max(time.perf_counter() - t_warm, 1e-4)))], dtype=torch.int64,
                          device=coll_dev)
    if dist:
        dist.all_reduce(n_warm, op=dist.ReduceOp.MAX)
    for _ in range(int(n_warm.item())):
        step()
        drain()
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if native:
        grp.kernel_ms(rank)  # reset the kernel-time window
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    drain()  # the last frame's exchange + scatter are inside the timed region
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if native:  # HIP events on the rank's render stream (rt_group_kernel_ms)
        kern_ms, nfr = grp.kernel_ms(rank)
        assert nfr == min(args.steps, 64), (nfr, args.steps)
    else:
        kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    # the frame the timed steps produced, checked (after timing): rank 0's assembled ARGB frame against
    # rt_render of the whole frame on rank 0's GPU, bit for bit (every rank takes part in the frame)
    frame_check = None
    if native:
        _, got = grp.render_host(W, H, rgb=False)
        if rank == 0:
            want = np.zeros((H, W), dtype=np.int32)
            scene.render_argb_into(want, W, H, spp=spp, seed=seed)
            frame_check = {"bit_exact_vs_rt_render": bool(np.array_equal(got, want)),
                           "pixels_differing": int((got != want).sum()),
                           "plan_checks": grp.info()["plan_checks"],
                           "transport": rt.TRANSPORT_NAMES[grp.info()["rccl"]]}

    # the drop-in path's cost (rank 0 of a 1-GPU run): rt_render of the whole frame into a host ARGB
    # buffer -- what the JNI draw() does: launch + the 4 B/pixel read-back to
    # pageable host memory, blocking. Timed apart from the steps, after them.
    host_ms = None
    if world == 1:
        px = np.zeros((H, W), dtype=np.int32)
        for _ in range(2):  # this layout's tile-schedule calibration (probe order, then measured order)
            scene.render_argb_into(px, W, H, spp=spp, seed=seed)
        n_host = max(3, min(args.steps, 5))
        t_h = time.perf_counter()
        for _ in range(n_host):
            scene.render_argb_into(px, W, H, spp=spp, seed=seed)
        host_ms = (time.perf_counter() - t_h) / n_host * 1e3

    t = torch.tensor([dt, kern_ms], dtype=torch.float64, device=coll_dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, kern_ms_max = t.tolist()
    ms_per_step = dt / args.steps * 1e3

    if rank == 0:
        # rank-0 kernel: its own algorithmic bytes over its own mean kernel duration
        achieved = my_wbytes / (kern_ms / 1e3) / 1e9
        achieved_lane = my_bytes / (kern_ms / 1e3) / 1e9
        achieved_lane_x = my_xbytes / (kern_ms / 1e3) / 1e9
        workload = f"{args.config} {cli} {W}x{H} {spp}spp"
        var_t, var_c = scene.variant()  # the timed and counted render_kernel<CNT, F> instances (same F)
        bid = rt.build_id()
        pmc, tsrc, why = find_pmc(workload, bid, kern_ms) if world == 1 else (None, None, "N > 1")
        traffic = traffic_rd = traffic_wr = traffic_lo = None
        fp64 = valu = valu_measured = None
        if pmc:
            traffic_rd = float(pmc["hbm_bytes_per_launch"])
            traffic_wr = pmc.get("hbm_write_bytes_per_launch")
            traffic = traffic_rd + float(traffic_wr or 0)
            traffic_lo = traffic_rd / 2 + float(traffic_wr or 0)
            if pmc.get("fp64_flop_per_launch"):
                tf = float(pmc["fp64_flop_per_launch"]) / (kern_ms / 1e3) / 1e12
                fp64 = {"tflops": tf, "peak_tflops_measured": FP64_PEAK_TFLOPS, "frac": tf / FP64_PEAK_TFLOPS,
                        "flop_per_launch": float(pmc["fp64_flop_per_launch"]),
                        "note": "fp64 VALU wave instructions x 64 lanes (inactive lanes included: an upper bound)"}
            cnt = pmc.get("counters") or {}
            vm, vm_src = find_valu_model(var_t)
            if cnt.get("SQ_INSTS_VALU") and vm:
                valu_measured = valu_issue(cnt, vm, 4 * torch.cuda.get_device_properties(dev).multi_processor_count,
                                           kern_ms)
                if valu_measured:
                    valu_measured["model"] = vm_src
            if cnt.get("SQ_INSTS_VALU"):
                # the bound this fp64 traversal actually runs into: the SIMDs' VALU issue. A wave64 VALU
                # instruction occupies a 16-lane SIMD for 4 cycles (the fp64 FMA rate the peak is quoted on)
                n_simd = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
                cyc = n_simd * SIMD_CLOCK_HZ * (kern_ms / 1e3)
                valu = {"issue_frac": float(cnt["SQ_INSTS_VALU"]) * 4 / cyc,
                        "active_frac": float(cnt.get("SQ_ACTIVE_INST_VALU", 0)) * 4 / cyc,
                        "resident_waves_per_simd": float(cnt.get("SQ_WAVE_CYCLES", 0)) * 4 / cyc,
                        "wave_instructions_per_launch": float(cnt["SQ_INSTS_VALU"]),
                        "salu_instructions_per_launch": float(cnt.get("SQ_INSTS_SALU", 0)),
                        "simds": n_simd, "clock_ghz": SIMD_CLOCK_HZ / 1e9,
                        "note": "SQ_INSTS_VALU x 4 cycles / (SIMDs x max clock x kernel time): the share of the "
                                "SIMDs' VALU issue slots the kernel fills (SQ_ACTIVE_INST_VALU and SQ_WAVE_CYCLES "
                                "count in 4-cycle units); from the same build's PMC summary"}
        out = {
            "metric": METRIC,
            "value": rays_frame / (ms_per_step / 1e3) / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "build_id": bid,
            "data": ("synthetic: bun69k = deterministic subdivision of data/bun500.cli (69,451 tris); "
                     "scene data/p3_t09.cli without the wood line") if args.config == "C3" else
                    f"scene scenes/{cli} (SURVEY 8(d) {args.config}); synthetic inputs where the reference's are missing",
            "config": {"workload": workload, "width": W, "height": H, "spp": spp, "seed": seed,
                       "rays_per_frame": int(rays_frame), "camera_samples": int(cam_frame),
                       "parallelism": parallelism},
            "camera_msamples_per_s": cam_frame / (ms_per_step / 1e3) / 1e6,
            "kernel_ms_max_over_ranks": kern_ms_max,
            "rank_render_ms_after_rebalance": rank_ms_rebalanced if native else None,
            "frame_check": frame_check,
            "transport_note": comm_note,
            "host_path_ms_per_step": host_ms,
            "host_path": "rt_render into a host ARGB buffer (the JNI draw(), INTEGRATION.md): kernel + "
                         f"{W * H * 4} B read-back to pageable memory, blocking; 1-GPU runs only",
            "host_build_s": host_build_s,
            "scene_load_s": scene_load_s,
            "photon_prepass_s": photon_s,
            "algorithmic_gbps": achieved,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS,
                         "frac_vs_measured_copy_peak": achieved / HBM_COPY_PEAK_GBPS,
                         "traffic": traffic, "traffic_read": traffic_rd, "traffic_write": traffic_wr,
                         "traffic_frac": (traffic / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBPS) if traffic else None,
                         "traffic_source": tsrc, "traffic_build_id": pmc.get("build_id") if pmc else None,
                         "traffic_kernel_ms": (pmc.get("derived") or {}).get("kernel_ms") if pmc else None,
                         "traffic_missing": why,
                         "traffic_lower_bound": traffic_lo,
                         "traffic_note": "L2-to-fabric request bytes (FETCH_SIZE x 2 + WRITE_SIZE x 1, "
                                         "MI355X_MICROARCH.md HBM section): Infinity-Cache hits are counted, and the "
                                         "x2 is the guide's rule for 16-B/lane streaming reads while this kernel "
                                         "reads mostly through scalar and 8-B loads -- an upper bound on HBM bytes; "
                                         "traffic_lower_bound takes FETCH_SIZE x 1",
                         "kernel": f"render_kernel<false, {var_t}u>", "kernel_ms": kern_ms,
                         "counted_kernel": f"render_kernel<true, {var_c}u>",
                         "bytes_per_launch": my_wbytes, "bytes_per_ray": wbytes_frame / max(1.0, rays_frame),
                         "accounting": "8(d) record sizes x record loads per wave step (packet / wave-uniform "
                                       "records) or per lane (texels), counted by counted_kernel: the "
                                       "instrumented instance of the timed kernel's variant",
                         # SURVEY 8(d) per lane, the reference algorithm's work (nothing culled): bytes
                         # the lanes consume, mostly served by the scalar cache / L2 (a wave loads a
                         # record once for all its lanes) -- a rate, not a fraction of HBM peak
                         "cache_served_gbps_8d_per_lane": achieved_lane,
                         "bytes_per_launch_8d_per_lane": my_bytes,
                         "bytes_per_ray_8d_per_lane": bytes_frame / max(1.0, rays_frame),
                         # ... and the same per-lane accounting of the work the kernel does (culling on)
                         "cache_served_gbps_8d_per_lane_executed": achieved_lane_x,
                         "bytes_per_ray_8d_per_lane_executed": xbytes_frame / max(1.0, rays_frame),
                         "fp64": fp64, "valu": valu, "valu_measured": valu_measured},
        }
        if world > 1 and args.backend == "gloo":
            out["rehearsal"] = f"gloo backend, {world} ranks on {ndev} GPU(s): not a scaling measurement"
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(cli, W, H, spp, seed, tex)
            cb["frame_s_1thread_extrapolated"] = rays_frame / (cb["value_1thread"] * 1e6)
            out["cpu_baseline"] = cb
        assert out["n_gpus"] == args.gpus
        print(json.dumps(out), flush=True)
    if native:
        grp.close()
    if comm is not None:
        comm.close()
    scene.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
