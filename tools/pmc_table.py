#!/usr/bin/env python3
"""Per-launch PMC means of the timed render kernel from tools/gpu_prof_cfg.sh output.

  python tools/pmc_table.py gpurun_out/<tag>/<cfg> [--json out.json] [--workload "C3 c3_bun69k.cli 1024x1024 16spp"]

Reads every pmc_*/run_counter_collection.csv under the directory, keeps the dispatches of
the non-counting render kernel (render_kernel<false, F>), and prints each counter's mean
per launch, plus derived figures: HBM bytes (FETCH_SIZE x 1024 x 2 per the gfx950 half-count
correction of MI355X_MICROARCH.md, WRITE_SIZE x 1024), wait / VALU-active fractions and the
fp64 VALU instruction mix. The kernel-trace mean duration comes from prof/run_kernel_stats.csv.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    workload = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else None
    vals = defaultdict(list)
    kname = None
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv"))):
        per = defaultdict(float)  # (dispatch, counter) -> summed over dimensions
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "render_kernel<false" not in n:
                continue
            kname = n
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    mean = {c: sum(v) / len(v) for c, v in vals.items()}
    ms = None
    st = os.path.join(d, "prof", "run_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            if "render_kernel<false" in r["Name"]:
                ms = float(r["AverageNs"]) / 1e6
    der = {"kernel": kname, "kernel_ms": ms}
    if "FETCH_SIZE" in mean:
        der["hbm_read_bytes"] = mean["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in mean:
        der["hbm_write_bytes"] = mean["WRITE_SIZE"] * 1024
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in mean:
                der[k.lower() + "_frac"] = mean[k] / wc
    f64 = {k: mean[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64") if k in mean}
    if f64 and ms:
        # SQ_INSTS_* count wave instructions: x64 lanes; an FMA is 2 FLOP
        flops = 64 * (2 * f64.get("SQ_INSTS_VALU_FMA_F64", 0) + f64.get("SQ_INSTS_VALU_ADD_F64", 0)
                      + f64.get("SQ_INSTS_VALU_MUL_F64", 0))
        der["fp64_flop_per_launch_upper"] = flops
        der["fp64_tflops_upper"] = flops / (ms / 1e3) / 1e12
        if "SQ_INSTS_VALU" in mean:
            der["fp64_share_of_valu"] = sum(f64.values()) / mean["SQ_INSTS_VALU"]
    try:  # the library the profiled run loaded (the same DISTRAYTRACER_LIB / in-tree library)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        from distraytracer_old_amd import rt
        bid = rt.build_id()
    except Exception:
        bid = None
    out = {"workload": workload, "build_id": bid, "counters": mean, "derived": der,
           # bench.py reads these (per launch of the timed render kernel)
           "hbm_bytes_per_launch": der.get("hbm_read_bytes"), "hbm_write_bytes_per_launch": der.get("hbm_write_bytes"),
           "fp64_flop_per_launch": der.get("fp64_flop_per_launch_upper"), "hbm_kernel": kname,
           "method": "rocprofv3 --pmc, one pass per counter group; FETCH_SIZE x 1024 x 2 (gfx950 half-count), "
                     "WRITE_SIZE x 1024; fp64 FLOP = 64 x (2 FMA + ADD + MUL) wave instructions (upper bound: "
                     "inactive lanes counted)"}
    print(json.dumps(out, indent=1))
    if out_json:
        json.dump(out, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
