#!/usr/bin/env python3
"""Summarise an SQ counter pass (tools/gpu_perf.sh) for the render kernel."""
import csv
import sys

rows = []
for f in sys.argv[1:]:
    rows += list(csv.DictReader(open(f)))
agg = {}
for r in rows:
    if "render_kernel" not in r["Kernel_Name"]:
        continue
    agg.setdefault(r["Kernel_Name"][:40] + "#" + r["Dispatch_Id"] if len(sys.argv) == 2 else r["Kernel_Name"][:40], {})[r["Counter_Name"]] = float(r["Counter_Value"])
for d, v in agg.items():
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(d, {k: f"{x:.3g}" for k, x in v.items()})
    print("   wait_any %.1f%%  wait_inst %.1f%%  active %.1f%%  valu-active %.1f%%" % (
        100 * v.get("SQ_WAIT_ANY", 0) / wc, 100 * v.get("SQ_WAIT_INST_ANY", 0) / wc,
        100 * v.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * v.get("SQ_ACTIVE_INST_VALU", 0) / wc))
