#!/usr/bin/env python3
"""Per-launch HBM bytes (FETCH_SIZE x 1024 x 2, gfx950) of the render kernel in each given counter CSV."""
import csv
import sys

for f in sys.argv[1:]:
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
         if r["Counter_Name"] == "FETCH_SIZE" and "render_kernel<false" in r["Kernel_Name"]]
    if v:
        print(f"{f}: {sum(v) / len(v) * 2048 / 1e9:.3f} GB/launch over {len(v)} launches")
