#!/usr/bin/env python3
"""Sum a PMC counter over every render-path kernel dispatch (render_kernel / wf_*), divided by the
frame count: python tools/pmc_frame_sum.py DIR COUNTER FRAMES MULT"""
import csv
import glob
import sys
from collections import defaultdict

d, counter, frames, mult = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
tot = defaultdict(float)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if r["Counter_Name"] != counter or not ("render_kernel<false" in n or "wf_" in n):
            continue
        key = "render_kernel" if "render_kernel" in n else n.split("(")[0].split("<")[0].split("::")[-1]
        tot[key] += float(r["Counter_Value"])
all_ = sum(tot.values())
print(counter, f"{all_ * mult / frames / 1e9:.3f} GB per frame;",
      ", ".join(f"{k} {v * mult / frames / 1e9:.3f}" for k, v in sorted(tot.items())))
