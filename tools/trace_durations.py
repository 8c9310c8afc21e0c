#!/usr/bin/env python3
"""Per-launch durations of the timed render kernel from a rocprofv3 --kernel-trace CSV.

  python tools/trace_durations.py run_kernel_trace.csv out.txt [timed_launches]
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "render_kernel<false" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 10
with open(sys.argv[2], "w") as f:
    f.write(f"{rows[0]['Kernel_Name'] if rows else '?'}: launch durations (ms), rocprofv3 --kernel-trace of bench.py\n")
    f.write("(setup renders: tile-schedule calibration + clock warm-up; then the warmup and the timed steps)\n")
    f.write(" ".join(f"{x:.3f}" for x in d) + "\n")
    if d:
        f.write(f"mean of the last {k} (timed) launches: {sum(d[-k:]) / len(d[-k:]):.3f} ms; mean of all {len(d)}: "
                f"{sum(d) / len(d):.3f} ms\n")
print(open(sys.argv[2]).read())
