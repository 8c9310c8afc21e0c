#!/bin/bash
# round 5 final build: C3's VALU instruction classes (one --pmc pass, 8 SQ counters)
set -o pipefail
OUT=gpurun_out/r05zf
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
  SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 --output-format csv \
  -d $OUT/valu -o run -- python3 tools/variant_sweep.py one --cfg C3 --iters 3 > $OUT/valu.log 2>&1
python3 - > $OUT/valu_mix.txt 2>&1 <<'PY'
import csv, glob
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob("gpurun_out/r05zf/valu/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "render_kernel<false" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
runs = list(per.values())
keys = sorted({k for v in runs for k in v})
med = {k: sorted(v[k] for v in runs)[len(runs) // 2] for k in keys}
tot = med.get("SQ_INSTS_VALU", 1.0)
for k in keys:
    print(f"{k:28s} {med[k]:16.0f}  {med[k] / tot:6.3f}")
rest = tot - sum(med[k] for k in keys if k != "SQ_INSTS_VALU")
print(f"{'rest (moves, compares, selects, lane ops, min/max)':28s} {rest:16.0f}  {rest / tot:6.3f}")
print("launches", len(runs))
PY
