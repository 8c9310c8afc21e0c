#!/bin/bash
# round 5: XCD-hashed tile dispatch (RT_XCD_HASH superblocks) A/B on C3 / C4 / C5 + C3 L2 hit rate
set -o pipefail
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C3 --names xh0,xh2,xh4,xh8,xh0,xh2,xh4,xh8 --iters 20 > $OUT/sweep_c3.log 2>&1 && \
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C4 --names xh0,xh2,xh4,xh0 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names xh0,xh2,xh4,xh0 --iters 3 > $OUT/sweep_c5.log 2>&1 && \
for n in xh0 xh4; do
  DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_$n.so timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
    -d $OUT/${n}_tcc -o run -- python3 tools/variant_sweep.py one --cfg C3 --iters 3 > $OUT/${n}_tcc.log 2>&1 || exit 1
done
python3 - > $OUT/tcc.txt 2>&1 <<'PY'
import csv, glob
from collections import defaultdict
for n in ["xh0", "xh4"]:
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"gpurun_out/r05r/{n}_tcc/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "render_kernel<false" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    rates = sorted(v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"]) for v in per.values())
    print(n, "L2 hit rate (median over launches)", rates[len(rates) // 2] if rates else None, len(rates))
PY
