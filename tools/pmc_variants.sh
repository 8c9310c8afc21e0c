#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the render kernel for tuning builds (tools/variant_sweep.py build),
# one rocprofv3 --pmc pass per counter and build, each with its own time limit.
#   tools/pmc_variants.sh TAG CFG name1,name2,...
set -o pipefail
TAG=$1; CFG=$2; NAMES=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for n in ${NAMES//,/ }; do
  for c in WRITE_SIZE FETCH_SIZE; do
    DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_$n.so timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv \
      -d $OUT/${n}_$c -o run -- python3 tools/variant_sweep.py one --cfg $CFG --iters 2 > $OUT/${n}_$c.log 2>&1 || { rc=$?; break 2; }
  done
  python3 - "$OUT" "$n" >> $OUT/summary.txt <<'PY'
import csv, glob, sys
from collections import defaultdict
d, n = sys.argv[1], sys.argv[2]
out = []
for c, mult in (("WRITE_SIZE", 1024), ("FETCH_SIZE", 2048)):
    per = defaultdict(float)
    for f in glob.glob(f"{d}/{n}_{c}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "render_kernel<false" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(per.values())
    out.append(f"{c} {(v[len(v) // 2] * mult / 1e9) if v else float('nan'):.3f} GB (median of {len(v)} launches)")
print(n, " | ".join(out))
PY
done
exit $rc
