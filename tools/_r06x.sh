#!/bin/bash
# PMC instruction counts of the C3 render kernel: RT_F32_TRI=0 (tri0) vs the fp32 triangle pre-test (head)
set -o pipefail
OUT=gpurun_out/r06x; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_BUSY_CYCLES"
for v in tri0 head; do
  for p in 1 2; do
    eval C=\$P$p
    DISTRAYTRACER_LIB=tools/_variants/lib_$v.so timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_${v}_$p -o run -- python3 tools/variant_sweep.py one --cfg C3 --iters 2 > $OUT/${v}_$p.log 2>&1 || exit 1
  done
done
python3 - > $OUT/summary.txt <<'P'
import csv, glob, collections
for v in ("tri0", "head"):
    per = collections.defaultdict(float); disp = set()
    for f in glob.glob(f"gpurun_out/r06x/pmc_{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "render_kernel<false, 0u" not in r["Kernel_Name"]: continue
            per[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add((f, r["Dispatch_Id"]))
    n = max(1, len(disp) // 2)
    print(v, {k: round(x / n / 1e6, 2) for k, x in sorted(per.items())})
P
