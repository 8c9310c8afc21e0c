#!/bin/bash
# round 5: kNN counting histogram 128 u8 buckets (RT_KNN_HBITS) / below-window count in a register (RT_KNN_LOREG), C5
set -o pipefail
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C5 --names hb16,hb16lo,hb8,hb8s12,hb8s13,hb16,hb8,hb8s12 --iters 3 --save /tmp/r05m > $OUT/sweep_c5.log 2>&1 && \
python3 - > $OUT/compare.log 2>&1 <<'PY'
import numpy as np
a = np.load("/tmp/r05m/hb16_C5.npz")
for n in ["hb16lo", "hb8", "hb8s12", "hb8s13"]:
    b = np.load(f"/tmp/r05m/{n}_C5.npz")
    d = np.abs(a["rgb"].astype(np.float64) - b["rgb"].astype(np.float64))
    print(n, "max|d| rgb", float(d.max()), "pixels differing", int((d.max(axis=-1) > 0).sum()),
          "argb differing", int((a["argb"] != b["argb"]).sum()))
PY
