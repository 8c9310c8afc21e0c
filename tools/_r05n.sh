#!/bin/bash
# round 5: kNN counting histogram 128 u8 buckets (RT_KNN_H8), minimal edit, C5
set -o pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C5 --names h8off,h8on,h8s12,h8s13,h8off,h8on,h8s12 --iters 3 --save /tmp/r05n > $OUT/sweep_c5.log 2>&1 && \
python3 - > $OUT/compare.log 2>&1 <<'PY'
import numpy as np
a = np.load("/tmp/r05n/h8off_C5.npz")
for n in ["h8on", "h8s12", "h8s13"]:
    b = np.load(f"/tmp/r05n/{n}_C5.npz")
    d = np.abs(a["rgb"].astype(np.float64) - b["rgb"].astype(np.float64))
    print(n, "max|d| rgb", float(d.max()), "pixels differing", int((d.max(axis=-1) > 0).sum()),
          "argb differing", int((a["argb"] != b["argb"]).sum()))
PY
