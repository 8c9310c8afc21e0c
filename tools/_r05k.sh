#!/bin/bash
# round 5: kNN start-window widening by density extrapolation (RT_KNN_EXTRAP) A/B on C5 + image compare
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C5 --names ex0,ex1s11,ex1s115,ex1s12,ex1s125,ex1s11,ex1s115,ex1s12 --iters 3 --save /tmp/r05k > $OUT/sweep_c5.log 2>&1 && \
python3 - > $OUT/compare.log 2>&1 <<'PY'
import numpy as np
a = np.load("/tmp/r05k/ex0_C5.npz")
for n in ["ex1s11", "ex1s115", "ex1s12", "ex1s125"]:
    b = np.load(f"/tmp/r05k/{n}_C5.npz")
    d = np.abs(a["rgb"].astype(np.float64) - b["rgb"].astype(np.float64))
    print(n, "max|d| rgb", float(d.max()), "pixels differing", int((d.max(axis=-1) > 0).sum()),
          "argb differing", int((a["argb"] != b["argb"]).sum()))
PY
