#!/bin/bash
# round 5: nearest-first grown-box entry as a lower bound from the exact box's slab values (RT_NF_LB), C3
set -o pipefail
OUT=gpurun_out/r05zc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C3 --names lb0,lb1,lb0,lb1,lb0,lb1 --iters 20 > $OUT/sweep_c3.log 2>&1
