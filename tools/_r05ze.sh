#!/bin/bash
# round 5 final build: divergent-gather lane-wise scans (RT_KNN_DIV) re-checked on C5
set -o pipefail
OUT=gpurun_out/r05ze
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names fin,kd0,fin,kd0 --iters 3 > $OUT/sweep_c5.log 2>&1
