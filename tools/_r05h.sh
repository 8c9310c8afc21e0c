#!/bin/bash
# round 5: top-level implicit primitives as scalar loads (RT_SPRIM) A/B on C4 and C5, alternated
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C4 --names sprim0,sprim1,sprim2,sprim0,sprim1 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names sprim0,sprim2,sprim0,sprim2 --iters 3 > $OUT/sweep_c5.log 2>&1
