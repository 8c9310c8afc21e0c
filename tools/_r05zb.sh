#!/bin/bash
# round 5: on the final build -- mask ops in every variant (RT_MASKOPS=2), XCD-hashed deal (RT_XCD_HASH=4), C4 / C5
set -o pipefail
OUT=gpurun_out/r05zb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python3 tools/variant_sweep.py run --cfg C4 --names fin,mo2,xh4,mo2xh4,fin,mo2,xh4,mo2xh4 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names fin,mo2,xh4,fin,mo2,xh4 --iters 3 > $OUT/sweep_c5.log 2>&1
