#!/bin/bash
# round 5: slim shading-tree frames (RT_FRAME_SLIM) A/B on C4 / C5 (time, image) + C4 writes (PMC)
set -o pipefail
OUT=gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C4 --names slim0,slim1,slim0,slim1 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names slim0,slim1,slim0,slim1 --iters 3 > $OUT/sweep_c5.log 2>&1 && \
bash tools/pmc_variants.sh r05q C4 slim0,slim1
