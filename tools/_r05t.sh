#!/bin/bash
# round 5: the exact slab fallback as a real call (RT_SLAB_CALL) A/B on C3 / C4 / C5
set -o pipefail
OUT=gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C3 --names sc0,sc1,sc0,sc1 --iters 20 > $OUT/sweep_c3.log 2>&1 && \
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C4 --names sc0,sc1 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names sc0,sc1 --iters 3 > $OUT/sweep_c5.log 2>&1
