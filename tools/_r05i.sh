#!/bin/bash
# round 5: wave-uniform leaf transforms / light fields as scalar loads (RT_ULOAD) A/B on C4, C5, C3
set -o pipefail
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C4 --names uload0,uload1,uload2,uload3,uload0,uload3 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names uload0,uload3,uload0,uload3 --iters 3 > $OUT/sweep_c5.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C3 --names uload0,uload3,uload0,uload3 --iters 20 > $OUT/sweep_c3.log 2>&1
