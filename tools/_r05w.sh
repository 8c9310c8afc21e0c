#!/bin/bash
# round 5: approximate box test as lane masks (RT_APX2) and lane bits by inverse ballot (RT_INV_BALLOT), C3 / C4 / C5
set -o pipefail
OUT=gpurun_out/r05w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C3 --names apx0,apx1,ib1,ib1apx1,apx0,apx1,ib1,ib1apx1 --iters 20 > $OUT/sweep_c3.log 2>&1 && \
timeout -k 10 900 python3 tools/variant_sweep.py run --cfg C4 --names apx0,ib1apx1,apx0,ib1apx1 --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names apx0,ib1apx1,apx0,ib1apx1 --iters 3 > $OUT/sweep_c5.log 2>&1
