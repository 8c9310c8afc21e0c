#!/bin/bash
# round 6: same-box alternating A/B of the fp32 box pre-test (f320 off / f32def default) on C4 and C3,
# then C3's profile + PMC passes (incl. the VALU classes) of the default build
set -o pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --names f320,f32def,f320,f32def --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1 && \
timeout -k 10 400 python3 tools/variant_sweep.py run --names f320,f32def,f320,f32def --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1 && \
bash tools/gpu_prof_cfg.sh C3 r06h/c3 20
echo "exit $?" >> $OUT/status.txt
