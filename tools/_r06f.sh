#!/bin/bash
# round 6: A/B of the fp32 box pre-test (f32all default, f32nf closest-hit only, f32nt not in the
# transparent variants' shadow rays, f320 off) on C3 / C5 / C4, same image hash required
set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/variant_sweep.py run --names f320,f32all,f32nf,f320,f32all --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1 && \
timeout -k 10 500 python3 tools/variant_sweep.py run --names f320,f32all,f32nf,f32nt --cfg C5 --iters 5 > $OUT/ab_c5.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --names f320,f32all,f32nf,f32nt --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1
echo "exit $?" >> $OUT/status.txt
