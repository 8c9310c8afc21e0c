#!/bin/bash
# round 6: VALU issue probe (more classes), available VALU counters, A/B of the uniform-opaque
# change (uo0 = round 5's hoisting) on C3 / C4 / C5, and C3's profile + PMC passes of the new build
set -o pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 tools/valu_issue > $OUT/valu_issue.json && \
(timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1; true) && \
timeout -k 10 400 python3 tools/variant_sweep.py run --names head,uo0 --cfg C3 --iters 10 > $OUT/ab_c3.log 2>&1 && \
timeout -k 10 400 python3 tools/variant_sweep.py run --names head,uo0 --cfg C5 --iters 5 > $OUT/ab_c5.log 2>&1 && \
timeout -k 10 500 python3 tools/variant_sweep.py run --names head,uo0 --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1 && \
bash tools/gpu_prof_cfg.sh C3 r06d/c3 20
echo "exit $?" >> $OUT/status.txt
