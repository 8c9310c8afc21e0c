#!/bin/bash
# round 6: nearest-first closest hit with the fp32 ray rebuilt per node (nflz) vs held (head), C3
set -o pipefail
OUT=gpurun_out/r06u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --names head,nflz,head,nflz,head,nflz --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1
echo "exit $?" >> $OUT/status.txt
