#!/bin/bash
# round 6: the shadow fp32 pre-test's ray rebuilt per node (lz, default) vs held (lz0), and in C3's
# opaque variant too (lzop); alternating, same box
set -o pipefail
OUT=gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/variant_sweep.py run --names lz0,lz,lzop,lz0,lz,lzop --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1 && \
timeout -k 10 900 python3 tools/variant_sweep.py run --names lz0,lz,lz0,lz --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --names lz0,lz,lz0,lz --cfg C5 --iters 5 > $OUT/ab_c5.log 2>&1
echo "exit $?" >> $OUT/status.txt
