#!/bin/bash
# round 6: fp32 box pre-test in the reference-order closest hit of the transparent variants (cpk) vs
# fp64 only (cpk0), and without it in the photon variant (cpkph0); alternating, same box
set -o pipefail
OUT=gpurun_out/r06n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/variant_sweep.py run --names cpk0,cpk,cpk0,cpk --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1 && \
timeout -k 10 900 python3 tools/variant_sweep.py run --names cpk0,cpk,cpkph0,cpk0,cpk,cpkph0 --cfg C5 --iters 5 > $OUT/ab_c5.log 2>&1 && \
timeout -k 10 400 python3 tools/variant_sweep.py run --names cpk0,cpk --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1
echo "exit $?" >> $OUT/status.txt
