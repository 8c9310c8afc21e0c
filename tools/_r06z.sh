#!/bin/bash
# photon variant's triangle pre-test switches (C5), and C3's kernel without the shading tree (nosample)
set -o pipefail
OUT=gpurun_out/r06z; mkdir -p $OUT
timeout -k 10 400 python3 tools/variant_sweep.py run --names tph00,head,tph11,tph00,head,tph11 --cfg C5 --iters 3 > $OUT/ab_c5.log 2>&1 && \
timeout -k 10 300 python3 tools/variant_sweep.py run --names nosample,head,nosample --cfg C3 --iters 20 > $OUT/nosample_c3.log 2>&1
