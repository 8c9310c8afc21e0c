#!/bin/bash
# round 5: LDS per-pixel sums / finished colours in the transparent variants (C4, C5) + C4 writes
set -o pipefail
OUT=gpurun_out/r05z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python3 tools/variant_sweep.py run --cfg C4 --names tl0,tlsum,tlres,tlboth,tl0,tlres,tlboth --iters 2 > $OUT/sweep_c4.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names tl0,tlsum,tl0,tlsum --iters 3 > $OUT/sweep_c5.log 2>&1 && \
bash tools/pmc_variants.sh r05z C4 tl0,tlres,tlboth
