#!/bin/bash
# round-4 A/B: a finished sample's colour in LDS (reslds) vs the frame-late build (flate)
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C3 --names flate,reslds,reslds0,flate,reslds --iters 10 > $O/c3.log 2>&1 && \
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C4 --names flate,reslds,c4mr --iters 2 > $O/c4.log 2>&1 && \
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C5 --names flate,reslds --iters 2 > $O/c5.log 2>&1 && \
bash tools/pmc_variants.sh r04z/c3pmc C3 reslds && \
bash tools/pmc_variants.sh r04z/c4pmc C4 reslds && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $O/parity.log 2>&1
