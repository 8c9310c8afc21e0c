#!/bin/bash
# fp32 triangle edge pre-test: GPU parity (product library) then same-box A/B against RT_F32_TRI=0
set -o pipefail
OUT=gpurun_out/r06w; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_parity.log 2>&1 && \
timeout -k 10 400 python3 tools/variant_sweep.py run --names tri0,head,tri0,head,tri0,head --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1 && \
timeout -k 10 400 python3 tools/variant_sweep.py run --names tri0,head,tri0,head --cfg C4 --iters 2 > $OUT/ab_c4.log 2>&1
