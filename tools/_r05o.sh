#!/bin/bash
# round 5: kNN u8 buckets + start-window change: the photon-gather GPU tests
set -o pipefail
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_knn_ties.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "knn or t11 or photon or C5 or c5 or gather or caustic" > $OUT/pytest.log 2>&1
