#!/bin/bash
# round 5: C5 kNN final pass skipping subtrees below the window -- A/B + parity
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u tools/variant_sweep.py run --cfg C5 --names head,inner0,head,inner0 --iters 5 > $O/c5_inner_ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kats.py tests/test_gpu_knn_ties.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/kats_knn.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "photon or t11 or c5 or caustic or knn" > $O/parity_photon.log 2>&1 || exit 1
