#!/bin/bash
# round 5: measured rebalancing of the N-GPU plan (emulated on one GPU)
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread > $O/group.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/group_overhead.py --config C3 --out $O/c3_n8.json > $O/c3_n8.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/group_overhead.py --config C3 --rebalance 2 --out $O/c3_n8_rb2.json > $O/c3_n8_rb2.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/group_overhead.py --config C3 --rebalance 4 --out $O/c3_n8_rb4.json > $O/c3_n8_rb4.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/group_overhead.py --config C5 --iters 10 --rebalance 2 --out $O/c5_n8_rb2.json > $O/c5_n8_rb2.txt 2>&1 || exit 1
