#!/bin/bash
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
for rb in 0 3 6; do
timeout -k 10 300 python -u tools/group_overhead.py --config C3 --rebalance $rb --out $O/c3_n8_rb$rb.json > $O/c3_n8_rb$rb.txt 2>&1 || exit 1
done
