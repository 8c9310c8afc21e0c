#!/bin/bash
# round 5 final build: emulated N = 8 (and 2 / 4 for C3) group steps on one MI355X, after 3 re-cuts
set -o pipefail
OUT=gpurun_out/r05y
mkdir -p $OUT
export TMPDIR=/tmp
for w in 2 4 8; do
  timeout -k 10 300 python3 tools/group_overhead.py --config C3 --world $w --rebalance 3 --out $OUT/c3_n$w.json > $OUT/c3_n$w.log 2>&1 || exit 1
done
timeout -k 10 600 python3 tools/group_overhead.py --config C5 --world 8 --rebalance 2 --iters 5 --warmup 1 --out $OUT/c5_n8.json > $OUT/c5_n8.log 2>&1 && \
timeout -k 10 900 python3 tools/group_overhead.py --config C4 --world 8 --rebalance 1 --iters 2 --warmup 1 --out $OUT/c4_n8.json > $OUT/c4_n8.log 2>&1
