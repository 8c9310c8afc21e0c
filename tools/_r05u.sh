#!/bin/bash
# round 5: C3 N = 8 emulated step vs the plan's heavy-tile threshold (finer split of the costliest waves)
set -o pipefail
OUT=gpurun_out/r05u
mkdir -p $OUT
export TMPDIR=/tmp
for h in 1.0 1.25 1.5 1.0x 1.25x 1.5x; do
  timeout -k 10 300 python3 tools/group_overhead.py --config C3 --world 8 --rebalance 3 --heavy ${h%x} --out $OUT/c3_n8_heavyc$h.json > $OUT/c3_n8_heavyc$h.log 2>&1 || exit 1
done
