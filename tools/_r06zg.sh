#!/bin/bash
# final build fe57cc3a: emulated N-rank group steps (one GPU, one rank at a time) and a 2-rank native
# rank-mode bench line over the host transport (gloo)
set -o pipefail
O=gpurun_out/r06zg
mkdir -p $O
export TMPDIR=/tmp
for w in 2 4 8; do
  timeout -k 10 200 python3 tools/group_overhead.py --config C3 --world $w --rebalance 3 --out $O/c3_n${w}_group_emulated.json > $O/go_c3_$w.log 2>&1 || { echo "exit $?" >> $O/status.txt; exit 1; }
done
timeout -k 10 300 python3 tools/group_overhead.py --config C5 --world 8 --rebalance 3 --iters 10 --out $O/c5_n8_group_emulated.json > $O/go_c5_8.log 2>&1 && \
timeout -k 10 400 python3 tools/group_overhead.py --config C4 --world 8 --rebalance 3 --iters 5 --out $O/c4_n8_group_emulated.json > $O/go_c4_8.log 2>&1 && \
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/bench_c3_gloo2_rehearsal.json 2> $O/bench_gloo2.err
echo "exit $?" >> $O/status.txt
