#!/bin/bash
# final build: C4 / C5 profiles + PMC passes, then their bench lines with those summaries
set -o pipefail
OUT=gpurun_out/r06zd
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_prof_cfg.sh C4 r06zd/c4 2 && bash tools/gpu_prof_cfg.sh C5 r06zd/c5 3 && \
BENCH_TRAFFIC_JSON=$OUT/c5/pmc.json timeout -k 10 300 python3 bench.py --config C5 --no-cpu-baseline --steps 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err && \
BENCH_TRAFFIC_JSON=$OUT/c4/pmc.json timeout -k 10 400 python3 bench.py --config C4 --no-cpu-baseline --steps 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
echo "exit $?" >> $OUT/status.txt
