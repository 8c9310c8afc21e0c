#!/bin/bash
# final build with the fp32 triangle pre-test: full GPU suite, smoke, C3 profile + PMC passes, C3 bench line
set -o pipefail
OUT=gpurun_out/r06zc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
bash tools/gpu_prof_cfg.sh C3 r06zc/c3 20 && \
BENCH_TRAFFIC_JSON=$OUT/c3/pmc.json timeout -k 10 300 python3 bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err
echo "exit $?" >> $OUT/status.txt
