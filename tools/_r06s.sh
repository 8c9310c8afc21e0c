#!/bin/bash
# round 6 final build (pack on the exchange stream): full GPU suite, smoke, C3 profile + PMC passes, C3/C4/C5 bench lines, C4/C5 profiles
set -o pipefail
OUT=gpurun_out/r06s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
bash tools/gpu_prof_cfg.sh C3 r06s/c3 20 && \
timeout -k 10 300 python3 bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err && \
timeout -k 10 300 python3 bench.py --config C5 --no-cpu-baseline --steps 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err && \
timeout -k 10 400 python3 bench.py --config C4 --no-cpu-baseline --steps 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err && \
bash tools/gpu_prof_cfg.sh C4 r06s/c4 2 && bash tools/gpu_prof_cfg.sh C5 r06s/c5 3
echo "exit $?" >> $OUT/status.txt
