#!/bin/bash
# One GPU evidence session: smoke -> rocprofv3 kernel trace -> rocprofv3 FETCH_SIZE pass ->
# PMC summary -> bench (N=1, with that summary as its traffic source) -> pytest -m gpu.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the chain.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
WL="C3 c3_bun69k.cli 1024x1024 16spp"
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc.log 2>&1 && \
python3 tools/pmc_summary.py $OUT/prof/run_kernel_stats.csv $OUT/pmc/run_counter_collection.csv "$WL" $OUT/c3_pmc.json > $OUT/pmc_summary.log 2>&1 && \
BENCH_TRAFFIC_JSON=$OUT/c3_pmc.json timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err && \
python3 tools/trace_durations.py $OUT/prof/run_kernel_trace.csv $OUT/c3_kernel_trace_durations.txt 10 > /dev/null 2>&1 && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err && \
timeout -k 10 300 python3 bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?
echo "chain exit $rc" >> $OUT/status.txt
exit $rc
