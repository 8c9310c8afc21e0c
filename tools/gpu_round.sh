#!/bin/bash
# One GPU evidence session (tag = round + letter, e.g. r02s):
#   part 1: smoke -> pytest -m gpu -> per-config rocprofv3 kernel trace + PMC passes (tools/gpu_prof_cfg.sh)
#   part 2: bench lines (C3 with the CPU baseline, C4, C5) reading those PMC summaries
# Every GPU step has its own time limit; steps are chained with && so a failure stops the chain.
#   tools/gpu_round.sh TAG [1|2|all]
set -o pipefail
TAG=${1:-r02}
PART=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
if [ "$PART" = 1 ] || [ "$PART" = all ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
  bash tools/gpu_prof_cfg.sh C3 $TAG/c3 10 && \
  bash tools/gpu_prof_cfg.sh C4 $TAG/c4 2 && \
  bash tools/gpu_prof_cfg.sh C5 $TAG/c5 2 || rc=$?
fi
if [ $rc -eq 0 ] && { [ "$PART" = 2 ] || [ "$PART" = all ]; }; then
  for c in c3 c4 c5; do [ -f $OUT/$c/pmc.json ] && cp $OUT/$c/pmc.json profiles/${TAG}_${c}_pmc.json; done
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err && \
  timeout -k 10 300 python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err && \
  timeout -k 10 300 python3 bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || rc=$?
fi
echo "chain exit $rc" >> $OUT/status.txt
exit $rc
