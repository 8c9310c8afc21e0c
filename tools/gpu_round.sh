#!/bin/bash
# One GPU session: smoke -> bench (N=1) -> rocprofv3 kernel trace -> rocprofv3 FETCH_SIZE pass.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the chain.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc.log 2>&1
rc=$?
echo "chain exit $rc" >> $OUT/status.txt
find $OUT -name "*.csv" | head -20 >> $OUT/status.txt
exit $rc
