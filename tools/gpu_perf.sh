#!/bin/bash
# Tuning session on the GPU box: sweep of tools/_variants builds + one PMC pass of the default build.
set -o pipefail
TAG=${1:-perf}
NAMES=${2:-w2,w3,w4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/variant_sweep.py run --names $NAMES > $OUT/sweep.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq -o run -- python3 tools/variant_sweep.py one --iters 1 > $OUT/pmc_sq.log 2>&1
rc=$?
echo "chain exit $rc" >> $OUT/status.txt
exit $rc
