#!/bin/bash
# Tuning session on the GPU box: sweep of tools/_variants builds + PMC passes.
#   tools/gpu_perf.sh TAG NAMES PASSES [PMC_NAMES]
# PASSES (comma list of sq, mem, tcp, fetch) run on the default build, or on each build of
# PMC_NAMES (tools/_variants/lib_<name>.so) when given.
set -o pipefail
TAG=${1:-perf}
NAMES=${2:-w2,w3,w4}
PASSES=${3:-sq}
PMC_NAMES=${4:-default}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
declare -A PMC
PMC[sq]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
PMC[mem]="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INST_LEVEL_VMEM SQ_IFETCH SQC_ICACHE_MISSES SQ_LEVEL_WAVES TCC_HIT_sum TCC_MISS_sum"
PMC[tcp]="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
PMC[fetch]="FETCH_SIZE"
rc=0
timeout -k 10 600 python3 tools/variant_sweep.py run --names $NAMES > $OUT/sweep.log 2>&1 || rc=$?
for n in ${PMC_NAMES//,/ }; do
  for p in ${PASSES//,/ }; do
    [ $rc -ne 0 ] && break 2
    if [ "$n" = default ]; then unset DISTRAYTRACER_LIB; else export DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_$n.so; fi
    timeout -k 10 300 rocprofv3 --pmc ${PMC[$p]} --output-format csv -d $OUT/pmc_${p}_$n -o run -- python3 tools/variant_sweep.py one --iters 1 > $OUT/pmc_${p}_$n.log 2>&1 || rc=$?
  done
done
echo "chain exit $rc" >> $OUT/status.txt
exit $rc
