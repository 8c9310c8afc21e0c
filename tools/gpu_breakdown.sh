#!/bin/bash
# Time breakdown by profiling builds (tools/variant_sweep.py) + per-build memory-instruction /
# HBM-write PMC pass, on the GPU box.
#   tools/gpu_breakdown.sh TAG CFGS NAMES PMC_NAMES
set -o pipefail
TAG=${1:-brk}
CFGS=${2:-C3}
NAMES=${3:-notrace,noshade,primary,nosec,noshadow,nophong}
PMC_NAMES=${4:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for c in ${CFGS//,/ }; do
  timeout -k 10 900 python3 tools/variant_sweep.py run --cfg $c --names $NAMES --iters 2 >> $OUT/sweep.log 2>&1 || { rc=$?; break; }
done
for n in ${PMC_NAMES//,/ }; do
  [ $rc -ne 0 ] && break
  if [ "$n" = default ]; then unset DISTRAYTRACER_LIB; else export DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_$n.so; fi
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_SMEM --output-format csv -d $OUT/pmc_wr_$n -o run -- python3 tools/variant_sweep.py one --iters 1 > $OUT/pmc_wr_$n.log 2>&1 || rc=$?
done
echo "chain exit $rc" >> $OUT/status.txt
exit $rc
