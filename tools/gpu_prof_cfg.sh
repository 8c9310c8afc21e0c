#!/bin/bash
# Profile one bench config on the GPU box: rocprofv3 kernel trace + stats of bench.py, then one
# PMC pass per counter group (FETCH_SIZE / WRITE_SIZE / SQ occupancy+issue), each its own run
# with its own time limit, chained with && (the first failure ends the script).
#   tools/gpu_prof_cfg.sh CFG TAG [STEPS]
set -o pipefail
CFG=${1:-C4}
TAG=${2:-prof}
STEPS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $B > $OUT/prof.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $B > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $B > $OUT/pmc_write.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq -o run -- python3 $B > $OUT/pmc_sq.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 --output-format csv -d $OUT/pmc_mem -o run -- python3 $B > $OUT/pmc_mem.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT --output-format csv -d $OUT/pmc_valu -o run -- python3 $B > $OUT/pmc_valu.log 2>&1
rc=$?
WL=$(python3 -c "import sys; sys.path.insert(0, '.'); from distraytracer_old_amd import scenes; c, W, H, s, _ = scenes.CONFIGS['$CFG']; print(f'$CFG {c} {W}x{H} {s}spp')")
[ $rc -eq 0 ] && python3 tools/pmc_table.py $OUT --workload "$WL" --json $OUT/pmc.json > /dev/null
echo "prof $CFG exit $rc" >> $OUT/status.txt
exit $rc
