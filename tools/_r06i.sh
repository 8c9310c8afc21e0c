#!/bin/bash
# round 6: C4 and C5 profiles + PMC passes (incl. VALU classes) of the final kernel build
set -o pipefail
OUT=gpurun_out/r06i
mkdir -p $OUT
bash tools/gpu_prof_cfg.sh C4 r06i/c4 2 && bash tools/gpu_prof_cfg.sh C5 r06i/c5 3
echo "exit $?" >> $OUT/status.txt
