#!/bin/bash
# round 6 final build (c31eeff2): C4 and C5 profiles + PMC passes
set -o pipefail
OUT=gpurun_out/r06m
mkdir -p $OUT
bash tools/gpu_prof_cfg.sh C4 r06m/c4 2 && bash tools/gpu_prof_cfg.sh C5 r06m/c5 3
echo "exit $?" >> $OUT/status.txt
