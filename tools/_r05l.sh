#!/bin/bash
# round 5: C5 region profile after the kNN start-window change (passes per gather call)
set -o pipefail
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
DISTRAYTRACER_LIB=tools/_variants/lib_regions.so timeout -k 10 600 python3 tools/regions.py C5 > $OUT/c5_regions.json 2> $OUT/c5_regions.err
