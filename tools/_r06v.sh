#!/bin/bash
# wave-level triangle hit rates (profiling build, counting kernel): C3
set -o pipefail
OUT=gpurun_out/r06v; mkdir -p $OUT
DISTRAYTRACER_LIB=tools/_variants/lib_pkstat.so timeout -k 10 300 python3 tools/pkstat.py C3 > $OUT/pkstat_c3.json 2> $OUT/pkstat_c3.err
