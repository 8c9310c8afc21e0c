#!/bin/bash
# Build the headless driver tools/rtrender against the in-tree libdistraytracer.so (rpath $ORIGIN-relative).
set -e
cd "$(dirname "$0")/.."
python3 -m distraytracer_old_amd.build > /dev/null
g++ -O2 -std=c++17 tools/rtrender.cpp -o tools/rtrender -Ldistraytracer_old_amd/lib -ldistraytracer -lz \
    -Wl,-rpath,'$ORIGIN/../distraytracer_old_amd/lib'
echo tools/rtrender
