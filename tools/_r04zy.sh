#!/bin/bash
# round-4 final multi-GPU plan timings (emulated on one GPU) and a 2-rank bench line over gloo
set -o pipefail
O=gpurun_out/r04zy
mkdir -p $O
timeout -k 10 240 python3 tools/band_timing.py 8 C3 --tiles --cut --heavy 1.25 --worlds 2,4,8 > $O/plan_c3.log 2>&1 && \
timeout -k 10 400 python3 tools/band_timing.py 8 C5 --tiles --cut --heavy 1.25 --worlds 2,4,8 > $O/plan_c5.log 2>&1 && \
timeout -k 10 600 python3 tools/band_timing.py 8 C4 --tiles --cut --heavy 1.25 --worlds 8 > $O/plan_c4.log 2>&1 && \
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err
