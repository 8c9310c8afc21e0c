#!/bin/bash
# persistent render launches (RT_PERSIST=1: resident grid, tiles from a ticket counter) vs the
# one-tile-per-workgroup launch: C3 same-box A/B (old = the in-tree build, head = this source without
# RT_PERSIST), the group tests on the persistent build, emulated C3 N = 8 group step, C5 / C4 A/B
set -o pipefail
OUT=gpurun_out/r06ze
mkdir -p $OUT
export TMPDIR=/tmp
V=tools/_ab
timeout -k 10 400 python3 tools/variant_sweep.py run --dir tools/_ab --names old,head,pers,old,head,pers --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1 && \
DISTRAYTRACER_LIB=$V/lib_pers.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_rank_mode.py -m gpu > $OUT/pytest_group_pers.log 2>&1 && \
DISTRAYTRACER_LIB=$V/lib_head.so timeout -k 10 200 python3 tools/group_overhead.py --config C3 --world 8 --rebalance 3 --out $OUT/c3_n8_head.json > $OUT/go_head.log 2>&1 && \
DISTRAYTRACER_LIB=$V/lib_pers.so timeout -k 10 200 python3 tools/group_overhead.py --config C3 --world 8 --rebalance 3 --out $OUT/c3_n8_pers.json > $OUT/go_pers.log 2>&1 && \
DISTRAYTRACER_LIB=$V/lib_head.so timeout -k 10 200 python3 tools/group_overhead.py --config C3 --world 8 --rebalance 3 --out $OUT/c3_n8_head2.json > $OUT/go_head2.log 2>&1 && \
DISTRAYTRACER_LIB=$V/lib_pers.so timeout -k 10 200 python3 tools/group_overhead.py --config C3 --world 8 --rebalance 3 --out $OUT/c3_n8_pers2.json > $OUT/go_pers2.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --dir tools/_ab --names old,pers,old,pers --cfg C5 --iters 5 > $OUT/ab_c5.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --dir tools/_ab --names old,pers --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1
echo "exit $?" >> $OUT/status.txt
