#!/bin/bash
# top-level identity-CTM entries transformed by xid (exact adds) instead of xpt / xvec: C3 same-box A/B
# (old = the in-tree build fe57cc3a, head = xid, xi0 = this source with RT_XF_IDENT=0), the parity and
# KAT GPU tests on head, C4 / C5 A/B
set -o pipefail
OUT=gpurun_out/r06zf
mkdir -p $OUT
export TMPDIR=/tmp
V=tools/_ab
timeout -k 10 400 python3 tools/variant_sweep.py run --dir $V --names old,head,xi0,old,head,xi0 --cfg C3 --iters 20 > $OUT/ab_c3.log 2>&1 && \
DISTRAYTRACER_LIB=$V/lib_head.so timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_kats.py tests/test_refpin.py -m gpu > $OUT/pytest_parity_head.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --dir $V --names old,head,old,head --cfg C5 --iters 5 > $OUT/ab_c5.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --dir $V --names old,head --cfg C4 --iters 3 > $OUT/ab_c4.log 2>&1
echo "exit $?" >> $OUT/status.txt
