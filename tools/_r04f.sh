set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 300 python3 tools/wf_debug.py plnts3ColsBunnies.cli 2048 4,64 default > $O/wf_debug_2048.log 2>&1 && \
timeout -k 10 300 python3 tools/wf_debug.py plnts3ColsBunnies.cli 1024 64 default > $O/wf_debug_1024.log 2>&1 && \
timeout -k 10 600 python3 tools/variant_sweep.py run --cfg C5 --names base,kd1,kd1f4,kd1f1,kd1r4,kd1r1 --iters 2 > $O/sweep_c5.log 2>&1 && \
for v in kd1 kd1f4 kd1f1 kd1r4 kd1r1; do DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_$v.so timeout -k 10 200 python3 tools/band_timing.py 8 C5 --tiles --worlds 8 > $O/bt_c5_$v.log 2>&1 || exit 1; done
