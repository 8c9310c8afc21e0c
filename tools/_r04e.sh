set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 300 python3 tools/wf_debug.py plnts3ColsBunnies.cli 256 64 default > $O/wf_debug_256.log 2>&1 && \
DISTRAYTRACER_WF_CHUNK=65536 timeout -k 10 300 python3 tools/wf_debug.py plnts3ColsBunnies.cli 256 64 default > $O/wf_debug_256_chunk.log 2>&1 && \
bash tools/pmc_variants.sh r04e/pmcv C3 base,nf0,an0,nfan0 && \
timeout -k 10 400 python3 tools/variant_sweep.py run --cfg C5 --names base,kd1 --iters 2 > $O/sweep_c5.log 2>&1 && \
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C3 --names base,ld1 --iters 10 > $O/sweep_c3.log 2>&1 && \
DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_kd1.so timeout -k 10 200 python3 tools/band_timing.py 8 C5 --tiles --worlds 8 > $O/bt_c5_kd1.log 2>&1 && \
timeout -k 10 300 python3 tools/band_timing.py 8 C5 --tiles --worlds 8 --flags 8 > $O/bt_c5_shc.log 2>&1 && \
DISTRAYTRACER_LIB=$PWD/tools/_variants/lib_ld1.so timeout -k 10 200 python3 tools/band_timing.py 8 C3 --tiles --worlds 8 > $O/bt_c3_ld1.log 2>&1
