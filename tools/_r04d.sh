set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 200 python3 tools/wf_debug.py > $O/wf_debug.log 2>&1 && \
timeout -k 10 200 python3 tools/slow_tiles.py C5 > $O/slow_c5.log 2>&1 && \
timeout -k 10 200 python3 tools/slow_tiles.py C3 > $O/slow_c3.log 2>&1 && \
timeout -k 10 120 python3 tools/ray_mix.py C4 > $O/mix_c4.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C4 --names base --iters 2 > $O/sweep_c4_base.log 2>&1 && \
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C4 --names base --iters 2 --flags 32 > $O/sweep_c4_wf.log 2>&1 && \
bash tools/pmc_variants.sh r04d/pmcv C3 base,nf0,an0,nfan0 && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_knn_ties.py tests/test_gpu_parity.py -k "knn or photon or c5 or gather or kdtree" -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
