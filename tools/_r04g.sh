set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/variant_sweep.py run --cfg C3 --names base,nfcode,base,nfcode --iters 20 > $O/sweep_c3_nfcode.log 2>&1 && \
bash tools/pmc_variants.sh r04g/pmcv C3 base,nfcode && \
timeout -k 10 300 python3 tools/variant_sweep.py one --cfg C4 --iters 2 --flags 32 > $O/c4_wf_time.log 2>&1 && \
timeout -k 10 300 python3 tools/variant_sweep.py one --cfg C4 --iters 2 > $O/c4_time.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4wf_w -o run -- python3 tools/frame_runner.py C4 2 32 > $O/c4wf_w.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4wf_f -o run -- python3 tools/frame_runner.py C4 2 32 > $O/c4wf_f.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4wf_k -o run -- python3 tools/frame_runner.py C4 2 32 > $O/c4wf_k.log 2>&1 && \
python3 tools/pmc_frame_sum.py $O/c4wf_w WRITE_SIZE 2 1024 > $O/c4wf_pmc.txt && python3 tools/pmc_frame_sum.py $O/c4wf_f FETCH_SIZE 2 2048 >> $O/c4wf_pmc.txt
