# End-of-round evidence on the final build: every GPU test, smoke(), the bench + rocprof +
# PMC traffic (profile_round.sh), the fp32/bf16 counter passes and the C3-C5 configurations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_final.log 2>&1 && \
tail -2 gpurun_out/gputests_final.log && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 && \
timeout -k 10 900 bash tools/profile_round.sh r2g > gpurun_out/profile_round_r2g.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_fp32_r2g fp32 8 > gpurun_out/pmc_fp32_r2g.txt 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16_r2g bf16 8 > gpurun_out/pmc_bf16_r2g.txt 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --frames 5 > gpurun_out/cfg_final_r2g.log 2>&1
