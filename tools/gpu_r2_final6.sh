# after the k_mlp16 register target change: every GPU test and the fp32/bf16 counter passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_final6.log 2>&1 && \
tail -2 gpurun_out/gputests_final6.log && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_fp32_r2h fp32 8 > gpurun_out/pmc_fp32_r2h.txt 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16_r2h bf16 8 > gpurun_out/pmc_bf16_r2h.txt 2>&1
