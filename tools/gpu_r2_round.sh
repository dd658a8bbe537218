set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_lowp_contract.py > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 900 bash tools/profile_round.sh r2b > gpurun_out/profile_round_r2b.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_fp32_r2b fp32 4 > gpurun_out/pmc_fp32_r2b.txt 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16_r2b bf16 6 > gpurun_out/pmc_bf16_r2b.txt 2>&1
