set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile_round.sh r2f > gpurun_out/profile_round_r2f.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_fp32_r2f fp32 8 > gpurun_out/pmc_fp32_r2f.txt 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16_r2f bf16 8 > gpurun_out/pmc_bf16_r2f.txt 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --frames 5 > gpurun_out/cfg_final.log 2>&1
