set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mlp_bench.py --precision all --bpc 2,3,4 --iters 10 > gpurun_out/mlp_bench_r2.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16 bf16 3 > gpurun_out/pmc_bf16.txt 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_fp32 fp32 3 > gpurun_out/pmc_fp32.txt 2>&1
