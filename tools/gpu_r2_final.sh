set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile_round.sh r2c > gpurun_out/profile_round_r2c.log 2>&1 && \
timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 4,5,6,8 --iters 10 --n 16777216 > gpurun_out/mlp_final.log 2>&1 && \
timeout -k 10 200 python -u tools/mlp_bench.py --precision fp32 --bpc 4,8 --iters 10 --n 16777216 >> gpurun_out/mlp_final.log 2>&1
