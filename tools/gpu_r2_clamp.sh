set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lowp_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 2,3,4 --iters 10 > gpurun_out/mlp_clamp.log 2>&1 && \
timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16 --bpc 2,3,4 --iters 10 --debug 512 >> gpurun_out/mlp_clamp.log 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 > gpurun_out/cfg_clamp.log 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 --debug 512 >> gpurun_out/cfg_clamp.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
