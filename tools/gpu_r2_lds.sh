set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_threads.py -x -v --timeout 200 --timeout-method thread > gpurun_out/lds_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 2,3,4,5,6 --iters 10 --n 16777216 > gpurun_out/mlp_lds.log 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 > gpurun_out/cfg_lds.log 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 --bpc 2 >> gpurun_out/cfg_lds.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
