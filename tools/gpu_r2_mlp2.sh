set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lowp.py -k "mlp or clamp or simpleinfer" -x -q --timeout 200 --timeout-method thread > gpurun_out/mlp2_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/mlp_bench.py --precision fp32,bf16,fp16 --bpc 8 --iters 20 --n 16777216 > gpurun_out/mlp2.log 2>&1
