#!/bin/bash
# reduced-precision MLP change, A/B against build/old (the previous commit's libnr.so):
# accuracy on the KAT points, MLP microbench, tracer batch timing; GPU box.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lowp or c3 or c4 or c5 or smoke" > gpurun_out/lowp_tests.log 2>&1
echo "== new" > gpurun_out/lowp.log
timeout -k 10 60 python tools/lowp_error.py >> gpurun_out/lowp.log 2>&1
timeout -k 10 100 python tools/mlp_bench.py --n 67108864 --iters 5 --bpc 4,8 --precision all >> gpurun_out/lowp.log 2>&1
echo "== old" >> gpurun_out/lowp.log
NR_LIBRARY=$PWD/build/old/libnr.so timeout -k 10 100 python tools/mlp_bench.py --n 67108864 --iters 5 --bpc 4,8 --precision all >> gpurun_out/lowp.log 2>&1
bash tools/ab_lib.sh build/old > gpurun_out/ab_lowp.log 2>&1
