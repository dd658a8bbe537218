#!/bin/bash
# GPU box: the reduced-precision evidence on the final tracer -- the endgame / lowp contract tests,
# C3-C5 timings (pure and endgame), and the bf16 tracer's counters (pure and endgame).
set -o pipefail
O=gpurun_out
TAG=${1:-r5d}
timeout -k 10 900 python -u -m pytest tests/test_gpu_endgame.py tests/test_gpu_lowp_contract.py -m gpu -v --timeout 600 --timeout-method thread > $O/eg_tests_$TAG.log 2>&1 &&
timeout -k 10 400 python -u tools/config_bench.py --frames 5 --endgame 0,0.0003 > $O/cfg_$TAG.log 2>&1 &&
EG=0 timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_bf16_$TAG bf16 3 > $O/pmc_bf16_$TAG.txt 2>&1 &&
EG=0.0003 timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_bf16eg_$TAG bf16 3 > $O/pmc_bf16eg_$TAG.txt 2>&1
