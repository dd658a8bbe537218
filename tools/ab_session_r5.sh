#!/bin/bash
# GPU box: round-5 late A/Bs in one call -- the group tests, 3 vs 4 workgroups per CU for the
# low-precision tracers (build/lowp3), and the fp32 tracer's age priority (build/age16, build/age40)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -m gpu -v --timeout 120 --timeout-method thread > $O/group_tests_r5e.log 2>&1 &&
bash tools/ab_age.sh build/age16 build/age40 > $O/ab_age.txt 2>&1 &&
timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0 > $O/cfg_lowp3_default.txt 2>&1 &&
NR_LIBRARY=$PWD/build/lowp3/libnr.so timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0 > $O/cfg_lowp3_alt.txt 2>&1 &&
timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0 > $O/cfg_lowp3_default2.txt 2>&1
