#!/bin/bash
# GPU box: the final layer on the matrix core (this tree) vs v_dot2c (build/olddot2): the -m gpu suite on
# this tree, then k_mlp16 (2^22 / 2^24 / 2^26) and C3 / C5 (pure 16-bit march) for both libraries.
set -o pipefail
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests_final_layer.log 2>&1 &&
LIBS="default build/olddot2 default" PRECS=bf16,fp16 BPC=0 SIZES="4194304 16777216 67108864" bash tools/ab_mlp.sh final_layer &&
timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0 > $O/cfg_fl_new.txt 2>&1 &&
NR_LIBRARY=$PWD/build/olddot2/libnr.so timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0 > $O/cfg_fl_old.txt 2>&1 &&
timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0 > $O/cfg_fl_new2.txt 2>&1
