#!/bin/bash
# Round 6, VERDICT r5 item 3: the endgame's fixed quality targets at a threshold, and the C3-C5 cost of
# thresholds 0 / 3e-4 / 1e-3 (GPU box).  bash tools/eg_session_r6.sh OUTDIR TAU
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/eg6}"); TAU=${2:-0.001}
mkdir -p "$OUT"
NR_TEST_EG_TAU=$TAU timeout -k 10 900 python -u -m pytest tests/test_gpu_lowp_contract.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/contract_$TAU.log" 2>&1 || exit 1
cp gpurun_out/lowp_contract.json "$OUT/lowp_contract_$TAU.json"
timeout -k 10 600 python -u tools/config_bench.py --frames 6 --only C3,C4-full,C5 --endgame 0,0.0003,0.001 \
  > "$OUT/cfg_tau.log" 2>&1 || exit 1
