#!/bin/bash
# Round 6: the endgame instances' shading normals as one two-tile fp32x3 pass (build/x3eg2: make
# EXTRA=-DNR_X3N_ONE_EG=0) against two one-tile passes (default), GPU box: endgame tests on the A/B
# build, then config_bench C3, C4-full, C5 at the default endgame, A/B/A.
#   bash tools/ab_x3n_session.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/x3n}")
mkdir -p "$OUT"
NR_LIBRARY=$PWD/build/x3eg2/libnr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_endgame.py -x -q --timeout 200 \
  --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
cb() { timeout -k 10 300 python -u tools/config_bench.py --frames 6 --only C3,C4-full,C5 --endgame 0.001 2>&1 | grep '^{'; }
echo "== default (one-tile passes)" > "$OUT/ab.log"; cb >> "$OUT/ab.log" || exit 1
echo "== x3eg2 (two-tile pass)" >> "$OUT/ab.log"; NR_LIBRARY=$PWD/build/x3eg2/libnr.so cb >> "$OUT/ab.log" || exit 1
echo "== default (again)" >> "$OUT/ab.log"; cb >> "$OUT/ab.log" || exit 1
