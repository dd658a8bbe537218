#!/bin/bash
# Round 6: the endgame instances as 12-wave workgroups with the fp32x3 pack in LDS (default build)
# against round 5's 4-wave form (build/eg4: make EXTRA=-DNR_EG_WAVES=4), GPU box:
# the endgame / parity tests on the default build, then config_bench C3, C4-full, C5 A/B/A.
#   bash tools/eg_waves_session.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/egw}")
mkdir -p "$OUT"
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_endgame.py tests/test_gpu_parity.py tests/test_gpu_x3_normals.py \
    tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
cb() { timeout -k 10 300 python -u tools/config_bench.py --frames 6 --only C3,C4-full,C5 --endgame 0.001; }
echo "== default (12 waves)" > "$OUT/ab.log"; cb >> "$OUT/ab.log" 2>&1 || exit 1
echo "== eg4" >> "$OUT/ab.log"; NR_LIBRARY=$PWD/build/eg4/libnr.so cb >> "$OUT/ab.log" 2>&1 || exit 1
echo "== default (12 waves, again)" >> "$OUT/ab.log"; cb >> "$OUT/ab.log" 2>&1 || exit 1
