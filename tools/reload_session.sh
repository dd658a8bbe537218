#!/bin/bash
# Round 6: k_trace's arguments re-read from the kernarg segment per phase (NR_ARG_RELOAD=1, default
# build) against holding them across the loop (build/noreload: make EXTRA=-DNR_ARG_RELOAD=0), GPU box:
# parity / endgame / default-path tests on the default build, then bench.py and config_bench A/B/A.
#   bash tools/reload_session.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/reload}")
mkdir -p "$OUT"
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_endgame.py tests/test_gpu_configs_default.py \
    tests/test_gpu_lowp.py tests/test_gpu_fp32x3.py -x -v -s --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
run() {
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 2>&1 | grep '^{' || return 1
  timeout -k 10 300 python -u tools/config_bench.py --frames 6 --only C3,C4-full,C5 --endgame 0,0.001 2>&1 | grep '^{' || return 1
}
echo "== default (reload)" > "$OUT/ab.log"; run >> "$OUT/ab.log" || exit 1
echo "== noreload" >> "$OUT/ab.log"; NR_LIBRARY=$PWD/build/noreload/libnr.so run >> "$OUT/ab.log" || exit 1
echo "== default (reload, again)" >> "$OUT/ab.log"; run >> "$OUT/ab.log" || exit 1
