#!/bin/bash
# A/B/A of the default build against build/prev (the previous commit's tree), GPU box: bench.py (fp32 headline)
# and config_bench C3 / C5 (pure march and default endgame).   bash tools/ab_prev_session.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/abprev}")
mkdir -p "$OUT"
run() {
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-single-frame --no-cpu-baseline 2>&1 | grep '^{' || return 1
  timeout -k 10 300 python -u tools/config_bench.py --frames 6 --only C3,C5 --endgame 0,0.001 2>&1 | grep '^{' || return 1
}
echo "== new" > "$OUT/ab.log"; run >> "$OUT/ab.log" || exit 1
echo "== prev" >> "$OUT/ab.log"; NR_LIBRARY=$PWD/build/prev/libnr.so run >> "$OUT/ab.log" || exit 1
echo "== new (again)" >> "$OUT/ab.log"; run >> "$OUT/ab.log" || exit 1
