#!/bin/bash
# HBM traffic and GB/s of the wavefront march kernel (k_march16), as north_star asks ("rocprof
# showing achieved HBM GB/s for the march"): C2 (plane_1 1024^2, 128 steps, fp32) on the
# wavefront schedule, BATCH frames per nr_render_batch call.  Three runs of the same program:
# a kernel trace (per-dispatch durations) and one --pmc pass each for FETCH_SIZE and
# WRITE_SIZE (they cannot share a pass); tools/march_traffic.py joins them per dispatch.
# usage (GPU box, repo root): bash tools/march_traffic.sh OUTDIR [batch] [precision]
set -e
OUT=$(realpath -m "$1"); BATCH=${2:-8}; PREC=${3:-fp32}
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--frames 2 --batch $BATCH --schedule wavefront --precision $PREC"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/tools/render_frames.py" $ARGS > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$REPO/tools/render_frames.py" $ARGS > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$REPO/tools/render_frames.py" $ARGS > "$OUT/write.log" 2>&1
python3 "$REPO/tools/march_traffic.py" "$OUT" "$BATCH" "$PREC"
