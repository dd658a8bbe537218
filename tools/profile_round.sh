#!/bin/bash
# One GPU-box call that regenerates the round's committed evidence:
#   bench.json (the driver's bench line), a rocprofv3 --kernel-trace --stats pass of the
#   bench without its single-frame figure and with a warmup batch as long as the timed
#   one (so the batched k_trace launches averaged are the ones bench.py's per-launch
#   events time), and FETCH_SIZE / WRITE_SIZE in two
#   separate --pmc passes (gfx950 HBM correction applied by tools/traffic.py).
# usage (GPU box, repo root): bash tools/profile_round.sh TAG  ->  gpurun_out/prof_TAG/
set -e
TAG=${1:-r1}
REPO=$(pwd)
OUT=$(realpath -m "gpurun_out/prof_$TAG")
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run -- \
    python3 "$REPO/bench.py" --no-cpu-baseline --no-live-traffic --no-single-frame --no-random-poses --warmup 32 > "$OUT/ktrace_bench.json" 2> "$OUT/ktrace.err"
# the PMC passes drive the bench's batched kernel (32 frames per launch, bench default)
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$REPO/tools/render_frames.py" --frames 3 --batch 32 > "$OUT/fetch.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$REPO/tools/render_frames.py" --frames 3 --batch 32 > "$OUT/write.log" 2>&1
python3 "$REPO/tools/traffic.py" "$OUT" 32 > "$OUT/traffic.json"
cp "$OUT/traffic.json" "$REPO/gpurun_out/pmc_traffic_$TAG.json"
