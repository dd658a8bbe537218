#!/bin/bash
# Round 6: the fp32 one-tile MLP's hidden layers as the generated stream in the
# tracers (build/f32stream: make EXTRA=-DNR_F32_STREAM=1) against the compiled loop (the default build
# since this A/B; run as measured, the default build was the stream one), GPU box: the fp32
# parity / fuzz tests, the lone-wave MLP latency (tools/mlp_latency.py), then bench.py A/B/A (the
# batched headline, config.single_frame and config.spin).
#   bash tools/f32_stream_session.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/f32s}")
mkdir -p "$OUT"
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_golden.py -x -q \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
timeout -k 10 240 python -u tools/mlp_latency.py > "$OUT/latency.log" 2>&1 || exit 1
run() { timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 2>&1 | grep '^{'; }
echo "== stream" > "$OUT/ab.log"; NR_LIBRARY=$PWD/build/f32stream/libnr.so run >> "$OUT/ab.log" || exit 1
echo "== default (loop)" >> "$OUT/ab.log"; run >> "$OUT/ab.log" || exit 1
echo "== stream (again)" >> "$OUT/ab.log"; NR_LIBRARY=$PWD/build/f32stream/libnr.so run >> "$OUT/ab.log" || exit 1
