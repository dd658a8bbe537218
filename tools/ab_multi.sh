#!/bin/bash
# tracer timing (tools/batch_bench.py, 32-frame batches of the bench frame) for the default
# libnr.so and each alternative build given: bash tools/ab_multi.sh build/a build/b ...
set -e
run() {
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 1,32 --shards 1,8
  [ -n "$FP32_ONLY" ] || timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 1,32 --shards 1,8 --precision bf16
}
echo "== default"; run
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so run; done
echo "== default (again)"; run
