#!/bin/bash
# bf16/fp16 tracer timing (tools/batch_bench.py: one-frame and 32-frame launches of the bench
# frame, 1 and 8 shards) for the default libnr.so and each alternative build given:
#   bash tools/ab_lowp.sh build/a build/b ...
set -e
run() {
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 1,32 --shards 1,8 --precision bf16 2>&1 | grep -v amdgpu.ids
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 32 --shards 1 --precision fp16 2>&1 | grep -v amdgpu.ids
}
echo "== default"; run
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so run; done
echo "== default (again)"; run
