#!/bin/bash
# fp32 tracer timing (tools/batch_bench.py: one-frame (nr_render_batch and nr_render_shard) and
# 20-frame launches of the bench frame
# -- the driver's --steps 20 shape -- at 1 and 8 shards) for the default libnr.so and each
# alternative build given:  bash tools/ab_fp32.sh build/a build/b ...
set -e
run() {
  timeout -k 10 120 python tools/batch_bench.py --frames 40 --batches 1,20 --shards 1,8 2>&1 | grep -v amdgpu.ids
  timeout -k 10 120 python tools/batch_bench.py --frames 40 --batches 1 --shards 1,8 --single 2>&1 | grep -v amdgpu.ids
}
echo "== default"; run
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so run; done
echo "== default (again)"; run
