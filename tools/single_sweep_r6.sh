#!/bin/bash
# Round 6: fp32 single frames (plane_1 1024^2, one nr_render_shard launch per frame) over the runtime knobs.
set -o pipefail
b() { timeout -k 10 120 python -u tools/batch_bench.py --frames 16 --batches 1 --shards 1 --single "$@" 2>&1 | grep -v amdgpu.ids; }
b || exit 1
for r in 16 32 48 64; do b --rays $r || exit 1; done
for sp in 0 1 4 16; do b --spread $sp || exit 1; done
for q in 4 16; do b --queues $q || exit 1; done
b || exit 1
