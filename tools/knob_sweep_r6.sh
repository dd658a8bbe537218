#!/bin/bash
# Round 6: the fp32 bench batch (plane_1 1024^2, 32 frames per launch) over the runtime knobs after this
# round's register changes: pixel-queue shards, pixel spread, rays per wave (tools/batch_bench.py).
set -o pipefail
b() { timeout -k 10 120 python -u tools/batch_bench.py --frames 32 --batches 32 --shards 1 "$@" 2>&1 | grep -v amdgpu.ids; }
b || exit 1
for q in 4 16 32; do b --queues $q || exit 1; done
for sp in 0 1 4 16 64; do b --spread $sp || exit 1; done
for rays in 32 48; do b --rays $rays || exit 1; done
b || exit 1
