#!/bin/bash
# GPU box: one-frame launches of the bench frame (fp32 plane_1 1024^2, 128 steps) over workgroups
# per CU x rays per wave, and the temporal orders -- the single-frame tail's schedule knobs
set -o pipefail
for bpc in 2 3 4; do
  for rays in 0 48 32; do
    timeout -k 10 60 python -u tools/batch_bench.py --single --batches 1 --shards 1 --frames 40 --bpc $bpc --rays $rays || exit 1
  done
done
for t in 1 2; do
  timeout -k 10 60 python -u tools/batch_bench.py --single --batches 1 --shards 1 --frames 40 --temporal $t || exit 1
done
