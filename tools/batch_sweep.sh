#!/bin/bash
# Schedule knobs of the batched tracer (32-frame launches of the bench frame), fp32 and bf16.
set -e
for prec in fp32 bf16; do
  for bpc in 2 3; do
    for spread in 0 16 64; do
      timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 32 --shards 1 --precision $prec --bpc $bpc --spread $spread
    done
  done
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 32 --shards 1 --precision $prec --bpc 3 --queues 16
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 32 --shards 1 --precision $prec --bpc 3 --queues 4
done
