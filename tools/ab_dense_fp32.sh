#!/bin/bash
# A/B: bulk ray generation in the fp32 tracer (build/d32) against the default build, at 3 and 4
# workgroups per CU (the ring's LDS leaves the fp32 batched instance 3), batched and single frames
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/ab_dense_fp32.log
: > $O
for lib in default build/d32 default build/d32; do
  if [ $lib = default ]; then unset NR_LIBRARY; else export NR_LIBRARY=$PWD/$lib/libnr.so; fi
  echo "== $lib" >> $O
  for bpc in 3 4; do
    timeout -k 10 120 python -u tools/batch_bench.py --frames 64 --batches 32 --shards 1 --bpc $bpc 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  done
  timeout -k 10 120 python -u tools/batch_bench.py --frames 32 --batches 1 --shards 1,8 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
