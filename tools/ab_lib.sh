#!/bin/bash
# A/B of two builds of libnr.so on the bench frame (GPU box):
#   bash tools/ab_lib.sh ALT_LIB_DIR [extra batch_bench args]
# default build first, then NR_LIBRARY=ALT_LIB_DIR/libnr.so; fp32 at 1 and 8 shards, bf16 at 1.
set -e
ALT=$1; shift
run() {
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 32 --shards 1,8 "$@"
  timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 32 --shards 1 --precision bf16 "$@"
}
echo "== default"; run "$@"
echo "== $ALT"; NR_LIBRARY=$PWD/$ALT/libnr.so run "$@"
echo "== default (again)"; run "$@"
