#!/bin/bash
# fp32 tracer timing of alternative builds at a given blocks-per-CU:
#   bash tools/ab_bpc.sh BPC build/a [build/b ...]   (the default libnr.so first and last)
set -e
B=$1; shift
run() { timeout -k 10 120 python tools/batch_bench.py --frames 64 --batches 1,32 --shards 1,8 --bpc "$@"; }
echo "== default (bpc auto)"; run 0
for alt in "$@"; do echo "== $alt (bpc $B)"; NR_LIBRARY=$PWD/$alt/libnr.so run $B; done
echo "== default (bpc auto, again)"; run 0
