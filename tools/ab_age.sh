#!/bin/bash
# GPU box: A/B of the fp32 tracer's age priority (NR_AGE_PRIO builds) on the bench frame: one-frame
# launches and 32-frame batches, default / each alternative / default again.
#   bash tools/ab_age.sh ALT_DIR [ALT_DIR ...]
set -o pipefail
run() {
  timeout -k 10 90 python -u tools/batch_bench.py --single --batches 1 --shards 1 --frames 60 || return 1
  timeout -k 10 90 python -u tools/batch_bench.py --batches 32 --shards 1 --frames 64 || return 1
}
echo "== default"; run || exit 1
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so run || exit 1; done
echo "== default (again)"; run
