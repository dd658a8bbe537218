#!/bin/bash
# Round 6: bf16 single frames below 2 M pixels with the default endgame (default_bpc's 2 blocks per CU
# used to become 2/3 of the CUs' worth of 12-wave workgroups), the current build against build/prev,
# A/B/A through tools/batch_bench.py --single (plane_1, 128 steps).
set -o pipefail
run() { for W in 512 768 1024; do timeout -k 10 120 python -u tools/batch_bench.py --single --precision bf16 --size $W \
  --frames 16 --batches 1 --shards 1 2>&1 | grep -v amdgpu.ids || return 1; done; }
echo "== new"; run || exit 1
echo "== prev"; NR_LIBRARY=$PWD/build/prev/libnr.so run || exit 1
echo "== new"; run || exit 1
