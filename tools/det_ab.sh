#!/bin/bash
# Batched reduced-precision reproducibility across A/B builds (GPU box):
#   bash tools/det_ab.sh TRIALS [ALT_LIB_DIR ...]
# For the default build and each ALT_LIB_DIR/libnr.so: tools/lowp_sentinel.py fp16 and bf16
# (TRIALS batched launches each, compared with the single-frame renders).
set -e
N=$1; shift
mkdir -p gpurun_out/r2
run() {
  for p in fp16 bf16; do
    timeout -k 10 240 python -u tools/lowp_sentinel.py $p $N | grep "batched trials" | cut -c1-150
  done
}
echo "== default"; run
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so run; done
