#!/bin/bash
# A/B of libnr.so builds on the stand-alone MLP (k_mlp16) and its bit-exactness tests (GPU box):
#   LIBS="default build/p1 ..." PRECS=bf16 bash tools/ab_mlp.sh TAG
# each build: tests/test_gpu_lowp.py (clamped vs max-form ReLU, bit-exact) then mlp_bench at
# 2^24 and 2^26 points; the default build runs first and last (box drift)
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
O=gpurun_out/abmlp_$TAG.log
: > $O
for lib in ${LIBS:-default}; do
  if [ $lib = default ]; then unset NR_LIBRARY; else export NR_LIBRARY=$PWD/$lib/libnr.so; fi
  echo "== $lib" >> $O
  if [ -n "$TESTS" ]; then
    timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || exit 1
  fi
  for n in ${SIZES:-16777216 67108864}; do
    timeout -k 10 120 python -u tools/mlp_bench.py --n $n --iters 20 --precision ${PRECS:-bf16} --bpc ${BPC:-8} 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  done
done
