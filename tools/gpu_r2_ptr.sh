# A/B: k_mlp16 with the input pointer strength-reduced by hand (build/ptr) vs the default build
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/ptr.log
: > $L
ab() {
  echo "== $1" >> $L
  for p in bf16 fp16 fp32; do
    NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision $p --bpc 8 >> $L 2>&1 || return 1
  done
}
for r in 1 2 3; do
  ab default $PWD/cudaneuralrender_amd/lib/libnr.so && ab ptr $PWD/build/ptr/libnr.so || exit 1
done
