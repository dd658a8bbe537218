# A/B of k_mlp16 builds: layer-0 swap (default), + uniform chunk addressing (build/addr), round-2 (build/prev)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/addr.log
: > $L
ab() {
  echo "== $1" >> $L
  for p in bf16 fp16 fp32; do
    NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision $p --bpc 8 >> $L 2>&1 || return 1
  done
}
for r in 1 2; do
  ab l0 $PWD/cudaneuralrender_amd/lib/libnr.so && ab addr $PWD/build/addr/libnr.so && ab prev $PWD/build/prev/libnr.so || exit 1
done
