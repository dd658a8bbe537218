# A/B: reduced-precision layer 0 built from each lane's own split dealt by permlane32_swap
# (default build) vs the round-2 per-tile split (build/prev); then the reduced-precision
# parity tests and the full GPU suite on the default build
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/l0swap.log
: > $L
ab() {
  echo "== $1" >> $L
  for p in bf16 fp16; do
    NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision $p --bpc 8 >> $L 2>&1 || return 1
  done
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/config_bench.py --only C3 --frames 6 --batch 8 >> $L 2>&1 || return 1
}
ab new $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev $PWD/build/prev/libnr.so &&
ab new-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev-again $PWD/build/prev/libnr.so &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_l0swap.log 2>&1 &&
tail -2 gpurun_out/gputests_l0swap.log
