# bf16 clamped conversion blocks without the accumulator touches (18 wait states in the
# block instead): lowp parity tests on that build, then A/B against the default build
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/touch.log
NR_LIBRARY=$PWD/build/notouch/libnr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_lowp_contract.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_touch.log 2>&1 || exit 1
tail -2 gpurun_out/gputests_touch.log
ab() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision bf16 --bpc 8 >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 20,32 --shards 1 --precision bf16 >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/config_bench.py --only C3 --frames 16 >> $L 2>&1
}
ab touch $PWD/build/prev/libnr.so &&
ab notouch $PWD/build/notouch/libnr.so &&
ab touch-again $PWD/build/prev/libnr.so &&
ab notouch-again $PWD/build/notouch/libnr.so
