# fp32 clamped ReLU: GPU tests, then A/B against the add + max build (build/f32max)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/f32clamp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_f32clamp.log 2>&1 || exit 1
tail -3 gpurun_out/gputests_f32clamp.log
ab() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/batch_bench.py --frames 96 --batches 20,32 --shards 1,8 >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision fp32 --bpc 8 >> $L 2>&1
}
ab clamp $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab max $PWD/build/f32max/libnr.so &&
ab clamp-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab max-again $PWD/build/f32max/libnr.so
