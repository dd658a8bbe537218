# fp32 refill threshold (NR_REFILL_MIN_FP32) after the clamped-ReLU change: bench frame,
# 20 and 32 frames per launch, 1 and 8 shards; default build (4) interleaved with 2/6/8
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/rmin.log
ab() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/batch_bench.py --frames 96 --batches 20,32 --shards 1,8 >> $L 2>&1
}
ab 4 $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab 2 $PWD/build/rmin2/libnr.so &&
ab 6 $PWD/build/rmin6/libnr.so &&
ab 8 $PWD/build/rmin8/libnr.so &&
ab 4-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab 6-again $PWD/build/rmin6/libnr.so
