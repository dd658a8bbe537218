# fp32 next-layer A-operand prefetch in the 1-2 tile MLP variants: lone-wave MLP latency,
# single-frame and 8-shard frame times, A/B against build/prev
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/pf2.log
ab() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_latency.py >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 1,20 --shards 1,8 >> $L 2>&1
}
ab prefetch $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev $PWD/build/prev/libnr.so &&
ab prefetch-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev-again $PWD/build/prev/libnr.so
