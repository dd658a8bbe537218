# A/B: pipelined clamped bf16 hidden layers (NR_LOWP_PIPE 1 = full guard, 2 = light guard)
# against the unpipelined form (0): k_mlp16 microbench and the C3 / bench-frame tracer.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/pipe.log
run() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision bf16 --bpc 8 >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/config_bench.py --only C3 --frames 16 >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 120 python -u tools/batch_bench.py --frames 64 --batches 32 --shards 1 --precision bf16 >> $L 2>&1
}
run pipe0 $PWD/build/pipe0/libnr.so &&
run pipe1 $PWD/cudaneuralrender_amd/lib/libnr.so &&
run pipe2 $PWD/build/pipe2/libnr.so &&
run pipe0-again $PWD/build/pipe0/libnr.so
