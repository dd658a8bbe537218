# centre-out block order (nr_set_debug bit 11) vs raster: bench frame single / 20 frames,
# 1 and 8 shards; car_1 C3 bf16 too
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/corder.log
for rep in 1 2; do
for d in 0 2048; do
timeout -k 10 200 python -u tools/batch_bench.py --frames 80 --batches 1,20 --shards 1,8 --debug $d >> $L 2>&1 || exit 1
timeout -k 10 200 python -u tools/batch_bench.py --frames 80 --batches 1,20 --shards 1,8 --debug $d --precision bf16 >> $L 2>&1 || exit 1
done
done
