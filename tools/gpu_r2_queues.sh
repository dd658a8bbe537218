# pixel-queue shard count at the driver's shape (20 frames per launch) for 1..8 row-band shards
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/queues.log
for rep in 1 2; do
for q in 8 2 4 1; do
timeout -k 10 200 python -u tools/batch_bench.py --frames 120 --batches 20 --shards 1,2,4,8 --queues $q >> $L 2>&1 || exit 1
done
done
