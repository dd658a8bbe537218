# 8-shard tail at the driver's 20 frames per launch: rays per wave and occupancy
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/rays8.log
B="timeout -k 10 200 python -u tools/batch_bench.py --frames 120 --batches 20 --shards 4,8"
$B >> $L 2>&1 &&
$B --rays 48 >> $L 2>&1 &&
$B --rays 32 >> $L 2>&1 &&
$B --bpc 4 >> $L 2>&1 &&
$B --bpc 4 --rays 48 >> $L 2>&1 &&
$B --queues 16 >> $L 2>&1 &&
$B --queues 2 >> $L 2>&1
