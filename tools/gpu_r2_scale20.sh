# Per-rank frame time at the driver's bench shape (20 frames per launch, band 1) for 1/2/4/8
# row-band shards, and the schedule knobs that act on the launch tail.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/scale20.log
B="timeout -k 10 200 python -u tools/batch_bench.py --frames 120 --batches 20,32"
$B --shards 1,2,4,8 >> $L 2>&1 &&
$B --shards 4,8 --bpc 3 >> $L 2>&1 &&
$B --shards 4,8 --bpc 4 >> $L 2>&1 &&
$B --shards 4,8 --bpc 2 >> $L 2>&1 &&
$B --shards 8 --temporal 1 >> $L 2>&1 &&
$B --shards 8 --hold 64 >> $L 2>&1 &&
$B --shards 8 --hold 96 >> $L 2>&1 &&
$B --shards 8 --spread 64 >> $L 2>&1 &&
$B --shards 8 --debug 1024 >> $L 2>&1
