# temporal block order on batched launches: parity tests, then frame times with and without
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/temporal.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_temporal.log 2>&1 || exit 1
tail -2 gpurun_out/gputests_temporal.log
B="timeout -k 10 200 python -u tools/batch_bench.py --frames 120 --batches 1,20,32 --shards 1,8"
$B >> $L 2>&1 &&
$B --temporal 1 >> $L 2>&1 &&
$B --precision bf16 >> $L 2>&1 &&
$B --precision bf16 --temporal 1 >> $L 2>&1
