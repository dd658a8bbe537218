set -o pipefail
mkdir -p gpurun_out
for b in 3 4; do for sp in 0 16; do
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 8 --bpc $b --spread $sp >> gpurun_out/sweep8.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 8 --bpc $b --spread $sp --precision bf16 >> gpurun_out/sweep8.log 2>&1 || exit 1
done; done
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 8 --queues 16 >> gpurun_out/sweep8.log 2>&1
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 8 --queues 4 >> gpurun_out/sweep8.log 2>&1
