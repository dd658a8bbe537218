set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_lowp_contract.py > gpurun_out/gputests.log 2>&1 && \
for i in 1 2; do
for b in 3 4; do timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 8,32 --shards 1,8 --bpc $b >> gpurun_out/occ4.log 2>&1 || exit 1; done
for b in 2 3; do timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 8,32 --shards 1,8 --bpc $b --precision bf16 >> gpurun_out/occ4.log 2>&1 || exit 1; done
done
