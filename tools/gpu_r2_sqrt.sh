set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/sqrt_exhaustive > gpurun_out/sqrt_exhaustive.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
for i in 1 2; do timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 1,8 >> gpurun_out/sqrt_ab.log 2>&1 && \
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 1,8 --precision bf16 >> gpurun_out/sqrt_ab.log 2>&1 || exit 1; done
