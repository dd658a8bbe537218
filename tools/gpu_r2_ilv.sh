set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "batch" -x -q --timeout 200 --timeout-method thread > gpurun_out/ilv_tests.log 2>&1 && \
for i in 1 2; do for d in 0 1024; do
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 8,32 --shards 1,2,4,8 --debug $d >> gpurun_out/ilv.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 1,8 --debug $d --precision bf16 >> gpurun_out/ilv.log 2>&1 || exit 1
done; done
