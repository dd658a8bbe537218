# reduced-precision tracers at launch bounds 4 + the size-based default occupancy: every GPU
# test, then the configurations and the bench frame in every precision
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_lowp4.log 2>&1 && \
tail -2 gpurun_out/gputests_lowp4.log && \
timeout -k 10 300 python -u tools/config_bench.py --frames 5 > gpurun_out/cfg_lowp4.log 2>&1 && \
timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 1,20,32 --shards 1,8 --precision bf16 >> gpurun_out/cfg_lowp4.log 2>&1 && \
timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 1,20,32 --shards 1,8 --precision fp32 >> gpurun_out/cfg_lowp4.log 2>&1
