# determinism sentinel (200 batched launches per precision) on the layer-0 swap build, then
# the driver's bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lowp_sentinel.py bf16 200 > gpurun_out/sentinel2_bf16.log 2>&1 && tail -1 gpurun_out/sentinel2_bf16.log &&
timeout -k 10 300 python -u tools/lowp_sentinel.py fp16 200 > gpurun_out/sentinel2_fp16.log 2>&1 && tail -1 gpurun_out/sentinel2_fp16.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_shape2.json 2> gpurun_out/bench_driver_shape2.err && tail -c 300 gpurun_out/bench_driver_shape2.json
