set -o pipefail
mkdir -p gpurun_out
ALT=build/alt_mfmafinal/libnr.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_parity.py -k "lowp or clamp" -x -v --timeout 200 --timeout-method thread > gpurun_out/dot2_tests.log 2>&1 && \
for i in 1 2; do
timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 4,6 --iters 10 --n 16777216 >> gpurun_out/mlp_dot2.log 2>&1 && \
NR_LIBRARY=$ALT timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 4,6 --iters 10 --n 16777216 | sed 's/^/mfmafinal /' >> gpurun_out/mlp_dot2.log 2>&1 || exit 1
done && \
timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 > gpurun_out/cfg_dot2.log 2>&1 && \
NR_LIBRARY=$ALT timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 | sed 's/^/mfmafinal /' >> gpurun_out/cfg_dot2.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16_dot2 bf16 4 > gpurun_out/pmc_bf16_dot2.txt 2>&1
