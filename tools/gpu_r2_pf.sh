set -o pipefail
mkdir -p gpurun_out
ALT=build/alt_nopf/libnr.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_parity.py -k "lowp or clamp" -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 && \
for i in 1 2; do
timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 3,4,6 --iters 10 --n 16777216 >> gpurun_out/mlp_pf.log 2>&1 && \
NR_LIBRARY=$ALT timeout -k 10 200 python -u tools/mlp_bench.py --precision bf16,fp16 --bpc 3,4,6 --iters 10 --n 16777216 | sed 's/^/nopf /' >> gpurun_out/mlp_pf.log 2>&1 || exit 1
done && \
timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full,C5 --frames 5 > gpurun_out/cfg_pf.log 2>&1 && \
NR_LIBRARY=$ALT timeout -k 10 300 python -u tools/config_bench.py --only C3,C4-full --frames 5 | sed 's/^/nopf /' >> gpurun_out/cfg_pf.log 2>&1
