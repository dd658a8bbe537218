set -o pipefail
O=gpurun_out
timeout -k 10 200 tools/bin/mfma_peak_random > $O/peak_r5c.txt 2>&1 &&
timeout -k 10 200 tools/bin/mlp_shape_ab 256 > $O/shape_r5c.txt 2>&1 &&
for n in 4194304 16777216 67108864; do timeout -k 10 200 python -u tools/mlp_bench.py --n $n --iters 20 --precision bf16,fp16 --bpc 0 || exit 1; done > $O/mlp_r5c.txt 2>&1 &&
timeout -k 10 200 tools/bin/mlp_shape_ab 1024 >> $O/shape_r5c.txt 2>&1
