# bf16/fp16 tracer at 4 workgroups per CU (launch bounds 4: 128 VGPRs, ~20 spilled) vs 3
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/lowp_bpc4.log
for rep in 1 2; do
echo "== default bpc3" >> $L
timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 20,32 --shards 1,8 --precision bf16 >> $L 2>&1 || exit 1
echo "== bounds4 bpc4" >> $L
NR_LIBRARY=$PWD/build/bpc4/libnr.so timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 20,32 --shards 1,8 --precision bf16 --bpc 4 >> $L 2>&1 || exit 1
done
NR_LIBRARY=$PWD/build/bpc4/libnr.so timeout -k 10 200 python -u tools/config_bench.py --only C3 --frames 16 --bpc 4 >> $L 2>&1
timeout -k 10 200 python -u tools/config_bench.py --only C3 --frames 16 >> $L 2>&1
