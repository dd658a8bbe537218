# reduced-precision tracer occupancy with launch bounds 4: workgroups per CU 2/3/4 for single
# frames, small and large batches, 1024^2 and 2048^2 (256 steps)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/lowp_occ.log
for b in 2 3 4; do
timeout -k 10 200 python -u tools/batch_bench.py --frames 40 --batches 1,4,20 --shards 1,8 --precision bf16 --bpc $b >> $L 2>&1 || exit 1
timeout -k 10 200 python -u tools/batch_bench.py --frames 16 --batches 1,8 --shards 1 --precision bf16 --size 2048 --steps 256 --bpc $b >> $L 2>&1 || exit 1
timeout -k 10 200 python -u tools/batch_bench.py --frames 40 --batches 1,4,20 --shards 1 --precision fp32 --bpc $b >> $L 2>&1 || exit 1
done
