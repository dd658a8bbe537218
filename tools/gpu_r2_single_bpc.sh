# one frame per launch after the fp32 clamped ReLU: occupancy 2 (default) vs 3 workgroups per CU
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/single_bpc.log
for rep in 1 2; do for b in 2 3; do
timeout -k 10 200 python -u tools/batch_bench.py --frames 64 --batches 1,4 --shards 1,8 --bpc $b >> $L 2>&1 || exit 1
done; done
