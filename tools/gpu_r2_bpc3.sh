# fp32 batched k_trace after the clamped ReLU: launch bounds 4 (128 VGPRs, a few scratch
# spills) vs 3 (134 VGPRs, no spills, 3 workgroups per CU)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/bpc3.log
ab() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/batch_bench.py --frames 96 --batches 20,32 --shards 1,8 ${3:-} >> $L 2>&1
}
ab bounds4 $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab bounds3-bpc3 $PWD/build/bpc3/libnr.so "--bpc 3" &&
ab bounds3-bpc4 $PWD/build/bpc3/libnr.so "--bpc 4" &&
ab bounds4-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab bounds3-bpc3-again $PWD/build/bpc3/libnr.so "--bpc 3"
