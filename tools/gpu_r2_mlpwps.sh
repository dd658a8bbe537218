# k_mlp16 register target 5 waves per SIMD (<= 96 VGPRs) vs 2 (build/prev: 100 VGPRs, 4 resident)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/mlpwps.log
ab() {
  echo "== $1" >> $L
  for p in bf16 fp16 fp32; do
    NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision $p --bpc 8 >> $L 2>&1 || return 1
  done
}
ab wps5 $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev $PWD/build/prev/libnr.so &&
ab wps5-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev-again $PWD/build/prev/libnr.so &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lowp.py -x -q -k "mlp" --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1
