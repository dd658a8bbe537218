set -o pipefail
mkdir -p gpurun_out
for lib in ${LIBS:-default build/wps2 build/wps4 default}; do
  if [ $lib = default ]; then unset NR_LIBRARY; else export NR_LIBRARY=$PWD/$lib/libnr.so; fi
  echo "== $lib"
  timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --iters 20 --precision bf16,fp16 --bpc 8 2>&1 | grep -v amdgpu.ids || exit 1
done
