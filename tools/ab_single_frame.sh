set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/sf_ab.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_pf.log 2>&1 || exit 1
timeout -k 10 60 python -u tools/mlp_latency.py > $O 2>&1 || exit 1
for lib in default build/old default build/old; do
  if [ $lib = default ]; then unset NR_LIBRARY; else export NR_LIBRARY=$PWD/$lib/libnr.so; fi
  echo "== $lib" >> $O
  timeout -k 10 120 python -u tools/batch_bench.py --frames 32 --batches 1 --shards 1,8 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
