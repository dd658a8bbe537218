# fp32 layer-0 input transpose by v_permlane{32,16}_swap: GPU tests, then A/B against the
# previous build (build/prev: ds_bpermute + selects)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/pl.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_pl.log 2>&1 || exit 1
tail -2 gpurun_out/gputests_pl.log
ab() {
  echo "== $1" >> $L
  NR_LIBRARY=$2 timeout -k 10 200 python -u tools/batch_bench.py --frames 96 --batches 20,32 --shards 1,8 >> $L 2>&1 &&
  NR_LIBRARY=$2 timeout -k 10 120 python -u tools/mlp_bench.py --n 16777216 --precision fp32 --bpc 8 >> $L 2>&1
}
ab permlane $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev $PWD/build/prev/libnr.so &&
ab permlane-again $PWD/cudaneuralrender_amd/lib/libnr.so &&
ab prev-again $PWD/build/prev/libnr.so
