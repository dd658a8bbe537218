set -o pipefail
O=gpurun_out/probe_sweep.txt
: > $O
for pr in 0,16 16,16 32,16 64,16 128,16 32,8 64,8 64,4 128,8; do
  for dbg in 0 16; do
    timeout -k 10 120 python3 -u tools/batch_bench.py --single --batches 1 --shards 1 --frames 40 --probe $pr --debug $dbg 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  done
done
