#!/bin/bash
# Round 6: workgroups per CU (nr_set_occupancy) after the argument re-reads changed the tracers'
# registers (fp32 115 / 113 VGPRs, bf16 128), GPU box: fp32 single frames and 32-frame batches at
# 1024^2, C3 / C5 at the default endgame, each at the library default (0) and 2 / 3 / 4 per CU.
#   bash tools/occ_sweep_r6.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/occ6}")
mkdir -p "$OUT"
for bpc in 0 2 3 4 0; do
  echo "== bpc $bpc" >> "$OUT/fp32.log"
  timeout -k 10 200 python -u tools/batch_bench.py --frames 32 --batches 1,32 --shards 1 --bpc $bpc 2>&1 | grep -v amdgpu.ids >> "$OUT/fp32.log" || exit 1
done
for bpc in 0 2 4; do
  echo "== bpc $bpc" >> "$OUT/cfg.log"
  timeout -k 10 300 python -u tools/config_bench.py --frames 4 --only C3,C5 --bpc $bpc 2>&1 | grep '^{' >> "$OUT/cfg.log" || exit 1
done
