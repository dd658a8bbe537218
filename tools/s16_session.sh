#!/bin/bash
# k_mlp16 on the 16x16x32 stream (default) against the 32x32x16 one (nr_set_debug bit 12), GPU box:
# the stream / lowp parity tests, then mlp_bench A/B/A/B at 2^22 and 2^24 (bf16, fp16), then one
# rocprofv3 counter pass per form (matrix-pipe busy, clock, VALU per MFMA).
#   bash tools/s16_session.sh OUTDIR
set -o pipefail
OUT=$(realpath -m "${1:-gpurun_out/s16}")
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd "$REPO"
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_lowp.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
for rep in 1 2; do
  for dbg in 0 4096; do
    for n in 4194304 16777216; do
      timeout -k 10 120 python3 -u tools/mlp_bench.py --n $n --iters 20 --precision bf16,fp16 --debug $dbg 2>&1 \
        | grep -v amdgpu.ids >> "$OUT/times.log" || exit 1
    done
  done
done
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for prec in bf16 fp16; do
  for dbg in 0 4096; do
    tag=pmc_${prec}_$dbg
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv \
       -d "$OUT/$tag" -o run -- python3 "$REPO/tools/mlp_bench.py" --n 16777216 --iters 10 --precision $prec --debug $dbg \
       > "$OUT/$tag.log" 2>&1) || exit 1
    python3 - "$OUT/$tag" "$prec dbg $dbg" <<'EOF' | tee -a "$OUT/pmc.txt"
import sys
sys.path.insert(0, "tools")
from pmc_lowp_summary import load
for k, (c, n, dur) in load(sys.argv[1]).items():
    if "k_mlp16" not in k:
        continue
    g = c["GRBM_GUI_ACTIVE"] / 8
    print(f"{sys.argv[2]}: {k}: dispatches {n}  MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g):.3f}  "
          f"clock {g / dur / 1e9:.3f} GHz  VALU/MFMA {c['SQ_INSTS_VALU'] / c['SQ_INSTS_MFMA']:.2f}  "
          f"WAIT_INST_ANY/WAVE {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  median {dur * 1e3:.4f} ms")
EOF
  done
done
