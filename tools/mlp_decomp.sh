#!/bin/bash
# Where k_mlp16 bf16's time goes beside its hidden layers (GPU box): the default build and the
# NR_MLP16_EXP builds (build/expN: 1 no final layer, 2 no range check, 4 no input split, 7 none
# of them -- wrong values, timing only), each timed at 2^22 and 2^24 points and counted once
# (rocprofv3 --pmc: matrix-pipe busy, clock, VALU per MFMA); then the hidden layers alone
# (tools/bin/mlp_shape_ab).
#   bash tools/mlp_decomp.sh OUTDIR [libs...]
set -o pipefail
OUT=$(realpath -m "$1"); shift
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for lib in ${@:-default build/exp1 build/exp2 build/exp4 build/exp7}; do
  if [ $lib = default ]; then unset NR_LIBRARY; else export NR_LIBRARY=$REPO/$lib/libnr.so; fi
  tag=$(basename $lib)
  echo "== $lib" | tee -a "$OUT/times.log"
  for n in 4194304 16777216; do
    timeout -k 10 120 python3 -u "$REPO/tools/mlp_bench.py" --n $n --iters 20 --precision ${PRECS:-bf16} 2>&1 \
      | grep -v amdgpu.ids | tee -a "$OUT/times.log" || exit 1
  done
  mkdir -p "$OUT/$tag"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv \
     -d "$OUT/$tag/mlp_A" -o run -- python3 "$REPO/tools/mlp_bench.py" --n 16777216 --iters 3 --precision ${PRECS:-bf16} \
     > "$OUT/$tag/pmc.log" 2>&1) || exit 1
  python3 - "$OUT/$tag" <<'EOF' | tee -a "$OUT/times.log"
import sys
sys.path.insert(0, "tools")
from pmc_lowp_summary import load
for k, (c, n, dur) in load(sys.argv[1] + "/mlp_A").items():
    if "k_mlp16" not in k:
        continue
    g = c["GRBM_GUI_ACTIVE"] / 8
    print(f"  {k}: MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g):.3f}  clock {g / dur / 1e9:.3f} GHz  "
          f"VALU/MFMA {c['SQ_INSTS_VALU'] / c['SQ_INSTS_MFMA']:.2f}  WAIT_INST_ANY/WAVE {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  "
          f"median {dur * 1e3:.4f} ms")
EOF
done
unset NR_LIBRARY
if [ -x "$REPO/tools/bin/mlp_shape_ab" ]; then
  timeout -k 10 120 "$REPO/tools/bin/mlp_shape_ab" 256 2>&1 | tee -a "$OUT/times.log"
fi
