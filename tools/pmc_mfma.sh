#!/bin/bash
# MFMA-pipe busy fraction and effective clock of the batched k_trace vs the MLP-only
# kernel k_mlp16 at the same occupancy (one --pmc pass each, with --kernel-trace for the
# dispatch durations).  GPU box:  bash tools/pmc_mfma.sh OUTDIR [precision]
#   util  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
#   clock = GRBM_GUI_ACTIVE / 8 / kernel duration  (MI355X_MICROARCH.md "DVFS give-back")
set -e
OUT=$(realpath -m "$1"); PREC=${2:-fp32}
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/tools/render_frames.py" --frames 2 --batch 32 --precision "$PREC" > "$OUT/trace.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/mlp" -o run -- \
    python3 "$REPO/tools/mlp_bench.py" --n 16777216 --iters 3 --precision "$PREC" --bpc 3 > "$OUT/mlp.log" 2>&1
python3 "$REPO/tools/pmc_mfma_summary.py" "$OUT"
