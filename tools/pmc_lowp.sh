#!/bin/bash
# Counter evidence for the reduced-precision MLP (k_mlp16<bf16|fp16>) and the batched
# k_trace of the same precision: two --pmc passes per program, each within the per-block
# limits (8 SQ + 1 GRBM), with --kernel-trace for the dispatch durations.
#   pass A: matrix-pipe busy, instruction mix, issue stalls (tools/pmc_mfma_summary.py)
#   pass B: LDS instructions, bank-conflict and LDS-array cycles, LDS issue stalls, SALU
# GPU box:  bash tools/pmc_lowp.sh OUTDIR [precision] [bpc]   (EG=tau: the tracer's endgame threshold,
# default 0 = the pure 16-bit march, so that the counters stay comparable with round 4's)
set -e
OUT=$(realpath -m "$1"); PREC=${2:-bf16}; BPC=${3:-3}
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for pass in A B; do
    CTR=${!pass}
    timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/mlp_$pass" -o run -- \
        python3 "$REPO/tools/mlp_bench.py" --n 16777216 --iters 3 --precision "$PREC" --bpc "$BPC" > "$OUT/mlp_$pass.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/trace_$pass" -o run -- \
        python3 "$REPO/tools/render_frames.py" --frames 2 --batch 32 --precision "$PREC" --endgame "${EG:-0}" > "$OUT/trace_$pass.log" 2>&1
done
python3 "$REPO/tools/pmc_lowp_summary.py" "$OUT"
