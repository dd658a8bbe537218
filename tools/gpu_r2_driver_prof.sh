# rocprofv3 kernel trace + stats of the driver's exact bench command (--steps 20 --warmup 5):
# per-dispatch k_trace durations, to set beside the BENCH line's per-launch HIP-event time
set -o pipefail
mkdir -p gpurun_out
OUT=$(realpath -m gpurun_out/prof_driver)
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$REPO/bench.py" --steps 20 --warmup 5 > "$OUT.json" 2> "$OUT.err"
