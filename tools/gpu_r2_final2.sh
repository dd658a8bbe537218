set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 900 bash tools/profile_round.sh r2d > gpurun_out/profile_round_r2d.log 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --frames 5 > gpurun_out/cfg_final.log 2>&1
