set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || true
