set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_final.log 2>&1 && timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1
