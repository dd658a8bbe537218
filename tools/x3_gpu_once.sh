set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/config_bench.py > gpurun_out/cfg_x3_a.log 2>&1 && timeout -k 10 300 python -u tools/config_bench.py --debug 32768 > gpurun_out/cfg_x3_b.log 2>&1 && timeout -k 10 300 python -u tools/config_bench.py > gpurun_out/cfg_x3_c.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_x3.log 2>&1
