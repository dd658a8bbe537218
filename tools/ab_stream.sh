#!/bin/bash
# Round-4 A/B of the tracer's two-tile stream: the stream tests, the lone-wave latencies, then C3
# (car_1 2048^2 bf16, single + 8-frame batch) and C5 plane_1 for the default library, the builtin
# form of the same library (debug bit 11), and each alternative build given.
#   bash tools/ab_stream.sh build/base build/bpc3 ...
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread
timeout -k 10 120 python tools/mlp_latency.py 2>&1 | grep -v amdgpu.ids
c3() { timeout -k 10 240 python tools/config_bench.py --only C3,C5 --frames 5 --batch 8 "$@" 2>&1 | grep -v amdgpu.ids | grep -E '"C3"|plane_1'; }
echo "== default (stream)"; c3
echo "== default, builtin form"; c3 --debug 2048
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so c3; done
echo "== default (again)"; c3
