#!/bin/bash
# Round-4 A/B of k_mlp16's chunk dealing (bf16/fp16, 2^24 points): the library default (one 12-wave
# workgroup per CU with an LDS chunk queue), then grid-stride over 4-wave workgroups (debug bit 12)
# at 3 and 12 workgroups per CU; alternative builds given as arguments.
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread -k "queue or equals_builtin"
b() { timeout -k 10 120 python tools/mlp_bench.py --n 16777216 --iters 20 --precision bf16,fp16 "$@" 2>&1 | grep -v amdgpu.ids; }
echo "== default (grid-stride, 12 per CU)"; b --bpc 0
echo "== CU queue (bit 12)"; b --debug 4096 --bpc 0
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so b --bpc 0; done
echo "== default (again)"; b --bpc 0
