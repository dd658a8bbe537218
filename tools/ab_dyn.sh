#!/bin/bash
# Round-4 A/B of k_mlp16's dynamic tail (bf16/fp16, 2^24 points): the library default (last eighth
# of the chunks claimed dynamically, resident grid), then grid-stride only (debug bit 12) at 12 and
# 3 workgroups per CU; alternative builds given as arguments (e.g. other NR_MLP16_DYN fractions).
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread -k "dynamic or equals_builtin"
b() { timeout -k 10 120 python tools/mlp_bench.py --n 16777216 --iters 20 --precision bf16,fp16 "$@" 2>&1 | grep -v amdgpu.ids; }
echo "== default (dynamic tail)"; b --bpc 0,4,6
echo "== grid-stride"; b --debug 4096 --bpc 12,3; echo "== dynamic tail (bit 13)"; b --debug 8192 --bpc 3
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so b --bpc 0; done
echo "== default (again)"; b --bpc 0
