#!/bin/bash
# Round-4 A/B of the two-ray-group tracer (k_trace2, nr_set_debug bit 14) against k_trace (the
# default for batched bf16/fp16), alternating, on C3/C4/C5 batches.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread -k "two_group"
c() { timeout -k 10 300 python tools/config_bench.py --only C3,C4,C5 --frames 3 --batch 8 --debug "$1" 2>&1 | grep -v amdgpu.ids | grep batch8 | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'], d['geometry'][:10], d['ms_per_frame'], d['frac_of_peak'])"; }
for r in 1 2; do echo "== round $r one group (k_trace, default)"; c 0; echo "== round $r two groups (bit 14)"; c 16384; done
