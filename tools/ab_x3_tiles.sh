#!/bin/bash
# Round-4 A/B: the tracers' x3 normals as one two-tile pass (default) or two one-tile passes
# (build/x3t1: -DNR_X3_NORMAL_TILES=1, fewer spilled registers), alternating, C3/C4/C5 batches.
set -e
c() { NR_LIBRARY="$1" timeout -k 10 300 python tools/config_bench.py --only C3,C4,C5 --frames 3 --batch 8 2>&1 | grep -v amdgpu.ids | grep batch8 | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'], d['geometry'][:10], d['ms_per_frame'], d['frac_of_peak'])"; }
for r in 1 2; do echo "== round $r two-tile pass (default)"; c ""; echo "== round $r one-tile passes"; c build/x3t1/libnr.so; done
