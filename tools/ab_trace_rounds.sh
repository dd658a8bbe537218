#!/bin/bash
# Alternating A/B of tracer builds on C3 (car_1 2048^2 bf16, 8-frame batch + single) and C5 plane_1
# fp16: ROUNDS rounds, each running the default library then every alternative once, so that clock
# drift does not favour one build.   bash tools/ab_trace_rounds.sh ROUNDS build/a build/b ...
set -e
R=${1:-2}; shift
c() { timeout -k 10 240 python tools/config_bench.py --only C3,C5 --frames 3 --batch 8 2>&1 | grep -v amdgpu.ids | grep -E '"C3"|plane_1"' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'], d['geometry'], d['schedule'], d['ms_per_frame'], d['frac_of_peak'])"; }
for r in $(seq $R); do
  echo "== round $r default"; c
  for alt in "$@"; do echo "== round $r $alt"; NR_LIBRARY=$PWD/$alt/libnr.so c; done
done
