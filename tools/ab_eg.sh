#!/bin/bash
# A/B of endgame (EG) tracer builds on C3 and C5 (GPU box):
#   bash tools/ab_eg.sh ALT_DIR [ALT_DIR ...]
# default build, then each NR_LIBRARY=ALT_DIR/libnr.so, then the default again; tau 1e-3.
set -e
run() { timeout -k 10 200 python -u tools/config_bench.py --frames 5 --only C3,C5 --endgame 0.001; }
echo "== default"; run
for alt in "$@"; do echo "== $alt"; NR_LIBRARY=$PWD/$alt/libnr.so run; done
echo "== default (again)"; run
