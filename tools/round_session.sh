#!/bin/bash
# GPU box: one call that runs an A/B of alternative endgame builds, smoke + the -m gpu suite, then
# the round's evidence (bench, rocprof kernel stats, HBM traffic, bf16 counters).
#   bash tools/round_session.sh TAG [ALT_BUILD_DIR ...]
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out
mkdir -p $O
if [ $# -gt 0 ]; then bash tools/ab_eg.sh "$@" > $O/ab_eg_$TAG.txt 2>&1 || exit 1; fi
bash tools/gpu_session.sh $TAG smoke tests &&
bash tools/evidence_session.sh $TAG
