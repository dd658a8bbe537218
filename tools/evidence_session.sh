#!/bin/bash
# GPU box, the round's committed evidence in one call: the bench line + rocprofv3 kernel stats +
# HBM traffic (profile_round.sh), then the reduced-precision counters of the bf16 tracer pure and
# with the endgame (pmc_lowp.sh; k_mlp16 beside it).  usage: bash tools/evidence_session.sh TAG
set -o pipefail
TAG=${1:?tag}
O=gpurun_out
timeout -k 10 900 bash tools/profile_round.sh $TAG > $O/profile_round_$TAG.log 2>&1 &&
EG=0 timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_bf16_$TAG bf16 3 > $O/pmc_bf16_$TAG.txt 2>&1 &&
EG=0.001 timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_bf16eg_$TAG bf16 3 > $O/pmc_bf16eg_$TAG.txt 2>&1
