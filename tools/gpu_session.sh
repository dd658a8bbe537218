#!/bin/bash
# One GPU-box session: smoke(), the -m gpu suite, the round's bench/rocprof/PMC evidence
# (profile_round.sh) and the MLP microbenchmark over every precision.  Each GPU step has
# its own time limit and the steps are chained, so the first failure ends the session.
# usage (GPU box, repo root): bash tools/gpu_session.sh TAG [steps...]
#   steps: smoke tests prof mlp cfg pmc_bf16 pmc_fp16 pmc_x3 march bench peak   (default: smoke tests prof mlp)
#   env: PYTEST_EXTRA (extra pytest arguments, no spaces inside one), PYTEST_K (a -k expression),
#        BENCH_ARGS
set -o pipefail
TAG=${1:?tag}; shift
STEPS=${*:-smoke tests prof mlp}
mkdir -p gpurun_out
O=gpurun_out
for s in $STEPS; do
    echo "[$(date +%T)] step $s" >&2
    case $s in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 ;;
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=6 -v $PYTEST_EXTRA ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread > $O/gputests_$TAG.log 2>&1 ;;
    prof) timeout -k 10 900 bash tools/profile_round.sh $TAG > $O/profile_round_$TAG.log 2>&1 ;;
    mlp) timeout -k 10 300 python -u tools/mlp_bench.py --n 16777216 --iters 10 --precision fp32,bf16,fp16,fp32x3 --bpc 0 > $O/mlp_$TAG.log 2>&1 ;;
    cfg) timeout -k 10 400 python -u tools/config_bench.py --frames 5 > $O/cfg_$TAG.log 2>&1 ;;
    pmc_bf16) timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_bf16_$TAG bf16 12 > $O/pmc_bf16_$TAG.txt 2>&1 ;;
    pmc_fp16) timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_fp16_$TAG fp16 12 > $O/pmc_fp16_$TAG.txt 2>&1 ;;
    pmc_x3) timeout -k 10 400 bash tools/pmc_lowp.sh $O/pmc_x3_$TAG fp32x3 12 > $O/pmc_x3_$TAG.txt 2>&1 ;;
    march) timeout -k 10 400 bash tools/march_traffic.sh $O/march_$TAG 8 > $O/march_$TAG.json 2> $O/march_$TAG.err ;;
    bench) timeout -k 10 300 python -u bench.py $BENCH_ARGS > $O/bench_$TAG.json 2> $O/bench_$TAG.err ;;
    peak) timeout -k 10 200 tools/bin/mfma_peak_random > $O/peak_$TAG.txt 2>&1 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
    esac
    rc=$?
    echo "[$(date +%T)] step $s rc=$rc" >&2
    [ $rc -eq 0 ] || exit $rc
done
