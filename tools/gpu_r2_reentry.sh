# re-entry check after the container rebuild: every GPU test, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_reentry.log 2>&1 && \
tail -2 gpurun_out/gputests_reentry.log && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_reentry.log 2>&1 && \
tail -1 gpurun_out/smoke_reentry.log && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_reentry.log 2>&1 && \
tail -1 gpurun_out/bench_reentry.log
