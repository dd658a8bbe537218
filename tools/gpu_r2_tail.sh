set -o pipefail
mkdir -p gpurun_out
ALT=build/alt_nt/libnr.so
for t in 0 1; do timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 8,32 --shards 1,8 --temporal $t >> gpurun_out/tail.log 2>&1 || exit 1; done
for t in 0 1; do timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 8 --temporal $t --spread 16 >> gpurun_out/tail.log 2>&1 || exit 1; done
NR_LIBRARY=$ALT timeout -k 10 200 python -u tools/batch_bench.py --frames 128 --batches 32 --shards 1,8 | sed 's/^/nt /' >> gpurun_out/tail.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
NR_LIBRARY=$GRAFT_REPO_ROOT/$ALT timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nt_write -o run -- python3 $GRAFT_REPO_ROOT/tools/render_frames.py --frames 3 --batch 32 > $GRAFT_REPO_ROOT/gpurun_out/nt_write.log 2>&1
