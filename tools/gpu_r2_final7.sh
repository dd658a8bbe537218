# Evidence on the build with the layer-0 swap: smoke(), bench + rocprof + PMC traffic
# (profile_round.sh), the bf16 counter passes and the C3-C5 configurations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final7.log 2>&1 && \
timeout -k 10 900 bash tools/profile_round.sh r2i > gpurun_out/profile_round_r2i.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_lowp.sh gpurun_out/pmc_bf16_r2i bf16 8 > gpurun_out/pmc_bf16_r2i.txt 2>&1 && \
timeout -k 10 300 python -u tools/config_bench.py --frames 5 > gpurun_out/cfg_final_r2i.log 2>&1
