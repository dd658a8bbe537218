set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/pmc_lowp.sh gpurun_out/pmc_x3 bf16 > gpurun_out/pmc_x3.txt 2>&1 && timeout -k 10 600 bash tools/ab_x3_tiles.sh > gpurun_out/ab_x3_tiles.txt 2>&1
