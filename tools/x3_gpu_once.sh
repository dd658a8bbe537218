set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/mfma_cases.py --prec f16 > gpurun_out/mfma_cases_f16.txt 2>&1 && timeout -k 10 120 python -u tools/mfma_cases.py --prec bf16 > gpurun_out/mfma_cases_bf16.txt 2>&1
