set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lowp_contract.py -v --timeout 300 --timeout-method thread > gpurun_out/contract_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_lowp_contract.py > gpurun_out/gputests.log 2>&1
