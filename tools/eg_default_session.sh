set -o pipefail
O=gpurun_out
timeout -k 10 120 python -u tools/itmap.py > $O/itmap.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_endgame.py tests/test_gpu_lowp_contract.py -m gpu -v --timeout 600 --timeout-method thread > $O/eg_tests_3e4.log 2>&1
