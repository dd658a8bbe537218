set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_x3_normals.py tests/test_gpu_lowp_contract.py tests/test_gpu_lowp.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py > gpurun_out/t1_tests.log 2>&1
