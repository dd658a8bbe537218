# GPU box: endgame threshold sweep (C3-C5 timing at tau 0 / 1e-4 / 3e-4 / 1e-3), the contract tests
# at tau 3e-4, then the single-frame tail stamps (fp32, bf16)
set -o pipefail
O=gpurun_out
timeout -k 10 120 python -u tools/tail_stamps.py --out $O/tail_f32.npz > $O/tail_f32.txt 2>&1 &&
timeout -k 10 120 python -u tools/tail_stamps.py --precision bf16 --out $O/tail_bf16.npz > $O/tail_bf16.txt 2>&1 &&
timeout -k 10 400 python -u tools/config_bench.py --frames 5 --only C3,C4-full,C5 --endgame 0,0.0001,0.0003,0.001 > $O/cfg_tau.log 2>&1 &&
NR_TEST_EG_TAU=0.0003 timeout -k 10 900 python -u -m pytest tests/test_gpu_lowp_contract.py -m gpu -v -k endgame --timeout 600 --timeout-method thread > $O/contract_tau3e4.log 2>&1
