#!/bin/bash
# round-4 A/B: the full GPU suite on the in-tree library and on the combined variant, parity of the
# row-pair variant, then the bench over the named libraries
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/exp_pytest_main.log 2>&1 || { echo "main pytest failed"; tail -30 gpurun_out/exp_pytest_main.log; exit 1; }
tail -1 gpurun_out/exp_pytest_main.log
HSDDP_LIB=$PWD/hkd-mpc_amd/libhsddp_amd_ust.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/exp_pytest_combo2.log 2>&1 || { echo "combo2 pytest failed"; tail -30 gpurun_out/exp_pytest_combo2.log; exit 1; }
tail -1 gpurun_out/exp_pytest_combo2.log
HSDDP_LIB=$PWD/hkd-mpc_amd/libhsddp_amd_pairs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/exp_pytest_pairs.log 2>&1 || { echo "pairs pytest failed"; tail -30 gpurun_out/exp_pytest_pairs.log; exit 1; }
bash tools/ab_bench.sh "$@"
