#!/bin/bash
# round-4 kernel experiments: parity of a variant library, then the A/B bench over the named libraries
# usage: bash tools/exp_r4.sh <variant-for-parity> <libs...>
set -o pipefail
mkdir -p gpurun_out
V=$1; shift
HSDDP_LIB=$PWD/hkd-mpc_amd/libhsddp_amd_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py tests/test_gpu_mpc.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/exp_pytest_$V.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/exp_pytest_$V.log; exit 1; }
tail -2 gpurun_out/exp_pytest_$V.log
bash tools/ab_bench.sh "$@"
