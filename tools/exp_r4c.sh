#!/bin/bash
# round-4 defaults check: the full GPU suite and smoke() on the in-tree library, parity of the
# U-staging variant, then the bench over the named libraries (r4base: the session's kernels before
# the write-line changes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4c_pytest.log; exit 1; }
tail -1 gpurun_out/r4c_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4c_smoke.log; exit 1; }
tail -1 gpurun_out/r4c_smoke.log
HSDDP_LIB=$PWD/hkd-mpc_amd/libhsddp_amd_ust.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py tests/test_gpu_mpc.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4c_pytest_ust.log 2>&1 || { echo "ust pytest failed"; tail -30 gpurun_out/r4c_pytest_ust.log; exit 1; }
bash tools/ab_bench.sh "$@"
