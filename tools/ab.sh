#!/bin/bash
# A/B round on the GPU box: parity tests, bench of the in-tree library and of a baseline build
# (hkd-mpc_amd/libhsddp_amd_base.so via HSDDP_LIB, when present).  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > "$O/new.log" 2>&1 || exit $?
if [ -f hkd-mpc_amd/libhsddp_amd_base.so ]; then
    HSDDP_LIB=$R/hkd-mpc_amd/libhsddp_amd_base.so timeout -k 10 200 python bench.py --no-cpu-baseline > "$O/base.log" 2>&1 || exit $?
fi
exit 0
