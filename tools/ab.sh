#!/bin/bash
# A/B round on the GPU box: parity tests, bench of the in-tree library and of a baseline build
# (HSDDP_LIB), stamps of the diagnostic build.  Stops at the first failing GPU step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > "$O/new.log" 2>&1 || exit $?
if [ -f hkd-mpc_amd/libhsddp_amd_base.so ]; then
    HSDDP_LIB=$R/hkd-mpc_amd/libhsddp_amd_base.so timeout -k 10 200 python bench.py --no-cpu-baseline > "$O/base.log" 2>&1 || exit $?
fi
if [ -f hkd-mpc_amd/libhsddp_amd_stamps.so ]; then
    for b in 1024 4096; do
        STAMP_B=$b HSDDP_LIB=$R/hkd-mpc_amd/libhsddp_amd_stamps.so timeout -k 10 120 python tools/stamps.py > "$O/stamps_$b.log" 2>&1 || exit $?
    done
fi
exit 0
