#!/bin/bash
# kernel-trace a short bench run for each library named on the command line (HSDDP_LIB variants)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for l in "$@"; do
    lib=$R/hkd-mpc_amd/libhsddp_amd_$l.so; [ "$l" = main ] && lib=$R/hkd-mpc_amd/libhsddp_amd.so
    HSDDP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kp_$l" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/kp_$l.log" 2>&1 || exit $?
done
exit 0
