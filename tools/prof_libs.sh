#!/bin/bash
# rocprofv3 kernel trace of `bench.py --steps 5` for every library named on the command line
# (main = the in-tree libhsddp_amd.so, otherwise hkd-mpc_amd/libhsddp_amd_<name>.so), one after
# another on the same box: per-kernel durations of A/B variants (gpurun_out/prof_<name>/).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for l in "$@"; do
    lib=$R/hkd-mpc_amd/libhsddp_amd_$l.so; [ "$l" = main ] && lib=$R/hkd-mpc_amd/libhsddp_amd.so
    export HSDDP_LIB=$lib
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$l" -o run -- \
        python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/prof_$l.log" 2>&1 || exit $?
done
exit 0
