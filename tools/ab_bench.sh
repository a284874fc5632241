#!/bin/bash
# Bench every library named on the command line (main = the in-tree libhsddp_amd.so, otherwise
# hkd-mpc_amd/libhsddp_amd_<name>.so) on the same box, interleaved twice; BENCH_ARGS extra args.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for l in "$@"; do
    lib=$R/hkd-mpc_amd/libhsddp_amd_$l.so; [ "$l" = main ] && lib=$R/hkd-mpc_amd/libhsddp_amd.so
    HSDDP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$O/ab_${l}_$rep.log" 2>&1 || exit $?
  done
done
exit 0
