#!/bin/bash
# MPC tick bench per library variant (interleaved twice)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in 1 2; do
  for l in "$@"; do
    lib=$R/hkd-mpc_amd/libhsddp_amd_$l.so; [ "$l" = main ] && lib=$R/hkd-mpc_amd/libhsddp_amd.so
    HSDDP_LIB=$lib timeout -k 10 200 python tools/mpc_bench.py --batch 4096 > "$R/gpurun_out/mpcab_${l}_$rep.log" 2>&1 || exit $?
  done
done
