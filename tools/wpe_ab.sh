#!/bin/bash
# Two-pair sweep workgroups with a one-wave-per-SIMD register budget (in-tree library) against the
# two-wave budget (libhsddp_amd_wpe2.so) at B = 1024 and 2048, interleaved twice on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wpe
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for B in 1024 2048; do
    for l in wpe2 main; do
      lib=$R/hkd-mpc_amd/libhsddp_amd_$l.so; [ "$l" = main ] && lib=$R/hkd-mpc_amd/libhsddp_amd.so
      HSDDP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --batch $B > "$O/${l}_${B}_$rep.log" 2>&1 || exit $?
    done
  done
done
exit 0
