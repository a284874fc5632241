#!/bin/bash
# One-wave sweep (k_riccati) at one vs two waves per workgroup (SWEEP_WPB; libhsddp_amd_wpb1.so vs
# the in-tree library), split off, across batch sizes, interleaved twice on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wpb
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for B in 512 1024 2048 4096; do
    for l in wpb1 main; do
      lib=$R/hkd-mpc_amd/libhsddp_amd_$l.so; [ "$l" = main ] && lib=$R/hkd-mpc_amd/libhsddp_amd.so
      HSDDP_SWEEP_SPLIT=0 HSDDP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --batch $B > "$O/${l}_${B}_$rep.log" 2>&1 || exit $?
    done
  done
done
exit 0
