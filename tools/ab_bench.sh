#!/bin/bash
# A/B of libraries on one box: every library named on the command line (main = the in-tree
# libhsddp_amd.so, otherwise hkd-mpc_amd/libhsddp_amd_<name>.so; name=VAR=value runs the in-tree
# library with that environment variable set, e.g. split0=HSDDP_SWEEP_SPLIT=0), interleaved REPS
# times (default 2), at every batch size of BATCHES (default: the bench's own), with BENCH_ARGS
# extra bench arguments; logs under gpurun_out/${AB_DIR:-.}/<name>_<batch>_<rep>.log.
# (Replaces round 5's one-off wpb_ab.sh / wpe_ab.sh / split_ab.sh: wpb1 wpe2 main, BATCHES="512 1024
# 2048 4096"; split1=HSDDP_SWEEP_SPLIT=1 split0=HSDDP_SWEEP_SPLIT=0, BENCH_ARGS="--config c2".)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${AB_DIR:-.}
mkdir -p "$O"
cd "$R"
for rep in $(seq 1 "${REPS:-2}"); do
  for B in ${BATCHES:-default}; do
    barg=""; [ "$B" = default ] || barg="--batch $B"
    for spec in "$@"; do
      name=${spec%%=*}
      envv=""; [ "$spec" = "$name" ] || envv=${spec#*=}
      lib=$R/hkd-mpc_amd/libhsddp_amd_$name.so
      { [ "$name" = main ] || [ -n "$envv" ]; } && lib=$R/hkd-mpc_amd/libhsddp_amd.so
      env HSDDP_LIB="$lib" $envv timeout -k 10 200 python bench.py --no-cpu-baseline $barg ${BENCH_ARGS:-} \
          > "$O/${name}_${B}_$rep.log" 2>&1 || exit $?
    done
  done
done
exit 0
