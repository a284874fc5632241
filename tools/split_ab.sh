#!/bin/bash
# Column-split sweep A/B on one box: C2 (B = 1024) and C1 (B = 1) with the split (auto) and with the
# one-wave kernel (HSDDP_SWEEP_SPLIT=0), interleaved twice; then a kernel trace of C2 with the split.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for sp in 1 0; do
    HSDDP_SWEEP_SPLIT=$sp timeout -k 10 200 python bench.py --no-cpu-baseline --config c2 > "$O/split_c2_${sp}_$rep.log" 2>&1 || exit $?
    HSDDP_SWEEP_SPLIT=$sp timeout -k 10 200 python bench.py --config c1 --steps 20 --warmup 3 > "$O/split_c1_${sp}_$rep.log" 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_split_c2" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --config c2 > "$O/prof_split_c2.log" 2>&1 || exit $?
exit 0
