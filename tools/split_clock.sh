#!/bin/bash
# Effective clock of the sweep kernels with and without the column split at B = 512 and 1024
# (GRBM_GUI_ACTIVE / 8 / kernel time, MI355X_MICROARCH.md "DVFS give-back"), one PMC pass each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for B in 512 1024; do
  for sp in 1 0; do
    HSDDP_SWEEP_SPLIT=$sp timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex 'k_riccati' \
        --output-format csv -d "$O/clk_${B}_$sp" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --batch $B \
        > "$O/clk_${B}_$sp.log" 2>&1 || exit $?
  done
done
exit 0
