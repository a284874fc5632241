#!/bin/bash
# Vector-memory counters of the rollout kernels (k_rollout, k_lin_rollout): L1 (TCP) requests to L2,
# L1 accesses, TA busy / stalls, L2 hits and misses — the addressing cost of row-per-lane accesses.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() { # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex 'k_rollout|k_lin_rollout' --output-format csv \
      -d "$O/romem_$n" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/romem_$n.log" 2>&1 || exit $?
}
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
run tcc TCC_HIT_sum TCC_MISS_sum TCC_READ_REQ_sum TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE
exit 0
