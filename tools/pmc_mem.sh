#!/bin/bash
# Memory-pipeline PMC passes (TA / TCP) for the knot-parallel kernels over a short bench run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
KERN=${KERN:-'k_rollout|k_lq|k_lin_rollout|k_riccati'}
pass() {
    local name=$1; shift
    timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-include-regex "$KERN" --output-format csv \
        -d "$O/pmc_$name" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
        > "$O/pmc_$name.log" 2>&1 || exit $?
}
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
pass tcp TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum
pass sqb SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
exit 0
