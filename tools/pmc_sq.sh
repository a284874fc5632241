#!/bin/bash
# One SQ counter pass (wave cycles, waits, VALU/LDS/SALU instruction counts) for the kernels in $KERN.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
KERN=${KERN:-'k_rollout|k_lq|k_lin_rollout|k_riccati|k_terminal'}
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --kernel-include-regex "$KERN" --output-format csv -d "$O/pmc_sq" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_sq.log" 2>&1
