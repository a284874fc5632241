#!/bin/bash
# PMC passes over k_riccati only (one counter group per rocprofv3 run, no tracing domains).
# Output: gpurun_out/pmcs_<name>/run_counter_collection.csv
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
KERN=${KERN:-k_riccati}
pass() { # name, counters...
    local name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KERN" --output-format csv \
        -d "$O/pmcs_$name" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmcs_$name.log" 2>&1
    local rc=$?
    [ $rc -eq 0 ] || exit $rc
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA
pass b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INSTS_SMEM
exit 0
