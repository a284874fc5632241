#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains) over a short bench run.
# Output: gpurun_out/pmc_<name>/run_counter_collection.csv
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
KERN='k_riccati|k_lin_rollout|k_lq|k_rollout|k_decide|k_terminal'
# PFX: output-directory prefix; BENCH_ARGS: extra bench.py arguments (e.g. --riccati-fp32)
PFX=${PFX:-pmc}
BENCH_ARGS=${BENCH_ARGS:-}
pass() { # name, counters...
    local name=$1; shift
    echo "== $PFX $name" >> "$O/round.log"
    timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-include-regex "$KERN" --output-format csv \
        -d "$O/${PFX}_$name" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
        > "$O/${PFX}_$name.log" 2>&1
    local rc=$?
    echo "$PFX $name exit $rc" >> "$O/round.log"
    [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
pass fetch FETCH_SIZE
pass write WRITE_SIZE
exit 0
