#!/bin/bash
# LDS counters of the sweep (k_riccati) at several batch sizes (one-wave kernel): array-busy cycles,
# bank conflicts, LDS instruction count and wait, against wave and busy cycles.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for B in ${BATCHES:-512 1024 4096}; do
  HSDDP_SWEEP_SPLIT=${SPLIT:-0} timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS \
      SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-include-regex 'k_riccati' \
      --output-format csv -d "$O/lds_$B" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --batch $B \
      > "$O/lds_$B.log" 2>&1 || exit $?
done
exit 0
