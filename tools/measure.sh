#!/bin/bash
# End-of-round measurement on the GPU box, in two calls (each well inside gpurun's 20-minute limit):
#   a: metric bench (with the CPU baseline), rocprofv3 kernel trace, fp64 PMC passes, configs C2..C5
#   b: fp32 PMC passes, C1 latency and its kernel trace, the MPC tick (tools/mpc_round.sh)
# Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
case "${1:-a}" in
a)
    bash tools/gpu_round.sh bench && bash tools/gpu_round.sh prof && bash tools/gpu_round.sh pmc || exit $?
    for c in c2 c3 c4 c5; do
        timeout -k 10 300 python bench.py --no-cpu-baseline --config $c > "$O/bench_$c.log" 2>&1 || exit $?
    done
    ;;
b)
    PFX=pmc32 BENCH_ARGS=--riccati-fp32 bash tools/pmc.sh || exit $?
    timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 3 > "$O/bench_c1.log" 2>&1 || exit $?
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c1" -o run -- \
        python3 "$R/bench.py" --config c1 --steps 5 --warmup 1 > "$O/prof_c1.log" 2>&1) || exit $?
    bash tools/mpc_round.sh || exit $?
    ;;
esac
exit 0
