#!/bin/bash
# GPU-box round: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; any exit status other than 0 (pass) or 1 (test failure) stops the script, so a
# fault, abort, segfault or timeout never leads to another GPU launch in the same call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
step() { # name, limit, command...
    local name=$1 lim=$2; shift 2
    echo "== $name" >> "$O/round.log"
    timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "$name exit $rc" >> "$O/round.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >> "$O/round.log"; exit $rc; fi
    return $rc
}
MODE=${1:-all}
cd "$R"
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    cd /tmp && export TMPDIR=/tmp
    step rocprof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_trace" -o run -- \
        python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline
    cd "$R"
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
    bash "$R/tools/pmc.sh" || exit $?
fi
# config C5: fp32 Riccati mode — bench line, tolerance against fp64, kernel trace and PMC traffic
if [ "$MODE" = all ] || [ "$MODE" = fp32 ]; then
    step bench_fp32 300 python bench.py --riccati-fp32
    step fp32_tolerance 600 python -u tools/fp32_tolerance.py
    cd /tmp && export TMPDIR=/tmp
    step rocprof_trace_fp32 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_trace_fp32" -o run -- \
        python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --riccati-fp32
    cd "$R"
    PFX=pmc32 BENCH_ARGS=--riccati-fp32 bash "$R/tools/pmc.sh" || exit $?
fi
exit 0
