#!/bin/bash
# GPU box: parity suite (including the graph-replay test), smoke, C1 latency with and without the
# iteration graph, the MPC tick at B = 1 / 64 both ways, the metric bench, and a C1 kernel trace.
# Each GPU step has its own limit; any failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
run() { # name, limit, command...
    local name=$1 lim=$2; shift 2
    echo "== $name" >> "$O/round.log"
    timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "$name exit $rc" >> "$O/round.log"
    [ $rc -eq 0 ] || exit $rc
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run c1_graph 300 python bench.py --config c1
HSDDP_NO_GRAPH=1 run c1_nograph 300 python bench.py --config c1
run mpc1_graph 300 python tools/mpc_bench.py --batch 1
HSDDP_NO_GRAPH=1 run mpc1_nograph 300 python tools/mpc_bench.py --batch 1
run mpc64_graph 300 python tools/mpc_bench.py --batch 64
HSDDP_NO_GRAPH=1 run mpc64_nograph 300 python tools/mpc_bench.py --batch 64
run bench 300 python bench.py
cd /tmp && export TMPDIR=/tmp
run prof_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c1" -o run -- \
    python3 "$R/bench.py" --config c1 --steps 3 --warmup 1
exit 0
