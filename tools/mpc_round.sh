#!/bin/bash
# The MPC tick benchmark (tools/mpc_bench.py) at B = 4096 (asynchronous and synchronous command
# extraction), 64 and 1, then a rocprofv3 kernel trace of the B = 4096 run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 300 python tools/mpc_bench.py --batch 4096 > "$O/mpc_4096.log" 2>&1 || exit $?
timeout -k 10 300 python tools/mpc_bench.py --batch 4096 --sync > "$O/mpc_4096_sync.log" 2>&1 || exit $?
timeout -k 10 300 python tools/mpc_bench.py --batch 64 > "$O/mpc_64.log" 2>&1 || exit $?
timeout -k 10 300 python tools/mpc_bench.py --batch 1 > "$O/mpc_1.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_mpc" -o run -- \
    python3 "$R/tools/mpc_bench.py" --batch 4096 > "$O/prof_mpc.log" 2>&1 || exit $?
exit 0
