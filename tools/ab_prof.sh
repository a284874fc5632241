#!/bin/bash
# GPU parity tests of the in-tree library, then a rocprofv3 kernel trace of every library named on
# the command line (tools/prof_libs.sh).  A test failure (exit 1) still profiles; any other non-zero
# exit (fault, abort, time limit) ends the call there.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"
[ $rc -le 1 ] || exit $rc
bash "$R/tools/prof_libs.sh" "$@"
