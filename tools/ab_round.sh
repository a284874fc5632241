#!/bin/bash
# Parity tests of the in-tree library, then tools/ab_bench.sh over the named libraries
# (e.g. `bash tools/ab_round.sh base main`).  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
bash "$R/tools/ab_bench.sh" "$@"
