#!/bin/bash
# round-4 final GPU calls.  a: the full GPU suite, smoke(), then tools/round4_measure.sh a;
# b: tools/round4_measure.sh b.  Stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ "${1:-a}" = a ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4_pytest_gpu.log; exit 1; }
    tail -1 gpurun_out/r4_pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4_smoke.log; exit 1; }
    tail -1 gpurun_out/r4_smoke.log
fi
bash tools/round4_measure.sh "${1:-a}"
