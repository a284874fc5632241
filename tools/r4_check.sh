#!/bin/bash
# Round-4 check on one box: the parity / MPC GPU tests, an A/B of the named libraries
# (tools/ab_bench.sh) and the MPC tick bench in both extraction modes.  Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mpc.py tests/test_gpu_reference.py -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > "$O/r4_check_pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -30 "$O/r4_check_pytest.log"; exit 1; }
tail -1 "$O/r4_check_pytest.log"
bash "$R/tools/ab_bench.sh" "$@" || exit $?
timeout -k 10 200 python tools/mpc_bench.py --batch 4096 --ticks 20 > "$O/r4_mpc_4096_async.json" 2>&1 || exit $?
timeout -k 10 200 python tools/mpc_bench.py --batch 4096 --ticks 20 --sync > "$O/r4_mpc_4096_sync.json" 2>&1 || exit $?
timeout -k 10 100 python tools/mpc_bench.py --batch 1 --ticks 20 > "$O/r4_mpc_1.json" 2>&1 || exit $?
python - <<'PY'
import json, glob, os
O = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
for f in sorted(glob.glob(os.path.join(O, "ab_*_*.log"))):
    lines = [x for x in open(f) if x.startswith("{")]
    if lines:
        d = json.loads(lines[-1]); e = d.get("extra", {})
        print(os.path.basename(f), round(d["value"]), d["ms_per_step"], e.get("device_ms_per_step"))
for f in sorted(glob.glob(os.path.join(O, "r4_mpc_*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), d["ms_per_tick_median"], round(d["robot_ticks_per_s"]), d.get("last_copy_wait_ms"))
PY
