#!/bin/bash
# Round-4 measurement on the GPU box: metric bench (with the CPU baseline), rocprofv3 kernel trace,
# PMC passes (fp64 and the C5 fp32 mode), the BASELINE.json configuration lines C1..C5, and the MPC
# tick (tools/mpc_bench.py: asynchronous extraction at B = 4096 / 64 / 1, the synchronous one at
# 4096, and a kernel trace of the 4096 run).  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
bash tools/gpu_round.sh bench && bash tools/gpu_round.sh prof && bash tools/gpu_round.sh pmc || exit $?
PFX=pmc32 BENCH_ARGS=--riccati-fp32 bash tools/pmc.sh || exit $?
for c in c2 c3 c4 c5; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --config $c > "$O/bench_$c.log" 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 3 > "$O/bench_c1.log" 2>&1 || exit $?
bash tools/mpc_round.sh || exit $?
exit 0
