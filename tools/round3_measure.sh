#!/bin/bash
# Round-3 measurement on the GPU box: metric bench (with the CPU baseline), rocprofv3 kernel trace,
# PMC passes (fp64 and the C5 fp32 mode), and the BASELINE.json configuration lines C1..C5.
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
exit 0
