set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_round.sh bench && bash tools/gpu_round.sh prof && bash tools/gpu_round.sh pmc || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --gait jump --phases 8 --knots 25 > gpurun_out/bench_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --riccati-fp32 > gpurun_out/bench_fp32.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --mixed > gpurun_out/bench_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 1024 > gpurun_out/bench_c1.log 2>&1 || exit $?
