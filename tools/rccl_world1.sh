#!/bin/bash
# GPU box: bench.py's RCCL leg at world size 1 (torch.distributed.run, one rank on the box's GPU):
# the GPU test of it, then the metric line through the RCCL path.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_graph.py -m gpu -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread > "$O/pytest_rccl.log" 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --no-cpu-baseline > "$O/bench_rccl1.log" 2>&1 || exit $?
exit 0
