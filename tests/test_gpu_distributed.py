"""Sharded HIP solve: two ranks, each solving its disjoint shard of one
global batch on the GPU, gathered to rank 0, equal bit for bit to one process solving the whole
batch — per-element results do not depend on which elements share a launch.  Both ranks run on
the box's one GPU (gloo carries the host-side gather); bench.py runs the same sharding with one GPU
per rank and RCCL."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import hsddp
from hsddp import synthetic as syn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gpu_shard_worker import OPTS  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gpu_shards_equal_single_process(tmp_path):
    world, B = 2, 24
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_shard_worker.py"), str(r), str(world),
                               str(port), str(B), str(tmp_path)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
    full = syn.make_batch(world * B, 4, 20, "trot", mixed=True)
    s = hsddp.Solver(full, hsddp.load_settings(**OPTS))
    s.solve()
    info, tr = s.element_info(), s.trajectory()
    cmds = s.extract_commands()
    s.close()
    from hsddp import shard
    assert np.array_equal(np.load(tmp_path / "summ.npy"), shard.summary_rows(info))
    assert np.array_equal(np.load(tmp_path / "cmds.npy"), shard.command_bytes(cmds))  # device extraction, gathered
    assert np.array_equal(np.load(tmp_path / "xbar.npy"), tr["Xbar"])


def test_bench_rccl_leg_world1():
    """bench.py as a torch.distributed.run rank on the box's one GPU: RCCL (backend "nccl")
    initialises, the timing all_gather and the final gather of summaries and command blocks
    (HKDMPC.cpp:254-286) run through it, and rank 0's line reports the gathered shard."""
    root = os.path.dirname(HERE)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(root, "bench.py"),
           "--gpus", "1", "--batch", "256", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    import json
    out = json.loads(line)
    ex = out["extra"]
    assert ex["rccl_world_size"] == 1
    assert ex["gathered_elements"] == 256
    assert ex["final_gather"]["commands_ok"] and "ms" in ex["final_gather"]
    assert ex["all_costs_finite"]
