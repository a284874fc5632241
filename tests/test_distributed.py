"""Multi-process path on CPU (gloo, world_size 2 and 4): the batch shards by element with no exchange
during the solve; only a final gather of per-element summaries.  The HIP solve is
replaced here by the oracle because this container has no GPU; bench.py runs the same sharding
with the HIP path and RCCL on the GPU box."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from hsddp import synthetic as syn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _commands(prob, r):
    """every element's command block (publish_mpc_cmd, HKDMPC.cpp:232-298) from the oracle solve,
    as the hsddp_mpc_command records the GPU path extracts"""
    import sys
    import hsddp
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import mpc_oracle as M
    out = np.zeros(prob["batch"], dtype=hsddp.MPC_COMMAND)
    P = len(prob["horizons"])
    for b in range(prob["batch"]):
        c = M.mpc_command(r["Xbar"][b], r["Ubar"][b], r["K"][b], prob["contacts"][b], prob["horizons"], 1, 0.0, 0.01,
                          np.zeros((P, 4)), np.zeros(12, np.float32), 0.0)
        for f, v in c.items():
            out[b][f] = v
    return out


def _worker(rank, world, port, B, out_dir):
    import torch
    import oracle_lib as O
    from hsddp import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = syn.make_batch(B, 2, 8, "trot", first_element=rank * B)
    r = O.solve_batch(prob, O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2))
    r["status"] = r["status"].astype(np.float64)
    # bench.py's final gather (hsddp/shard.py): summaries and command blocks to rank 0
    summ = torch.from_numpy(shard.summary_rows(r))
    cmd = torch.from_numpy(shard.command_bytes(_commands(prob, r)))
    rows, cmds = shard.final_gather(dist, summ, cmd)
    x0 = torch.from_numpy(prob["x0"])
    g_x = [torch.empty_like(x0) for _ in range(world)] if rank == 0 else None
    dist.gather(x0, g_x, dst=0)
    if rank == 0:
        np.save(os.path.join(out_dir, "summ.npy"), rows)
        np.save(os.path.join(out_dir, "x0.npy"), torch.cat(g_x).numpy())
        np.save(os.path.join(out_dir, "cmds.npy"), shard.command_bytes(cmds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_rank_shards_and_gather(tmp_path, world):
    import oracle_lib as O
    B = 3
    mp.spawn(_worker, args=(world, _free_port(), B, str(tmp_path)), nprocs=world, join=True)
    full = syn.make_batch(world * B, 2, 8, "trot")
    assert np.array_equal(np.load(tmp_path / "x0.npy"), full["x0"])  # disjoint, reproducible shards
    r = O.solve_batch(full, O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2))
    from hsddp import shard
    r["status"] = r["status"].astype(np.float64)
    assert np.array_equal(np.load(tmp_path / "summ.npy"), shard.summary_rows(r))  # sharding changes nothing per element
    # the gathered command blocks are the full batch's, element for element
    assert np.array_equal(np.load(tmp_path / "cmds.npy"), shard.command_bytes(_commands(full, r)))
