"""Multi-process path on CPU (gloo, world_size 2): the batch shards by element with no exchange
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


def _worker(rank, world, port, B, out_dir):
    import torch
    import oracle_lib as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = syn.make_batch(B, 2, 8, "trot", first_element=rank * B)
    r = O.solve_batch(shard, O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2))
    summ = torch.from_numpy(np.stack([r["cost"], r["feas"], r["max_tconstr"], r["max_pconstr"]], 1))
    x0 = torch.from_numpy(shard["x0"])
    if rank == 0:
        g_s = [torch.empty_like(summ) for _ in range(world)]
        g_x = [torch.empty_like(x0) for _ in range(world)]
    else:
        g_s = g_x = None
    dist.gather(summ, g_s, dst=0)
    dist.gather(x0, g_x, dst=0)
    if rank == 0:
        np.save(os.path.join(out_dir, "summ.npy"), torch.cat(g_s).numpy())
        np.save(os.path.join(out_dir, "x0.npy"), torch.cat(g_x).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_and_gather(tmp_path):
    import oracle_lib as O
    world, B = 2, 3
    mp.spawn(_worker, args=(world, _free_port(), B, str(tmp_path)), nprocs=world, join=True)
    full = syn.make_batch(world * B, 2, 8, "trot")
    assert np.array_equal(np.load(tmp_path / "x0.npy"), full["x0"])  # disjoint, reproducible shards
    r = O.solve_batch(full, O.default_options(no_early_exit=1, max_AL_iter=1, max_DDP_iter=2))
    ref = np.stack([r["cost"], r["feas"], r["max_tconstr"], r["max_pconstr"]], 1)
    assert np.array_equal(np.load(tmp_path / "summ.npy"), ref)  # sharding changes nothing per element
