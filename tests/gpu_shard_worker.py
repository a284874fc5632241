"""Test helper (tests/test_gpu_distributed.py): one rank of a sharded HIP solve on cuda:0.

    python tests/gpu_shard_worker.py <rank> <world> <port> <batch_per_rank> <out_dir>

Each rank solves its disjoint shard of one global synthetic batch (mixed gaits) through the C-ABI,
then the per-element summaries and nominal trajectories are gathered to rank 0 (gloo, host
tensors) — the multi-GPU path of bench.py with every rank on the one GPU of the box."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp  # noqa: E402
from hsddp import shard, synthetic as syn  # noqa: E402

OPTS = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=3)


def main():
    rank, world, port, B = (int(a) for a in sys.argv[1:5])
    out = sys.argv[5]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    part = syn.make_batch(B, 4, 20, "trot", mixed=True, first_element=rank * B)
    s = hsddp.Solver(part, hsddp.load_settings(**OPTS), device=0)
    s.solve()
    info, tr = s.element_info(), s.trajectory()
    # the command block extracted on the device into a torch tensor (as bench.py), sent from the host
    cmd = torch.empty(B * hsddp.MPC_COMMAND.itemsize, dtype=torch.uint8, device="cuda:0")
    s.extract_commands_device(cmd.data_ptr())
    s.close()
    rows, cmds = shard.final_gather(dist, torch.from_numpy(shard.summary_rows(info)), cmd.cpu())
    xbar = torch.from_numpy(np.ascontiguousarray(tr["Xbar"]))
    gx = [torch.empty_like(xbar) for _ in range(world)] if rank == 0 else None
    dist.gather(xbar, gx, dst=0)
    if rank == 0:
        np.save(os.path.join(out, "summ.npy"), rows)
        np.save(os.path.join(out, "cmds.npy"), shard.command_bytes(cmds))
        np.save(os.path.join(out, "xbar.npy"), torch.cat(gx).numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
