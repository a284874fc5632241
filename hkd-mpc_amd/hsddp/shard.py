"""The multi-GPU exchange of the batched solve: every rank solves its own disjoint
shard of the batch with no exchange during the solve; afterwards one gather to rank 0 of

* the per-element summary rows (cost, feasibility, max terminal / path violation, inner iterations,
  status: 48 B per element), and
* optionally the command block of every element — the hkd_command_lcmt record of
  HKDMPCSolver::publish_mpc_cmd (first knots' Ubar, body states, 12 x 12 feedback gains ...,
  HKDMPC.cpp:232-298; 7.8 KB per element), extracted on the device straight into the tensor the
  collective sends (hsddp_extract_commands_device).

Used by bench.py (RCCL, device tensors) and tests/test_distributed.py (gloo, host tensors), so the
CPU test runs the same gather code as the GPU run."""
from __future__ import annotations

import numpy as np

from ._lib import MPC_COMMAND

SUMMARY_FIELDS = ("cost", "feas", "max_tconstr", "max_pconstr", "iters", "status")


def summary_rows(info: dict) -> np.ndarray:
    """[B][6] float64 summary rows of hsddp_element_info fields."""
    return np.stack([np.asarray(info[f], dtype=np.float64) for f in SUMMARY_FIELDS], 1)


def final_gather(dist, summ, cmd=None):
    """Gather the summaries (torch [B][6] float64) and the command bytes (torch uint8 [B * 7824] or
    None) of every rank to rank 0.  Returns (summaries [world * B][6], commands record array
    [world * B] or None) on rank 0, (None, None) elsewhere."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    gs = [torch.empty_like(summ) for _ in range(world)] if rank == 0 else None
    dist.gather(summ, gs, dst=0)
    gc = None
    if cmd is not None:
        gc = [torch.empty_like(cmd) for _ in range(world)] if rank == 0 else None
        dist.gather(cmd, gc, dst=0)
    if rank != 0:
        return None, None
    rows = torch.cat(gs).cpu().numpy()
    cmds = None
    if gc is not None:
        raw = torch.cat(gc).cpu().numpy()
        cmds = np.frombuffer(raw.tobytes(), dtype=MPC_COMMAND)
    return rows, cmds


def command_bytes(records: np.ndarray) -> np.ndarray:
    """hsddp_mpc_command records as the uint8 stream the gather sends."""
    return np.frombuffer(np.ascontiguousarray(records, dtype=MPC_COMMAND).tobytes(), dtype=np.uint8).copy()
