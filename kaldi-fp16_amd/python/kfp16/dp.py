"""Data-parallel plumbing of the training step.

One process per GPU; each rank trains on its own shard of egs (weak scaling) and
the ranks exchange exactly one thing per step: the flat fp32 gradient, summed by
an all-reduce (RCCL over xGMI with the "nccl" backend, gloo on CPU) and scaled by
1/world before the identical SGD update on every rank. The reference has no
multi-GPU code; the minibatch semantics match one process running
world x egs_per_rank egs with the gradient averaged over ranks.
Pure torch.distributed; no device kernels here.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env():
    """(rank, local_rank, world) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def eg_index(rank: int, egs_per_rank: int, e: int) -> int:
    """Global index of this rank's e-th eg (drives its synthetic seeds)."""
    return rank * egs_per_rank + e


def allreduce_mean_(grad: torch.Tensor, world: int) -> torch.Tensor:
    """In-place sum over ranks, then 1/world (the gradient the SGD sees)."""
    if world > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM)
        grad.mul_(1.0 / world)
    return grad


def max_over_ranks(x: float, device) -> float:
    """The step time every rank reports is the slowest rank's."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device):
    """Objective statistics {objf, num, den, frames, ok} summed over ranks."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()
