"""Data-parallel training step (BASELINE configs[3]).

One process per GPU; each rank trains on its own shard of egs (weak scaling) and
the ranks exchange exactly one thing per step: the weight gradient, averaged over
ranks before the identical SGD update on every rank. The reference has no
multi-GPU code (it selects one device, cpp/cuda/bridge.cu:38-47); the minibatch
semantics match one process running world x egs_per_rank egs with the gradient
averaged over ranks.

The exchange is native: ``Communicator`` wraps the kf_dp_* C-ABI
(include/kf_dp.h, csrc/dp.cpp) over RCCL, and ``Network.bind_dp`` makes
nnet_backward all-reduce the gradient in buckets on a high-priority communication
stream while the rest of the backward runs (the bucket plan is kf_dp_plan's).
torch.distributed only carries the 128-byte RCCL unique id at start-up and the
timing / statistics reductions of the bench, as any out-of-band channel would.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 16 << 20


def env():
    """(rank, local_rank, world) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def eg_index(rank: int, egs_per_rank: int, e: int) -> int:
    """Global index of this rank's e-th eg (drives its synthetic seeds)."""
    return rank * egs_per_rank + e


def _core():
    from . import core
    return core


def _dp_err(core):
    s = core.kf_dp_last_error()
    return s.decode() if s else "unknown error"


def unique_id() -> bytes:
    """ncclGetUniqueId (kf_dp_unique_id), on rank 0."""
    core = _core()
    buf = C.create_string_buffer(128)
    if core.kf_dp_unique_id(buf) != 0:
        raise RuntimeError("kf_dp_unique_id: " + _dp_err(core))
    return buf.raw


def broadcast_id(id_bytes: bytes | None, device) -> bytes:
    """Rank 0's 128-byte id to every rank through the torch.distributed group."""
    t = torch.zeros(128, dtype=torch.uint8, device=device)
    if dist.get_rank() == 0:
        t.copy_(torch.frombuffer(bytearray(id_bytes), dtype=torch.uint8))
    dist.broadcast(t, 0)
    return bytes(t.cpu().numpy().tobytes())


class Communicator:
    """This rank's RCCL communicator (kf_dp_create) and its communication stream."""

    def __init__(self, rank: int, world: int, id_bytes: bytes, device: int):
        core = _core()
        self.h = core.kf_dp_create(int(rank), int(world), C.c_char_p(bytes(id_bytes)), int(device))
        if not self.h:
            raise RuntimeError("kf_dp_create: " + _dp_err(core))
        self.rank, self.world = rank, world

    @classmethod
    def from_process_group(cls, device: int):
        """Collective over the default torch.distributed group: rank 0 makes the id."""
        dev = torch.device("cuda", device) if dist.get_backend() == "nccl" else "cpu"
        uid = unique_id() if dist.get_rank() == 0 else None
        return cls(dist.get_rank(), dist.get_world_size(), broadcast_id(uid, dev), device)

    def allreduce_mean(self, ptr, count: int):
        """In-place average over ranks of `count` fp32 values at device `ptr`,
        stream-ordered on the library's current stream."""
        core = _core()
        if core.kf_dp_allreduce_mean(self.h, ptr, int(count)) != 0:
            raise RuntimeError("kf_dp_allreduce_mean: " + _dp_err(core))

    def allreduce_sum_f64(self, ptr, count: int):
        core = _core()
        if core.kf_dp_allreduce_sum_f64(self.h, ptr, int(count)) != 0:
            raise RuntimeError("kf_dp_allreduce_sum_f64: " + _dp_err(core))

    DEBUG_SNAPSHOT, DEBUG_PEER_MEAN = 1, 2

    def debug(self, mode: int, grad_base=None, aux_base=None, count: int = 0):
        """kf_dp_debug test hooks: DEBUG_SNAPSHOT copies each bucket to aux (same offset
        from grad_base) as its exchange starts; DEBUG_PEER_MEAN averages each exchanged
        bucket with aux, a second rank's gradient. 0 turns them off. count: fp32 values
        of both buffers (buckets outside them then fail)."""
        core = _core()
        if core.kf_dp_debug(self.h, int(mode), grad_base, aux_base, int(count)) != 0:
            raise RuntimeError("kf_dp_debug: " + _dp_err(core))

    def stats(self):
        """(all-reduce launches, fp32 values exchanged) since creation."""
        n, v = C.c_longlong(), C.c_longlong()
        _core().kf_dp_stats(self.h, C.byref(n), C.byref(v))
        return n.value, v.value

    def close(self):
        if getattr(self, "h", None):
            _core().kf_dp_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan(lo, hi, total: int, bucket_elems: int, max_buckets: int = 256):
    """kf_dp_plan over explicit groups: [(after_step, begin, end)]."""
    core = _core()
    n = len(lo)
    L = (C.c_longlong * max(n, 1))(*lo)
    H = (C.c_longlong * max(n, 1))(*hi)
    a = (C.c_int * max_buckets)()
    b = (C.c_longlong * max_buckets)()
    e = (C.c_longlong * max_buckets)()
    nb = core.kf_dp_plan(n, L, H, int(total), int(bucket_elems), max_buckets, a, b, e)
    if nb < 0:
        raise RuntimeError("kf_dp_plan: " + _dp_err(core))
    return [(a[i], b[i], e[i]) for i in range(nb)]


def exchange_by_plan(flat: torch.Tensor, buckets, world: int):
    """What nnet_backward does with a bound communicator, restated on a torch tensor
    with torch.distributed (the gloo CPU tests): every bucket averaged over ranks in
    issue order. Test helper, not the product path."""
    for _, b, e in buckets:
        seg = flat[b:e]
        dist.all_reduce(seg, op=dist.ReduceOp.SUM)
        seg.mul_(1.0 / world)
    return flat


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


def covers_exactly(buckets, total: int) -> bool:
    """The buckets partition [0, total)."""
    seen = np.zeros(total, dtype=np.int8)
    for _, b, e in buckets:
        seen[b:e] += 1
    return bool((seen == 1).all())
