"""Shot sharding across GPUs and the counter all-reduce (the path's only collective).

The reference parallelises ``WordErrorRate`` with a fork pool fed one shot at a
time through ``multiprocessing.Queue`` (``parmap``, src/Simulators.py:37-61).
Here every process drives one GPU (``torch.distributed`` rank = local GPU) and
owns a contiguous block of *global shot indices*; since each shot's errors are
keyed by its global index (Philox counter, ``bp_kernels.h``), the totals are
bit-identical for any number of ranks.  After the fused launches the int64
counter vector (``qldpc_counters``: shots, failures, per-sector decodes /
iterations / non-converged / failures, iteration histograms) is summed with ONE
all-reduce — RCCL over xGMI on MI355X nodes (backend ``nccl``), gloo on CPU.
"""
from __future__ import annotations

import os


def world():
    """(rank, world_size) of the initialised default process group, else (0, 1)."""
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except ImportError:
        pass
    return 0, 1


def shard_range(total: int, rank: int, world_size: int, begin: int = 0):
    """Contiguous block ``[b, b+c)`` of ``total`` shots owned by ``rank`` (sizes differ by <= 1)."""
    if world_size <= 0 or not (0 <= rank < world_size):
        raise ValueError("bad rank / world size")
    base, extra = divmod(int(total), int(world_size))
    b = begin + rank * base + min(rank, extra)
    c = base + (1 if rank < extra else 0)
    return b, c


def allreduce_counters(counters):
    """Sum a counter tensor over all ranks in place (no-op when not distributed).

    ``counters`` is an int64 ``torch.Tensor`` on the rank's device (CUDA for
    RCCL, CPU for gloo).  Returns the same tensor.
    """
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM)
    return counters


def local_device_index() -> int:
    """This rank's GPU: LOCAL_RANK from torch.distributed.run (else 0), modulo the visible
    device count when ``QLDPC_SHARE_GPU=1`` (multi-rank rehearsal on fewer GPUs)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("QLDPC_SHARE_GPU") == "1":
        import torch

        local %= max(1, torch.cuda.device_count())
    return local
