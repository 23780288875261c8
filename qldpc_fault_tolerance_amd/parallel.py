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

import ctypes
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


def native_shard_range(total: int, nparts: int, part: int):
    """The split ``qldpc_mc_run_sharded`` applies inside the C ABI (``qldpc_shard_range``; host-only,
    no GPU): must equal :func:`shard_range` (tests/test_distributed_cpu.py)."""
    from . import _native

    b, c = ctypes.c_int64(), ctypes.c_int64()
    _native.check(_native.lib().qldpc_shard_range(int(total), int(nparts), int(part), ctypes.byref(b), ctypes.byref(c)),
                  "qldpc_shard_range")
    return b.value, c.value


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


class NativeComm:
    """An RCCL communicator owned by the engine's C ABI (``qldpc_comm_*``, include/qldpc_hip.h).

    The same counter all-reduce as :func:`allreduce_counters` without torch.distributed: a host
    that binds only ``libqldpc_hip.so`` (the ctypes stub of INTEGRATION.md §3) shards shots over
    GPUs with it.  One process per GPU: rank 0 calls :func:`unique_id`, the host ships the 128
    bytes to every rank, each rank calls ``NativeComm(device, nranks, rank, uid)``.  One process
    driving several GPUs: :meth:`init_all`.
    """

    def __init__(self, device: int = 0, nranks: int = 1, rank: int = 0, uid: bytes | None = None, _handle=None):
        from . import _native

        self.device, self.nranks, self.rank = int(device), int(nranks), int(rank)
        if _handle is not None:
            self.handle = _handle
            return
        if uid is None or len(uid) != _native.COMM_ID_BYTES:
            raise ValueError(f"uid must be the {_native.COMM_ID_BYTES} bytes of unique_id()")
        buf = ctypes.create_string_buffer(bytes(uid), _native.COMM_ID_BYTES)
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_comm_init_rank(self.device, self.nranks, self.rank, buf, ctypes.byref(h)),
                      "qldpc_comm_init_rank")
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        from . import _native

        buf = ctypes.create_string_buffer(_native.COMM_ID_BYTES)
        _native.check(_native.lib().qldpc_comm_unique_id(buf), "qldpc_comm_unique_id")
        return buf.raw

    @staticmethod
    def init_all(devices) -> list:
        """One communicator per listed device, all owned by this process (``ncclCommInitAll``)."""
        from . import _native

        devices = [int(d) for d in devices]
        nd = len(devices)
        darr = (ctypes.c_int32 * nd)(*devices)
        out = (ctypes.c_void_p * nd)()
        _native.check(_native.lib().qldpc_comm_init_all(nd, darr, ctypes.cast(out, ctypes.POINTER(ctypes.c_void_p))),
                      "qldpc_comm_init_all")
        return [NativeComm(d, nd, r, _handle=ctypes.c_void_p(out[r])) for r, d in enumerate(devices)]

    def info(self):
        from . import _native

        v = [ctypes.c_int32() for _ in range(3)]
        _native.check(_native.lib().qldpc_comm_rank(self.handle, *[ctypes.byref(x) for x in v]), "qldpc_comm_rank")
        return {"rank": v[0].value, "nranks": v[1].value, "device": v[2].value}

    def allreduce_counters(self, counters, stream=None):
        """In-place sum of a device ``qldpc_counters`` buffer (an int64 CUDA tensor) on ``stream``
        (default: torch's current stream of the counters' device)."""
        from . import _native

        if stream is None:
            import torch

            stream = ctypes.c_void_p(torch.cuda.current_stream(counters.device).cuda_stream)
        _native.check(_native.lib().qldpc_comm_allreduce_counters(self.handle, ctypes.c_void_p(counters.data_ptr()),
                                                                  stream), "qldpc_comm_allreduce_counters")
        return counters

    def close(self):
        from . import _native

        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_comm_destroy(h)
        self.handle = None

    def __del__(self):
        self.close()
