"""Multi-process (world_size 2, gloo) test of the shot sharding + counter all-reduce.

On a GPU node each rank runs the fused HIP launch on its shard and all-reduces
over RCCL; here each rank computes its shard's counters with the CPU oracle (a
test stand-in for the device counters) and the product's own sharding /
all-reduce helpers (:mod:`qldpc_fault_tolerance_amd.parallel`) must reproduce
the single-process totals exactly.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _counter_vector(r):
    return [r["shots"], r["failures"], *r["sector_decodes"], *r["sector_iters"], *r["sector_nonconv"],
            *r["sector_fail"]]


def _worker(rank, world_size, port, total, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import oracle
    from qldpc_fault_tolerance_amd import codes, parallel

    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        r, ws = parallel.world()
        assert (r, ws) == (rank, world_size)
        b, c = parallel.shard_range(total, r, ws, begin=1000)
        code = codes.get_code("hgp_34_n225")
        res = oracle.mc_run(code, 0.03, 0.03, 0.03, seed=11, shot_begin=b, shot_count=c, logical_mode="Total",
                            probs_x=0.06, probs_z=0.06, max_iter=22, precision=32, nthreads=2)
        t = torch.tensor(_counter_vector(res), dtype=torch.int64)
        parallel.allreduce_counters(t)
        if rank == 0:
            q.put(t.tolist())
    finally:
        dist.destroy_process_group()


def test_two_rank_allreduce_equals_single_process(oracle):
    import torch.multiprocessing as mp

    from qldpc_fault_tolerance_amd import codes

    total = 900
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = oracle.mc_run(codes.get_code("hgp_34_n225"), 0.03, 0.03, 0.03, seed=11, shot_begin=1000,
                          shot_count=total, logical_mode="Total", probs_x=0.06, probs_z=0.06, max_iter=22,
                          precision=32, nthreads=2)
    assert got == _counter_vector(whole)
    assert got[0] == total
