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


# ----------------------------------------------------------------------------------------------
# The product's own fused_counts path (CodeSimulator_DataError) across 2 gloo ranks, with a stub
# device counter standing in for the HIP launch: the stub credits every global shot index it is
# given with deterministic per-shot counts, so the all-reduced totals show that the simulator's
# sharding (parallel.shard_range over the running shot offset) covers every shot exactly once,
# across consecutive WordErrorRate calls and adaptive batches.


def _stub_counts(b, c):
    """Per-shot deterministic counters of global shots [b, b+c): (shots, failures, iters)."""
    idx = np.arange(b, b + c, dtype=np.int64)
    return c, int(np.sum(idx % 7 == 3)), int(np.sum(idx % 11))


class _StubMC:
    """Stands in for engine.DeviceMC: counters on the CPU, filled per launched shot range."""

    device = 0
    launched = []

    def new_counters(self):
        import torch

        from qldpc_fault_tolerance_amd import _native

        return torch.zeros(_native.COUNTER_WORDS, dtype=torch.int64)

    def launch(self, px, py, pz, seed, shot_begin, shot_count, logical_mode, counters, *a, **k):
        s, f, it = _stub_counts(shot_begin, shot_count)
        _StubMC.launched.append((shot_begin, shot_count))
        counters[0] += s
        counters[1] += f
        counters[2] += s
        counters[4] += it


def _patch_engine(sim):
    import torch

    from qldpc_fault_tolerance_amd import engine

    class _T:
        cuda = type("C", (), {"synchronize": staticmethod(lambda *a, **k: None)})

    engine._torch = lambda: _T  # noqa: E731 (the stub counters live on the CPU)
    sim._engine_ready = lambda: (True, object(), object())
    sim._mc = _StubMC()
    return torch


def _sim_worker(rank, world_size, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from qldpc_fault_tolerance_amd import codes, simulators

    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        code = codes.get_code("hgp_34_n225")
        sim = simulators.CodeSimulator_DataError(code=code, pauli_error_probs=[0.01] * 3, eval_logical_type="Total",
                                                 seed=5)
        _patch_engine(sim)
        r1 = sim.fused_counts(1001)  # odd total: shards of 501 / 500
        r2 = sim.fused_counts(250)   # continues the global shot stream at 1001
        wer, total = sim.WordErrorRate_TargetFailure(target_failures=40, batch_size=97, max_batches=50)
        q.put((rank, [r1.shots, r1.failures, r1.sector_iters[0]], [r2.shots, r2.failures, r2.sector_iters[0]],
               total, list(_StubMC.launched)))
    finally:
        dist.destroy_process_group()


def test_two_rank_fused_counts_sharding_covers_every_shot_once():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sim_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=240) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, a1, a2, tot0, l0), (_, b1, b2, tot1, l1) = got
    assert a1 == b1 and a2 == b2 and tot0 == tot1  # every rank holds the all-reduced totals
    s, f, it = _stub_counts(0, 1001)
    assert a1 == [s, f, it]
    s, f, it = _stub_counts(1001, 250)
    assert a2 == [s, f, it]
    # the two ranks' launches tile the global shot range without overlap or gap
    spans = sorted(l0 + l1)
    pos = 0
    for b, c in spans:
        assert b == pos
        pos = b + c
    assert pos == 1001 + 250 + tot0
    # adaptive batches stopped at the same (first) batch reaching the target on both ranks
    fails = [_stub_counts(1251 + 97 * i, 97)[1] for i in range(tot0 // 97)]
    assert sum(fails) >= 40 and sum(fails[:-1]) < 40


def test_decoders_default_to_local_rank_device(monkeypatch):
    """drop-in decoders resolve device=None to LOCAL_RANK (one rank per GPU)."""
    from qldpc_fault_tolerance_amd import parallel

    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.delenv("QLDPC_SHARE_GPU", raising=False)
    assert parallel.local_device_index() == 3
    import inspect

    from qldpc_fault_tolerance_amd import decoders, engine

    for cls in (decoders.BPDecoder, decoders.BPOSD_Decoder, decoders.ST_BP_Decoder_syndrome, decoders.BP_Decoder_Class,
                decoders.BPOSD_Decoder_Class, decoders.ST_BP_Decoder_Class, decoders.FirstMinBPDecoder,
                engine.DeviceBP, engine.DeviceGraph, engine.DeviceFirstMin):
        assert inspect.signature(cls.__init__).parameters["device"].default is None, cls


def test_native_shard_split_equals_shard_range():
    """qldpc_mc_run_sharded's per-device shot blocks (the C ABI's qldpc_shard_range, host-only) are
    parallel.shard_range's: contiguous, covering, sizes within one (bench.py --comm native)."""
    from qldpc_fault_tolerance_amd import _native, parallel

    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libqldpc_hip.so not built")
    for total in (0, 1, 7, 64, 1000, 262_144 * 8 + 5):
        for n in (1, 2, 3, 4, 7, 8):
            blocks = [parallel.native_shard_range(total, n, d) for d in range(n)]
            assert blocks == [parallel.shard_range(total, d, n) for d in range(n)]
            assert sum(c for _, c in blocks) == total
            assert all(blocks[d][0] + blocks[d][1] == blocks[d + 1][0] for d in range(n - 1))
