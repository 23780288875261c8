"""The multi-GPU half of the C ABI and the standalone sampler.

* qldpc_sample_errors == the reference's _generate_error on the recorded CPython uniforms
  (reference_harness_n225.npz, src/Simulators.py:89-115) and == the d_err output of the fused
  launch on the Philox stream.
* qldpc_mc_run_sharded: shots split over several MC handles (contiguous global blocks, the
  split of parallel.shard_range) give counters identical to one handle running every shot —
  summed on the host, and through an RCCL communicator of qldpc_comm_init_all.
* qldpc_comm_init_rank / qldpc_comm_allreduce_counters on a one-rank communicator.
(One GPU on the test box: RCCL refuses two ranks on one device, so the N>1 collective itself is
covered by the gloo tests of test_distributed_cpu.py and the driver's multi-GPU bench.)
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes

pytestmark = pytest.mark.gpu
N225 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_harness_n225.npz")


def _mc(code, p, precision=64):
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

    n = code.N
    dx = DeviceBP(code.hz, p * np.ones(n), max_iter=int(n / 10), precision=precision, device=0)
    dz = DeviceBP(code.hx, p * np.ones(n), max_iter=int(n / 10), precision=precision, device=0,
                  vars_per_thread=dx.geometry()["vars_per_thread"])
    return DeviceMC(code, dx, dz)


@pytest.mark.parametrize("tag", ["dep05", "dep10", "asym"])
def test_sample_errors_replays_generate_error(gpu, tag):
    from qldpc_fault_tolerance_amd.engine import sample_errors

    g = np.load(N225, allow_pickle=False)
    px, py, pz = (float(x) for x in g[f"gen_{tag}_probs"])
    u = g[f"gen_{tag}_u"]
    e = sample_errors(225, px, py, pz, 0, 0, u.shape[0], uniforms=u, device=0).cpu().numpy()
    assert np.array_equal(e & 1, g[f"gen_{tag}_ex"])
    assert np.array_equal(e >> 1, g[f"gen_{tag}_ez"])


def test_sample_errors_matches_fused_launch(gpu):
    from qldpc_fault_tolerance_amd.engine import sample_errors

    code = codes.get_code("hgp_34_n1600")
    p, S, seed, s0 = 0.06, 512, 0x51D5EED2, 123_456_789
    res = _mc(code, p).run(p / 2, p / 2, p / 2, seed, s0, S, "Total", per_shot=True)
    e = sample_errors(code.N, p / 2, p / 2, p / 2, seed, s0, S, device=0).cpu().numpy()
    assert np.array_equal(e, res.err)
    # the class frequencies of the 3-way split (z, x, y each p/2 = 0.03)
    assert abs((e == 1).mean() - 0.03) < 0.004 and abs((e == 2).mean() - 0.03) < 0.004


def test_mc_run_sharded_equals_one_handle(gpu):
    from qldpc_fault_tolerance_amd.engine import run_sharded

    code = codes.get_code("hgp_34_n225")
    p, S, seed = 0.06, 20_003, 77
    one = _mc(code, p).run(p / 2, p / 2, p / 2, seed, 1000, S, "Total")
    mcs = [_mc(code, p) for _ in range(3)]
    split = run_sharded(mcs, None, p / 2, p / 2, p / 2, seed, 1000, S, "Total")
    assert split.shots == S == one.shots
    assert (split.failures, split.sector_iters, split.sector_nonconv) == (one.failures, one.sector_iters,
                                                                          one.sector_nonconv)
    assert np.array_equal(split.iter_hist, one.iter_hist)


def test_native_comm_one_rank(gpu):
    import torch

    from qldpc_fault_tolerance_amd.engine import run_sharded
    from qldpc_fault_tolerance_amd.parallel import NativeComm

    uid = NativeComm.unique_id()
    assert len(uid) == 128
    c = NativeComm(0, 1, 0, uid)
    assert c.info() == {"rank": 0, "nranks": 1, "device": 0}
    w = torch.arange(gpu.COUNTER_WORDS, dtype=torch.int64, device="cuda:0")
    ref = w.clone()
    c.allreduce_counters(w)
    torch.cuda.synchronize()
    assert torch.equal(w, ref)  # a one-rank sum is the identity
    c.close()
    comms = NativeComm.init_all([0])
    code = codes.get_code("hgp_34_n225")
    p, S = 0.05, 8192
    one = _mc(code, p).run(p / 2, p / 2, p / 2, 5, 0, S, "Total")
    via = run_sharded([_mc(code, p)], comms, p / 2, p / 2, p / 2, 5, 0, S, "Total")
    assert (via.shots, via.failures, via.sector_iters) == (one.shots, one.failures, one.sector_iters)
    for x in comms:
        x.close()
