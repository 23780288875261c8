"""GPU replays of the reference-harness fixtures (fp64 = ldpc's arithmetic, bit for bit).

* reference_harness_n225.npz: the reference's _generate_error outputs (gen_*) and _single_run
  failure flags (run_p{3,6}_{X,Z,Total}_fail) replayed directly through DeviceMC on the
  recorded CPython uniforms.
* reference_harness_configs.npz: the same on every BASELINE config code (configs 2-4: the
  hgp_34_n1600 stand-in, LP_Matg8_L30_Dmin20, GenBicycleA1-A4) and config 5's space-time
  detector histories / final syndromes / failures on hgp_34_n1225_q3 (num_rep 3) through
  DevicePhenl in fp64.
Reference: src/Simulators.py:89-168, src/Simulators_SpaceTime.py:444-529.
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes
from golden.replay import CONFIG_CODES, CONFIGS, unpack, uniforms

pytestmark = pytest.mark.gpu
N225 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_harness_n225.npz")


def _mc(code, p, precision=64):
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

    n = code.N
    dx = DeviceBP(code.hz, p * np.ones(n), max_iter=int(n / 10), precision=precision)
    dz = DeviceBP(code.hx, p * np.ones(n), max_iter=int(n / 10), precision=precision,
                  vars_per_thread=dx.geometry()["vars_per_thread"])
    return DeviceMC(code, dx, dz)


@pytest.mark.parametrize("pc", [3, 6])
def test_n225_single_run_flags_replayed_on_gpu(gpu, pc):
    g = np.load(N225, allow_pickle=False)
    code = codes.get_code("hgp_34_n225")
    p = pc / 100
    u = g[f"run_p{pc}_u"]
    res = _mc(code, p).run(p / 2, p / 2, p / 2, seed=0, shot_begin=0, shot_count=u.shape[0], logical_mode="Total",
                           uniforms=u, per_shot=True)
    fx, fz = res.fail & 1, res.fail >> 1
    assert np.array_equal(fx, g[f"run_p{pc}_X_fail"])
    assert np.array_equal(fz, g[f"run_p{pc}_Z_fail"])
    assert np.array_equal(fx | fz, g[f"run_p{pc}_Total_fail"])
    assert res.failures == int(g[f"run_p{pc}_Total_fail"].sum())


@pytest.mark.parametrize("tag", ["dep05", "dep10", "asym"])
def test_n225_generate_error_replayed_on_gpu(gpu, tag):
    g = np.load(N225, allow_pickle=False)
    code = codes.get_code("hgp_34_n225")
    px, py, pz = (float(x) for x in g[f"gen_{tag}_probs"])
    u = g[f"gen_{tag}_u"]
    res = _mc(code, 0.05).run(px, py, pz, seed=0, shot_begin=0, shot_count=u.shape[0], logical_mode="Total",
                              uniforms=u, per_shot=True)
    assert np.array_equal(res.err & 1, g[f"gen_{tag}_ex"])
    assert np.array_equal(res.err >> 1, g[f"gen_{tag}_ez"])


@pytest.mark.parametrize("name", CONFIG_CODES)
def test_config_harness_replayed_on_gpu(gpu, name):
    g = np.load(CONFIGS, allow_pickle=False)
    code = codes.get_code(name)
    n = code.N
    for gtag in ("dep08", "asym"):
        ex_ref = unpack(g[f"{name}_gen_{gtag}_ex"], n)
        u = uniforms(int(g[f"{name}_gen_{gtag}_seed0"][0]), ex_ref.shape[0], n)
        px, py, pz = (float(x) for x in g[f"{name}_gen_{gtag}_probs"])
        res = _mc(code, 0.05).run(px, py, pz, 0, 0, u.shape[0], "Total", uniforms=u, per_shot=True)
        assert np.array_equal(res.err & 1, ex_ref), gtag
        assert np.array_equal(res.err >> 1, unpack(g[f"{name}_gen_{gtag}_ez"], n)), gtag
    for pc in (4, 8):
        p = pc / 100
        S = g[f"{name}_run_p{pc}_X_fail"].shape[0]
        u = uniforms(int(g[f"{name}_run_p{pc}_seed0"][0]), S, n)
        res = _mc(code, p).run(p / 2, p / 2, p / 2, 0, 0, S, "Total", uniforms=u, per_shot=True)
        fx, fz = res.fail & 1, res.fail >> 1
        assert np.array_equal(fx, g[f"{name}_run_p{pc}_X_fail"]), pc
        assert np.array_equal(fz, g[f"{name}_run_p{pc}_Z_fail"]), pc
        assert np.array_equal(fx | fz, g[f"{name}_run_p{pc}_Total_fail"]), pc


@pytest.mark.parametrize("family", ["one_word", "two_word", "hbm"])
def test_config5_space_time_replayed_on_gpu_fp64(gpu, monkeypatch, family):
    """Config 5 in ldpc's float64 arithmetic: the 1764 x 5439 space-time decoder at the drop-in's default
    precision — engine 3's tail layout (rows of 9 = 4 fp64 chunks + a tail slot, 1024 threads x 6
    variables, the first slot's 1024 degree-2 measurement variables on 2 edge slots) in the one-word
    "m2 in slot" family (round 6, engine id 111313, the default) and the two-word family (engine id
    101013, QLDPC_M2ST=0), and the same histories forced onto the HBM-resident message engine (engine 6)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DevicePhenl

    if family == "two_word":
        monkeypatch.setenv("QLDPC_M2ST", "0")
    g = np.load(CONFIGS, allow_pickle=False)
    code = codes.get_code("hgp_34_n1225_q3")
    m, n, p = code.hz.shape[0], code.N, 0.01
    mi = int(n / 10)
    S = g["st1225_fail"].shape[0]
    for hbm in ((True,) if family == "hbm" else (False,)):
        st = [DeviceBP(codes.space_time_csr(h, 3), np.hstack([p * np.ones(n), p * np.ones(m)] * 3), max_iter=mi,
                       precision=64, hbm=hbm) for h in (code.hz, code.hx)]
        geo = st[0].geometry()
        assert geo["engine"] == (6 if hbm else 3), geo
        if not hbm:
            assert geo["lds_bytes"] > 64 * 1024 and geo["threads"] == 1024, geo  # the tail-layout family
            assert geo["kernel_id"] == (111313 if family == "one_word" else 101013), geo
        d2 = [DeviceBP(code.csr(k), p * np.ones(n), max_iter=mi, precision=64) for k in ("hz", "hx")]
        ph = DevicePhenl(code, st[0], st[1], d2[0], d2[1], num_rep=3)
        u = uniforms(int(g["st1225_seed0"][0]), S, ph.uniforms_per_sample(3))
        res = ph.run(p / 2, p / 2, p / 2, p, 0, 0, S, 3, "Total", uniforms=u, per_shot=True)
        tr = res.trace
        body = tr[:, :2 * 2 * 3 * m].reshape(S, 2, 2, 3, m)
        assert np.array_equal(body[:, :, 0].reshape(2 * S, 3, m), unpack(g["st1225_d1z_hist"], m)), hbm
        assert np.array_equal(body[:, :, 1].reshape(2 * S, 3, m), unpack(g["st1225_d1x_hist"], m)), hbm
        assert np.array_equal(tr[:, 12 * m:13 * m], unpack(g["st1225_d2z_synd"], m)), hbm
        assert np.array_equal(tr[:, 13 * m:], unpack(g["st1225_d2x_synd"], m)), hbm
        assert np.array_equal((res.fail != 0).astype(np.uint8), g["st1225_fail"]), hbm
