"""CPU: the oracle replays the reference harness on every BASELINE config code.

Fixtures: tests/golden/reference_harness_configs.npz, made by running the reference's own
CodeSimulator_DataError / CodeSimulator_Phenon_SpaceTime (stub-imported; BP = the oracle) on the
synthesized hgp_34_n1600 stand-in, the reference's LP_Matg8_L30_Dmin20 and GenBicycleA1-A4
matrices (configs 2-4), and the hgp_34_n1225_q3 stand-in's 1764 x 5439 space-time graph
(config 5).  The GPU replays the same fixtures in tests/test_gpu_golden.py.
"""
import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes, simulators
from golden.replay import CONFIG_CODES, CONFIGS, unpack, uniforms


@pytest.fixture(scope="module")
def gold():
    return np.load(CONFIGS, allow_pickle=False)


@pytest.mark.parametrize("name", CONFIG_CODES)
@pytest.mark.parametrize("gtag", ["dep08", "asym"])
def test_generate_error_configs(gold, name, gtag):
    """A5 (src/Simulators.py:89-115) on each config code, CPython's stream regenerated from the seeds."""
    n = codes.get_code(name).N
    ex_ref = unpack(gold[f"{name}_gen_{gtag}_ex"], n)
    u = uniforms(int(gold[f"{name}_gen_{gtag}_seed0"][0]), ex_ref.shape[0], n)
    ex, ez = simulators.pauli_split(u, gold[f"{name}_gen_{gtag}_probs"])
    assert np.array_equal(ex, ex_ref)
    assert np.array_equal(ez, unpack(gold[f"{name}_gen_{gtag}_ez"], n))


@pytest.mark.parametrize("name", CONFIG_CODES)
@pytest.mark.parametrize("pc", [4, 8])
def test_oracle_single_run_configs(gold, oracle, name, pc):
    """A5-A8 on each config code: the oracle's shot loop on the reference's uniforms == its failure flags."""
    code = codes.get_code(name)
    n, p = code.N, pc / 100
    S = gold[f"{name}_run_p{pc}_X_fail"].shape[0]
    u = uniforms(int(gold[f"{name}_run_p{pc}_seed0"][0]), S, n)
    ref = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=0, shot_begin=0, shot_count=S, logical_mode="Total",
                        probs_x=p, probs_z=p, max_iter=int(n / 10), precision=64, uniforms=u, per_shot=True)
    fx, fz = ref["fail"] & 1, ref["fail"] >> 1
    assert np.array_equal(fx, gold[f"{name}_run_p{pc}_X_fail"])
    assert np.array_equal(fz, gold[f"{name}_run_p{pc}_Z_fail"])
    assert np.array_equal(fx | fz, gold[f"{name}_run_p{pc}_Total_fail"])


def test_oracle_phenl_space_time_n1225(gold, oracle):
    """Config 5: detector histories (Z differenced, X raw: Q3), final syndromes and failures of the
    reference's CodeSimulator_Phenon_SpaceTime on the 1764 x 5439 space-time graph."""
    code = codes.get_code("hgp_34_n1225_q3")
    m, n, p = code.hz.shape[0], code.N, 0.01
    S = gold["st1225_fail"].shape[0]
    n_u = (2 * 3 + 1) * (n + code.hx.shape[0] + code.hz.shape[0])
    u = uniforms(int(gold["st1225_seed0"][0]), S, n_u)
    r = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 0, 0, S, 3, 3, "Total", p_data=p, p_synd=p, uniforms=u,
                         per_shot=True)
    body = r["trace"][:, :2 * 2 * 3 * m].reshape(S, 2, 2, 3, m)
    assert np.array_equal(body[:, :, 0].reshape(2 * S, 3, m), unpack(gold["st1225_d1z_hist"], m))
    assert np.array_equal(body[:, :, 1].reshape(2 * S, 3, m), unpack(gold["st1225_d1x_hist"], m))
    assert np.array_equal(r["trace"][:, 12 * m:13 * m], unpack(gold["st1225_d2z_synd"], m))
    assert np.array_equal(r["trace"][:, 13 * m:], unpack(gold["st1225_d2x_synd"], m))
    assert np.array_equal((r["fail"] != 0).astype(np.uint8), gold["st1225_fail"])
