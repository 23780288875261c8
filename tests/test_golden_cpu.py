"""CPU tests: the oracle and the host logic against the reference's own harness.

``tests/golden/reference_harness_n225.npz`` was produced by running the
reference's ``Simulators.py`` / ``Decoders*.py`` (stub-imported, BP backed by
this repository's oracle: tests/golden/make_golden.py).  Everything except the
BP arithmetic is therefore the reference's behaviour; BP parity is pinned by the
oracle's known-answer tests below (the reference has no BP fixtures: DESIGN.md
§Oracle, "parity of the BP arithmetic unpinned by the reference").
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes, decoders, simulators

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_harness_n225.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


@pytest.fixture(scope="module")
def n225():
    return codes.get_code("hgp_34_n225")


@pytest.mark.parametrize("tag", ["dep05", "dep10", "asym"])
def test_pauli_split_matches_reference_generate_error(gold, tag):
    """A5: src/Simulators.py:89-115 on identical uniforms."""
    u = gold[f"gen_{tag}_u"]
    ex, ez = simulators.pauli_split(u, gold[f"gen_{tag}_probs"])
    assert np.array_equal(ex, gold[f"gen_{tag}_ex"])
    assert np.array_equal(ez, gold[f"gen_{tag}_ez"])


@pytest.mark.parametrize("pc", [3, 6])
def test_bp_factory_matches_reference(gold, n225, pc):
    """A2: BP_Decoder_Class.GetDecoder arguments (max_iter = n/ratio as float, quirk Q1)."""
    cls = decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    n, probs = cls._probs({"h": n225.hz, "p_data": pc / 100})
    assert n / 10 == gold[f"factory_p{pc}_max_iter_arg"][0]
    assert np.array_equal(probs, gold[f"factory_p{pc}_probs"][0])
    assert decoders._int_max_iter(n / 10, n) == 22


def test_factory_asserts_like_reference():
    cls = decoders.BP_Decoder_Class(10, "minimum_sum", 0.625)
    with pytest.raises(AssertionError):
        cls.GetDecoder({"p_data": 0.1})
    with pytest.raises(AssertionError):
        cls.GetDecoder({"h": np.eye(3)})
    st = decoders.ST_BP_Decoder_Class(10, "minimum_sum", 0.625)
    with pytest.raises(AssertionError):
        st.GetDecoder({"h": np.eye(3), "p_data": 0.1})


@pytest.mark.parametrize("pc", [3, 6])
@pytest.mark.parametrize("mode", ["X", "Z", "Total"])
def test_oracle_mc_replays_reference_single_run(gold, n225, oracle, pc, mode):
    """A5-A7: the fused shot loop on the reference's uniforms gives its failure flags."""
    p = pc / 100
    u = gold[f"run_p{pc}_u"]
    ref = oracle.mc_run(n225, p / 2, p / 2, p / 2, seed=0, shot_begin=0, shot_count=u.shape[0], logical_mode=mode,
                        probs_x=p, probs_z=p, max_iter=22, precision=64, uniforms=u, per_shot=True)
    fx, fz = ref["fail"] & 1, ref["fail"] >> 1
    want = gold[f"run_p{pc}_{mode}_fail"]
    got = fx if mode == "X" else fz if mode == "Z" else (fx | fz)
    assert np.array_equal(got, want)
    assert ref["failures"] == int(want.sum())


def test_wer_formula_matches_reference(gold):
    """A8: WordErrorRate arithmetic incl. quirk Q2."""
    for num_run, nfail, wer, eb in gold["wer_cases"]:
        w, e = simulators.word_error_rate(int(nfail), int(num_run), 17)
        assert w == wer
        assert (e == eb) or (np.isnan(e) and np.isnan(eb))


def test_spacetime_wer_formula_matches_reference(gold):
    """A13: per-cycle WER of CodeSimulator_Phenon_SpaceTime.WordErrorRate (Simulators_SpaceTime.py:531-548)."""
    for num_cycles, num_samples, nfail, w in gold["phenst_wer_cases"]:
        num_rounds = int((num_cycles - 1) / 3 + 1)
        total = (num_rounds - 1) * 3 + 1
        assert simulators.word_error_rate_per_cycle(int(nfail), int(num_samples), 17, total) == w


def test_oracle_phenl_replays_reference_harness(gold, n225, oracle):
    """A13: the oracle's CodeSimulator_Phenon_SpaceTime restatement, fed CPython's recorded uniforms, reproduces
    the reference harness's detector histories (Z differenced, X raw: quirk Q3), final syndromes and failures."""
    p = 0.02
    r = oracle.phenl_run(n225, p / 2, p / 2, p / 2, p, 0, 0, 12, 3, 3, "Total", p_data=p, p_synd=p,
                         uniforms=gold["phenst_u"], per_shot=True)
    tr, m = r["trace"], n225.hz.shape[0]
    body = tr[:, :2 * 2 * 3 * m].reshape(12, 2, 2, 3, m)
    assert np.array_equal(body[:, :, 0].reshape(24, 3, m), gold["phenst_d1z_hist"])
    assert np.array_equal(body[:, :, 1].reshape(24, 3, m), gold["phenst_d1x_hist"])
    assert np.array_equal(tr[:, 12 * m:13 * m], gold["phenst_d2z_synd"])
    assert np.array_equal(tr[:, 13 * m:], gold["phenst_d2x_synd"])
    assert np.array_equal((r["fail"] != 0).astype(np.uint8), gold["phenst_fail"])


def test_phenl_simulator_plugin_path_matches_oracle(gold, n225, oracle):
    """The drop-in CodeSimulator_Phenon_SpaceTime._single_run (per-sample plugin path, CPython random) with
    oracle-backed decoders draws and decides exactly like the reference harness."""
    import random

    p = 0.02

    class OracleST:
        def __init__(self, h):
            self.h, self.csr = h, codes.space_time_csr(h, 3)
            mh, nh = h.shape
            self.probs = np.hstack([p * np.ones(nh), p * np.ones(mh)] * 3)

        def decode(self, det):
            e, _, _ = oracle.bp_decode_batch(self.csr, self.probs, 22, synd=np.asarray(det).reshape(1, -1))
            return decoders.fold_space_time_correction(e[0], self.h.shape[1], self.h.shape[0], 3)

    class OracleBP:
        def __init__(self, h):
            self.h = h

        def decode(self, s):
            return oracle.bp_decode_batch(self.h, p, 22, synd=np.asarray(s).reshape(1, -1))[0][0].astype(int)

    sim = simulators.CodeSimulator_Phenon_SpaceTime(
        code=n225, decoder1_x=OracleST(n225.hz), decoder1_z=OracleST(n225.hx), decoder2_x=OracleBP(n225.hz),
        decoder2_z=OracleBP(n225.hx), pauli_error_probs=[p / 2] * 3, q=p, eval_logical_type="Total", num_rep=3)
    flags = []
    for s in range(12):
        random.seed(9000 + s)
        flags.append(int(sim._single_run(3)))
    assert flags == gold["phenst_fail"].tolist()


@pytest.mark.parametrize("t0", [1, 2, 3])
def test_space_time_matrix_matches_reference(gold, n225, t0):
    """A10: GetSpaceTimeCheckMat (Decoders_SpaceTime.py:179-194)."""
    c = codes.space_time_csr(n225.hx, t0)
    assert [c.m, c.n] == list(gold[f"st_t{t0}_shape"])
    assert np.array_equal(c.row_ptr, gold[f"st_t{t0}_row_ptr"])
    assert np.array_equal(c.col_idx, gold[f"st_t{t0}_col_idx"])
    assert np.array_equal(decoders.GetSpaceTimeCheckMat(n225.hx, t0), c.to_dense().astype(float))


def test_space_time_decoder_matches_reference(gold, n225, oracle):
    """A11/A12: ST_BP_Decoder_Class factory priors/max_iter and the decode+fold of ST_BP_Decoder_syndrome."""
    assert gold["stfactory_max_iter_arg"][0] == n225.N / 10
    probs = np.hstack([0.02 * np.ones(n225.N), 0.02 * np.ones(n225.hz.shape[0])] * 3)
    assert np.array_equal(probs, gold["stfactory_probs"])
    st = codes.space_time_csr(n225.hz, 3)
    hist = gold["stdec_hist"]
    synd = hist.reshape(hist.shape[0], -1)
    corr, _, _ = oracle.bp_decode_batch(st, probs, 22, "minimum_sum", 0.625, synd, 64)
    folded = decoders.fold_space_time_correction(corr, n225.N, n225.hz.shape[0], 3)
    assert np.array_equal(folded, gold["stdec_corr"])


# ----------------------------------------------------------- oracle KATs


def test_oracle_zero_syndrome_is_zero_correction(n225, oracle):
    s = np.zeros((3, n225.hz.shape[0]), np.uint8)
    corr, iters, conv = oracle.bp_decode_batch(n225.hz, 0.05, 22, "minimum_sum", 0.625, s, 64)
    assert not corr.any() and (iters == 1).all() and conv.all()


@pytest.mark.parametrize("precision", [64, 32])
def test_oracle_corrects_every_weight_one_error(n225, oracle, precision):
    H = n225.hz
    E = np.eye(n225.N, dtype=np.uint8)
    S = (E.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)
    corr, iters, conv = oracle.bp_decode_batch(H, 0.05, 22, "minimum_sum", 0.625, S, precision)
    assert conv.all()
    # the decoding reproduces the syndrome (the residual is a stabiliser or zero)
    assert np.array_equal(codes.CSR.from_dense(H).matvec(corr), S)


def test_oracle_is_deterministic_and_threaded_identically(n225, oracle):
    rng = np.random.default_rng(5)
    e = (rng.random((64, n225.N)) < 0.06).astype(np.uint8)
    S = codes.CSR.from_dense(n225.hx).matvec(e).astype(np.uint8)
    a = oracle.bp_decode_batch(n225.hx, 0.06, 22, "minimum_sum", 0.625, S, 64, nthreads=1)
    b = oracle.bp_decode_batch(n225.hx, 0.06, 22, "minimum_sum", 0.625, S, 64, nthreads=4)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_oracle_philox_known_answer(oracle):
    """Philox4x32-10 published KAT (Salmon et al., SC'11 / Random123 kat_vectors)."""
    assert oracle.philox4x32_10([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                       0x6D5451FD]
    assert oracle.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                                [0xA4093822, 0x299F31D0]) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_oracle_mc_shard_invariance(n225, oracle):
    """Counters over a shot range do not depend on how the range is split (multi-GPU invariant)."""
    kw = dict(logical_mode="Total", probs_x=0.05, probs_z=0.05, max_iter=22, precision=32)
    whole = oracle.mc_run(n225, 0.025, 0.025, 0.025, seed=3, shot_begin=100, shot_count=600, **kw)
    parts = [oracle.mc_run(n225, 0.025, 0.025, 0.025, seed=3, shot_begin=b, shot_count=c, **kw)
             for b, c in [(100, 250), (350, 350)]]
    for key in ("shots", "failures", "sector_iters", "sector_nonconv", "sector_fail"):
        tot = parts[0][key]
        tot = tot + parts[1][key] if not isinstance(tot, list) else [x + y for x, y in zip(tot, parts[1][key])]
        assert tot == whole[key], key


# ---------------------------------------------------------------- single-shot phenomenological (§8f rank 1)
@pytest.fixture(scope="module")
def phen_gold():
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_harness_phen_n225.npz"))


def test_oracle_phen_single_shot_replays_reference(phen_gold, n225, oracle):
    """CodeSimulator_Phenon (src/Simulators.py:189-327) = the space-time loop at num_rep = 1: the oracle's
    restatement fed CPython's recorded uniforms reproduces the reference's decoder inputs and failures."""
    p, m = 0.02, n225.hz.shape[0]
    r = oracle.phenl_run(n225, p / 2, p / 2, p / 2, p, 0, 0, 16, 3, 1, "Total", p_data=p, p_synd=p,
                         uniforms=phen_gold["phen_u"], per_shot=True)
    body = r["trace"][:, :2 * 2 * m].reshape(16, 2, 2, m)
    assert np.array_equal(body[:, :, 0].reshape(32, m), phen_gold["phen_d1z_synd"])
    assert np.array_equal(body[:, :, 1].reshape(32, m), phen_gold["phen_d1x_synd"])
    assert np.array_equal(r["trace"][:, 4 * m:5 * m], phen_gold["phen_d2z_synd"])
    assert np.array_equal(r["trace"][:, 5 * m:], phen_gold["phen_d2x_synd"])
    assert np.array_equal((r["fail"] != 0).astype(np.uint8), phen_gold["phen_fail"])


def test_phen_single_shot_plugin_path(phen_gold, n225, oracle):
    """The drop-in CodeSimulator_Phenon._single_run (CPython random, oracle-backed BP decoders) == reference."""
    import random

    p = 0.02

    class OracleBP:
        def __init__(self, h, probs):
            self.h, self.probs = h, probs

        def decode(self, s):
            return oracle.bp_decode_batch(self.h, self.probs, 22, synd=np.asarray(s).reshape(1, -1))[0][0].astype(int)

    mx, mz, n = n225.hx.shape[0], n225.hz.shape[0], n225.N
    ext = lambda h: np.hstack([h, np.identity(h.shape[0])])  # noqa: E731
    sim = simulators.CodeSimulator_Phenon(
        code=n225, decoder1_x=OracleBP(ext(n225.hz), np.hstack([p * np.ones(n), p * np.ones(mz)])),
        decoder1_z=OracleBP(ext(n225.hx), np.hstack([p * np.ones(n), p * np.ones(mx)])),
        decoder2_x=OracleBP(n225.hz, p), decoder2_z=OracleBP(n225.hx, p), pauli_error_probs=[p / 2] * 3, q=p)
    flags = []
    for s in range(16):
        random.seed(7000 + s)
        flags.append(int(sim._single_run(3)))
    assert flags == phen_gold["phen_fail"].tolist()
    # BP_Decoder_Class with p_syndrome: max_iter = (n_ext - m)/ratio = n/ratio (src/Decoders.py:154-162)
    assert list(phen_gold["phen_factory_max_iter_arg"]) == [n / 10, n / 10]


def test_phen_wer_formulas_match_reference(phen_gold):
    """WordErrorRate (:329-358) and WordErrorProbability (:360-381) of CodeSimulator_Phenon."""
    for num_rounds, num_samples, nfail, which, w, eb in phen_gold["phen_wer_cases"]:
        if int(which) == 0:
            assert simulators.word_error_rate_phenl(int(nfail), int(num_samples), 17, int(num_rounds)) == w
        else:
            w2, eb2 = simulators.word_error_rate(int(nfail), int(num_samples), 17)
            assert w2 == w and ((eb2 == eb) or (np.isnan(eb2) and np.isnan(eb)))
