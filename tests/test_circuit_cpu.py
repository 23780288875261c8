"""Circuit-level space-time path on the CPU (qldpc_fault_tolerance_amd/circuit.py).

* CX schedules == the reference's own ``CircuitScheduling`` (golden fixture made by importing it).
* Detector error models: hand-derived DEMs of small repetition-code circuits, and the product's
  backward sensitivity analysis == the oracle's forward one-fault-at-a-time propagation
  (``oracle/circuit_oracle.py``) on the reference's syndrome circuits.
* The fault hypergraphs of the demo configuration (``SpaceTimeDecodingDemo.ipynb`` cell 2).
Against stim itself the DEM is parity unpinned (absent package); see circuit.py.
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import circuit as C
from qldpc_fault_tolerance_amd import codes

HERE = os.path.dirname(os.path.abspath(__file__))


def _ring(d):
    h = np.zeros((d, d), np.uint8)
    for i in range(d):
        h[i, i] = h[i, (i + 1) % d] = 1
    return h


def _cases():
    tor = codes.hgp(_ring(3), _ring(3))
    sur = codes.hgp(_ring(3)[:-1, :], _ring(3)[:-1, :])
    n225 = codes.get_code("hgp_34_n225")
    gbc = codes.get_code("GenBicycleA1")
    return [("toric3_hx", tor.hx), ("toric3_hz", tor.hz), ("surface3_hx", sur.hx), ("surface3_hz", sur.hz),
            ("n225_hx", n225.hx), ("n225_hz", n225.hz), ("gbcA1_hx", gbc.hx)]


@pytest.mark.parametrize("kind", ["color", "random"])
def test_schedules_match_reference(kind):
    z = np.load(os.path.join(HERE, "golden", "reference_circuit_schedules.npz"))
    for name, H in _cases():
        sched = (C.ColorationCircuit if kind == "color" else C.RandomCircuit)(H)
        keys, vals, offs = (z[f"{name}_{kind}_{k}"] for k in ("keys", "vals", "offs"))
        assert len(sched) == len(offs) - 1, name
        for t, step in enumerate(sched):
            assert list(step.keys()) == list(keys[offs[t]:offs[t + 1]]), (name, t)
            assert list(step.values()) == list(vals[offs[t]:offs[t + 1]]), (name, t)


def _rep_circuit():
    """d = 3 repetition code, checks Z0Z1 (ancilla 3) and Z1Z2 (ancilla 4), one round, then the data
    measured with observable Z0."""
    c = C.StimCircuit()
    c.append("R", [0, 1, 2, 3, 4])
    return c


def test_hand_derived_repetition_dems():
    c = _rep_circuit()
    c.append("X_ERROR", [0], 0.1)
    c.append("X_ERROR", [1], 0.2)
    c.append("DEPOLARIZE1", [2], 0.03)
    c.append("CX", [0, 3, 1, 3, 1, 4, 2, 4])
    c.append("MR", [3, 4])
    c.append("DETECTOR", [-2])
    c.append("DETECTOR", [-1])
    c.append("M", [0, 1, 2])
    c.append("OBSERVABLE_INCLUDE", [-3], 0)
    got = {(d, k): p for p, d, k in zip(*(lambda m: (m.probs, m.dets, m.obs))(c.detector_error_model()))}
    q = C.depolarize1_component(0.03)
    # X on q0 flips check 0 and the observable; X on q1 flips both checks; X or Y on q2 flips check 1
    # (Z on q2 is invisible): X and Y merge into 2q(1-q) = 2p/3 exactly
    assert set(got) == {((0,), (0,)), ((0, 1), ()), ((1,), ())}
    assert got[((0,), (0,))] == 0.1 and got[((0, 1), ())] == 0.2
    assert abs(got[((1,), ())] - 2 * 0.03 / 3) < 1e-15 and abs(got[((1,), ())] - 2 * q * (1 - q)) < 1e-15


def test_hand_derived_measurement_and_reset_errors():
    """Errors after MR reset are invisible to it; a Z error before an X-basis measurement flips it;
    a second round's difference detector sees a data error once."""
    c = C.StimCircuit()
    c.append("RX", [0])
    c.append("R", [1])
    c.append("Z_ERROR", [0], 0.05)          # flips the MX of q0 -> D1 and the observable
    c.append("CX", [0, 1])
    c.append("MR", [1])
    c.append("X_ERROR", [1], 0.3)           # after MR: reset by the next MR's measurement? no: it flips it
    c.append("DETECTOR", [-1])
    c.append("MR", [1])
    c.append("DETECTOR", [-1, -2])
    c.append("MX", [0])
    c.append("DETECTOR", [-1])
    c.append("OBSERVABLE_INCLUDE", [-1], 0)
    dem = c.detector_error_model()
    got = {(d, k): p for p, d, k in zip(dem.probs, dem.dets, dem.obs)}
    # q0 in |+>, CX(0 -> 1) with q1 in |0>: Z on q0 commutes through the control -> MX flips (D2, L0);
    # X_ERROR on q1 after the first MR flips the second MR -> D1 (difference of the two MRs)
    assert got == {((2,), (0,)): 0.05, ((1,), ()): 0.3}


@pytest.fixture(scope="module")
def demo():
    tor = codes.hgp(_ring(3), _ring(3))
    ep = {"p_i": 0.0, "p_state_p": 0.0, "p_m": 0.0, "p_CX": 1e-3, "p_idling_gate": 0.0}
    sx, sz = C.ColorationCircuit(tor.hx), C.ColorationCircuit(tor.hz)
    full, fault = C.syndrome_circuits(tor.hx, tor.hz, tor.lx, ep, 1e-3, 4, 3, sx, sz)
    return tor, full, fault


def test_demo_circuit_shape(demo):
    tor, full, fault = demo
    m = tor.hx.shape[0]
    # num_cycles = 13 = num_rounds * num_rep + 1 syndrome layers of m detectors
    assert full.num_detectors == 13 * m and fault.num_detectors == 4 * m
    assert full.num_observables == fault.num_observables == tor.lx.shape[0]
    # every CX instruction is followed by its DEPOLARIZE2 (AddCXError)
    for a, b in zip(full.ops, full.ops[1:]):
        if a.name == "CX":
            assert b.name == "DEPOLARIZE2" and b.targets == a.targets and b.arg == 1e-3


@pytest.mark.parametrize("which", ["fault", "full2"])
def test_dem_backward_equals_forward_oracle(which):
    import circuit_oracle

    tor = codes.hgp(_ring(3), _ring(3))
    # every noise source switched on, distinct rates, so no two locations share a probability by accident
    ep = {"p_i": 2e-3, "p_state_p": 3e-3, "p_m": 4e-3, "p_CX": 5e-3, "p_idling_gate": 1e-3}
    sx, sz = C.ColorationCircuit(tor.hx), C.RandomCircuit(tor.hz)
    full, fault = C.syndrome_circuits(tor.hx, tor.hz, tor.lx, ep, 6e-3, 2, 2, sx, sz)
    circ = fault if which == "fault" else full
    want = circuit_oracle.dem_forward(circ)
    got = circuit_oracle.dem_as_map(circ.detector_error_model())
    assert set(got) == set(want)
    for k in want:
        assert abs(got[k] - want[k]) <= 1e-15 + 1e-12 * want[k], k


def test_fault_hypergraphs_of_the_demo(demo):
    tor, _, fault = demo
    m, K = tor.hx.shape[0], tor.lx.shape[0]
    dem = fault.detector_error_model()
    H, L, P = C.GenFaultHyperGraph(dem, 4, 3, K)
    h1, h2 = H
    assert h1.shape[0] == 3 * m and h2.shape[0] == m
    assert L[0].shape == (K, h1.shape[1]) and L[1].shape == (K, h2.shape[1])
    assert len(P[0]) == h1.shape[1] and len(P[1]) == h2.shape[1]
    assert (h1.sum(axis=0) > 0).all() and (h2.sum(axis=0) > 0).all()
    assert all(0 < p < 0.01 for p in P[0] + P[1])
    Hs = C.GenCorrecHyperGraph(dem, 4, 3, m, K)
    assert Hs.shape == (m, h1.shape[1]) and set(np.unique(Hs)) <= {0.0, 1.0}
    # the space correction of a layer-0 error = its syndrome change summed over the repetitions and
    # the final layer: a data error in the first repetition flips its checks once (its first
    # repetition), so its column equals hx's column for that qubit when it touches no other layer
    full_cols = {tuple(np.flatnonzero(tor.hx[:, q])) for q in range(tor.N)}
    assert any(tuple(np.flatnonzero(Hs[:, j])) in full_cols for j in range(Hs.shape[1]))


def test_dem_text_lists_errors_then_detectors(demo):
    _, _, fault = demo
    txt = str(fault.detector_error_model()).split("\n")
    nerr = sum(1 for t in txt if t.startswith("error("))
    assert all(t.startswith("error(") for t in txt[:nerr])
    assert txt[nerr] == "shift_detectors(1) 0" and txt.count("shift_detectors(1) 0") == 2


# ---------------------------------------------------------------- reference-generated fixtures
# tests/golden/reference_circuit.npz (make_golden.py circuit): the reference's own
# CodeSimulator_Circuit_SpaceTime._generate_circuit / AddCXError run through a recording stim.Circuit
# stand-in (op lists), and its own _generate_circuit_graph / GenFaultHyperGraph / GenCorrecHyperGraph
# run on this engine's DEM of the recorded fault circuit, rendered as DEM text (exact and stim style).
REF_CIRCUIT = os.path.join(HERE, "golden", "reference_circuit.npz")
CIRCUIT_TAGS = ["demo", "all3c", "all3r", "mixed", "low"]


def _ref_sim(z, tag, compat=False):
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_Circuit_SpaceTime

    p, pi, ps, pm, pcx, pid, ncyc, nrep, rnd = z[f"{tag}_params"]
    ep = {"p_i": pi, "p_state_p": ps, "p_m": pm, "p_CX": pcx, "p_idling_gate": pid}
    code = codes.hgp(_ring(3), _ring(3))
    return CodeSimulator_Circuit_SpaceTime(code=code, p=float(p), num_cycles=int(ncyc), num_rep=int(nrep),
                                           error_params=ep, eval_logical_type="Z",
                                           circuit_type="random" if rnd else "coloration", compat_dem_text=compat)


@pytest.mark.parametrize("tag", CIRCUIT_TAGS)
def test_circuit_op_lists_match_reference(tag):
    """Every instruction of the full and the one-round fault circuit (gate, argument, targets, in
    order) == what the reference's _generate_circuit + AddCXError produced (src/Simulators_SpaceTime.py
    :737-940, src/ErrorPlugin.py:11-25)."""
    z = np.load(REF_CIRCUIT)
    sim = _ref_sim(z, tag)
    sim._generate_circuit()
    for which, circ in (("circuit", sim.circuit), ("fault", sim.fault_circuit)):
        names, args = z[f"{tag}_{which}_names"], z[f"{tag}_{which}_args"]
        offs, tg = z[f"{tag}_{which}_offs"], z[f"{tag}_{which}_targets"]
        assert len(circ.ops) == len(names), (which, len(circ.ops), len(names))
        for i, o in enumerate(circ.ops):
            assert o.name == names[i], (which, i, o.name, names[i])
            a = np.nan if o.arg is None else o.arg
            assert (np.isnan(a) and np.isnan(args[i])) or a == args[i], (which, i, o.name, a, args[i])
            assert list(o.targets) == list(tg[offs[i]:offs[i + 1]]), (which, i, o.name)


@pytest.mark.parametrize("style", ["exact", "stim"])
@pytest.mark.parametrize("tag", CIRCUIT_TAGS)
def test_fault_hypergraphs_match_reference(tag, style):
    """h1 / L1 / channel_ps1 / h2 / L2 / channel_ps2 / h1_space_cor == the reference's
    _generate_circuit_graph (:943-967) on the same DEM text: ``exact`` = the drop-in default (exact
    probabilities), ``stim`` = ``compat_dem_text=True`` (stim's mechanism order, 6-digit %g text and the
    reference's ``\\d+\\.\\d+`` parse, mantissa-only for exponent notation)."""
    z = np.load(REF_CIRCUIT)
    sim = _ref_sim(z, tag, compat=(style == "stim"))
    sim._generate_circuit()
    sim._generate_circuit_graph()
    g = sim.circuit_graph
    for k in ("h1", "L1", "h2", "L2"):
        want = z[f"{tag}_{style}_{k}"]
        assert np.asarray(g[k]).shape == want.shape and np.array_equal(np.asarray(g[k]).astype(np.uint8), want), k
    import re

    for k in ("channel_ps1", "channel_ps2"):
        got, want = np.asarray(g[k], dtype=np.float64), z[f"{tag}_{style}_{k}"]
        if style == "exact":
            # the drop-in default keeps exact probabilities; where the reference's regex met a repr in
            # exponent notation (p < 1e-4) it read the mantissa: that is the documented deviation
            bad = np.array(["e" in repr(float(x)) for x in got], dtype=bool)
            assert np.array_equal(got[~bad], want[~bad]), k
            assert all(float(re.findall(r"\d+\.\d+", repr(float(x)))[0]) == y for x, y in zip(got[bad], want[bad])), k
            assert bad.any() == (tag == "low"), (tag, int(bad.sum()))
        else:
            assert np.array_equal(got, want), k
    assert np.array_equal(np.asarray(sim.h1_space_cor).astype(np.uint8), z[f"{tag}_{style}_h1_space_cor"])


def test_compat_parse_reads_mantissas_of_exponent_notation():
    """At p = 5e-5 (every source) stim prints some mechanisms below 1e-4 in exponent notation; the
    reference's regex keeps their mantissa (e.g. 5.99982e-05 -> 5.99982).  The reference's fixtures hold
    exactly those values, the exact (default) path keeps the true probabilities."""
    z = np.load(REF_CIRCUIT)
    sim = _ref_sim(z, "low")
    sim._generate_circuit()
    sim._generate_circuit_graph()
    bad = C.misparsed_mechanisms(sim.fault_dem)
    assert bad, "the low-rate case should contain exponent-notation mechanisms"
    comp = np.concatenate([z["low_stim_channel_ps1"], z["low_stim_channel_ps2"]])
    assert (comp > 1).any() and (np.concatenate([sim.circuit_graph["channel_ps1"], sim.circuit_graph["channel_ps2"]])
                                 < 1e-2).all()
    for tag in ("demo", "all3c", "all3r", "mixed"):  # the GPU tests' rates: nothing mis-parsed
        s = _ref_sim(z, tag)
        s._generate_circuit()
        s._generate_circuit_graph()
        assert not C.misparsed_mechanisms(s.fault_dem), tag


def test_skip_sampler_oracle_is_batch_invariant_and_exact():
    """oracle/circuit_oracle.py's restatement of the geometric-skip DEM sampler (the device default):
    keyed by global 64-sample words, so any split of the shot range draws the same samples; p = 0 never
    fires, p = 1 always does; the thresholds are (1 - p)^k by repeated multiplication, ceil(2^53 x)."""
    import math

    import circuit_oracle as co

    probs = [0.0, 1.0, 1e-3, 0.05, 0.3, 0.5]
    whole = co.sample_mechanisms(probs, 99, 70, 300)
    split = np.vstack([co.sample_mechanisms(probs, 99, 70, 111), co.sample_mechanisms(probs, 99, 181, 189)])
    assert np.array_equal(whole, split)
    assert not whole[:, 0].any() and whole[:, 1].all()
    T = co.skip_thresholds(0.25)
    t = 1.0
    for k in range(64):
        t *= 0.75
        assert T[k] == math.ceil(math.ldexp(t, 53))
    assert all(T[k] >= T[k + 1] for k in range(63))
    big = co.sample_mechanisms([0.05], 5, 0, 64 * 300)
    assert abs(big.mean() - 0.05) < 5 * np.sqrt(0.05 * 0.95 / big.size)
