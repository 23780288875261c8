"""CodeSimulator_Phenon with FirstMinBPDecoder decoder1 and BPOSD_Decoder decoder2 (the Single-Shot
notebook, cell 18 / 22 form: [h | I] priors p_data = p_synd = 2p/3, max_iter = N/10, alpha 0.625,
osd_e order 10), fused on the GPU (qldpc_phenl_set_round_firstmin) against the reference's per-sample
loop over the same device decoders.

    python tools/dev/probe_phen_firstmin.py [code] [samples] [rounds]
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from qldpc_fault_tolerance_amd import codes, decoders, simulators  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n625"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
code = codes.get_code(name)
p = 0.01
pd = 2 * p / 3
mi = int(code.N / 10)
ext = lambda h: np.hstack([h, np.identity(h.shape[0])])  # noqa: E731


def sim(seed):
    d1x = decoders.FirstMinBPDecoder(ext(code.hz), np.hstack([pd * np.ones(code.N), pd * np.ones(code.hz.shape[0])]),
                                     mi, "minimum_sum", 0.625)
    d1z = decoders.FirstMinBPDecoder(ext(code.hx), np.hstack([pd * np.ones(code.N), pd * np.ones(code.hx.shape[0])]),
                                     mi, "minimum_sum", 0.625)
    d2x = decoders.BPOSD_Decoder(code.hz, pd * np.ones(code.N), mi, "minimum_sum", 0.625, "osd_e", 10)
    d2z = decoders.BPOSD_Decoder(code.hx, pd * np.ones(code.N), mi, "minimum_sum", 0.625, "osd_e", 10)
    return simulators.CodeSimulator_Phenon(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x, decoder2_z=d2z,
                                           pauli_error_probs=[p / 3] * 3, q=pd, eval_logical_type="Total", seed=seed)


s = sim(11)
s.WordErrorRate(R, 1024)  # warm-up (graphs, anneal, first launch)
t0 = time.perf_counter()
wer, _ = s.WordErrorRate(R, S)
t_fused = time.perf_counter() - t0
res = s.last_result
s2 = sim(12)
n_ps = 64
t0 = time.perf_counter()
fails = sum(int(s2._single_run(R)) for _ in range(n_ps))
t_ps = time.perf_counter() - t0
print(json.dumps({"code": name, "samples": S, "rounds": R, "fused_samples_per_s": S / t_fused, "fused_s": t_fused,
                  "wer": wer, "failures": res.failures, "mean_firstmin_steps_x": res.sector_iters[0] / max(1, res.sector_decodes[0]),
                  "per_sample_path_samples_per_s": n_ps / t_ps, "per_sample_samples": n_ps, "per_sample_failures": fails}))
