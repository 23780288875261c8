"""Device-resident FirstMinBPDecoder vs the host-stepped loop (one engine launch per first-min step):
decode rate on [h | I] of hgp_34_n625 (the Single-Shot notebook's configuration: p_data = p_synd =
2p/3, p = 0.01, max_iter = N/10, alpha 0.625), and the two paths' agreement.

    python tools/dev/probe_firstmin.py [B]
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from qldpc_fault_tolerance_amd import codes, decoders  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
code = codes.get_code("hgp_34_n625")
hz_ext = np.hstack([code.hz, np.identity(code.hz.shape[0])]).astype(np.uint8)
n = hz_ext.shape[1]
p = 0.01
probs = np.full(n, 2 * p / 3)
rng = np.random.default_rng(5)
e = (rng.random((B, n)) < 2 * p / 3).astype(np.uint8)
synd = (e.astype(np.int64) @ hz_ext.T.astype(np.int64) % 2).astype(np.uint8)
mi = int(code.N / 10)
fm = decoders.FirstMinBPDecoder(hz_ext, probs, mi, "minimum_sum", 0.625)
fm.decode_batch(synd[:256])
torch.cuda.synchronize()
t0 = time.perf_counter()
out = fm.decode_batch(synd)
t_dev = time.perf_counter() - t0
steps = fm.steps_batch
# the host-stepped loop over the engine's one-iteration BP (round 4's path)
st = decoders.FirstMinBPDecoder(hz_ext, probs, mi, "minimum_sum", 0.625)
st._fm = None
st._bp = decoders.BPDecoder(hz_ext, probs, 1, "minimum_sum", 0.625)
Bs = min(B, 8192)
t0 = time.perf_counter()
ref = st._decode_batch_stepped(synd[:Bs])
t_step = time.perf_counter() - t0
print(json.dumps({"B": B, "n": n, "m": int(hz_ext.shape[0]), "max_iter": mi,
                  "device_syndromes_per_s": B / t_dev, "device_s": t_dev,
                  "stepped_syndromes_per_s": Bs / t_step, "stepped_B": Bs,
                  "mean_steps": float(steps.mean()), "max_steps": int(steps.max()),
                  "agree": bool(np.array_equal(out[:Bs], ref))}))
