import numpy as np, sys
sys.path.insert(0, '/root/repo')
from oracle import oracle
from qldpc_fault_tolerance_amd import codes
H = codes.get_code('hgp_34_n1600').hz.astype(np.uint8)
m, n = H.shape
p = 0.04
rng = np.random.default_rng(1)
B = 96
e = (rng.random((B, n)) < p).astype(np.uint8)
synd = (e.astype(np.int64) @ H.T % 2).astype(np.uint8)
c, it, conv, post = oracle.bp_decode_batch_soft(H, p, 160, 0.625, synd, 64)
last = []
for b in np.flatnonzero(~conv)[:60]:
    order = np.argsort(post[b], kind='stable')
    A = np.packbits(H[:, order], axis=1, bitorder='little').view(np.uint8)  # rows as bytes
    A = H[:, order].copy()
    used = np.zeros(m, bool); r = 0
    for c_ in range(n):
        cand = np.flatnonzero(A[:, c_] & ~used)
        if len(cand) == 0: continue
        pr = cand[0]; used[pr] = True; r += 1
        rows = np.flatnonzero(A[:, c_]); rows = rows[rows != pr]
        A[rows] ^= A[pr]
        if r == 768: last.append(c_); break
last = np.array(last)
print("n non-conv", (~conv).sum(), "last pivot pos: min", last.min(), "median", np.median(last), "p90", np.percentile(last, 90), "max", last.max())
print("words needed", np.bincount(last // 64 + 1))
