"""CPU model of the kNN query waves at C3: 64 key points' 11^3 candidate grids
over one synthetic target cloud, the queries in Morton order at several resolutions, and per
query the points inside its wave's box expanded by the wave's largest 32nd-neighbour distance (a
proxy of the union of tiles the wave scans).  Needs scipy; no GPU."""
import os
import sys

import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'deepvcp-pointcloud-registration_amd'))
from scipy.spatial import cKDTree
from dvcp.synthetic import make_pairs
src, tgt, R, t = make_pairs(1, 16384, seed=1234)
P = tgt[0].numpy().T.astype(np.float64)           # (N, 3) target cloud
rng = np.random.default_rng(0)
P = P[rng.choice(len(P), 10000, replace=False)]   # the FE's 10000 target points
kp = P[rng.choice(len(P), 64, replace=False)]      # key points (stand-in: target points)
g = (np.arange(11) - 5) * 0.4
G = np.stack(np.meshgrid(g, g, g, indexing='ij'), -1).reshape(-1, 3)
Q = (kp[:, None, :] + G[None]).reshape(-1, 3)      # 85184 candidate queries
tree = cKDTree(P)
dk, _ = tree.query(Q, k=32)
rk = dk[:, -1]                                     # each query's 32nd-NN distance
lo, hi = Q.min(0), Q.max(0)

def spread(v, bits):
    out = np.zeros_like(v)
    for i in range(bits):
        out |= ((v >> i) & 1) << (3 * i)
    return out

def morton(Q, bits):
    s = (1 << bits)
    q = np.clip(((Q - lo) / (hi - lo) * s).astype(np.int64), 0, s - 1)
    return spread(q[:, 0], bits) | (spread(q[:, 1], bits) << 1) | (spread(q[:, 2], bits) << 2)

def evals(order):
    tot = 0
    for w in range(0, len(order), 64):
        idx = order[w:w + 64]
        q = Q[idx]
        r = rk[idx].max()
        blo, bhi = q.min(0) - r, q.max(0) + r
        # points inside the expanded wave box (a proxy of the union of tiles the wave scans)
        tot += np.count_nonzero(np.all((P >= blo) & (P <= bhi), 1)) * len(idx)
    return tot / len(Q)

for bits in (4, 5, 6, 8, 10):
    code = morton(Q, bits)
    order = np.argsort(code, kind='stable')  # (within-cell order: the generation order)
    print(f"morton {3*bits}-bit: mean points in expanded wave box per query {evals(order):.0f}")
print("mean 32nd-NN distance", rk.mean(), "queries", len(Q))
