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


# ---- tile-level union: 64-point Morton tiles of the target points with boxes; a wave scans a tile
# when some lane's box distance to it is within that lane's 32nd-neighbour distance
def tile_union(order, tiles_lo, tiles_hi):
    tot = 0
    for w in range(0, len(order), 64):
        idx = order[w:w + 64]
        q = Q[idx][:, None, :]
        gap = np.maximum(np.maximum(tiles_lo[None] - q, q - tiles_hi[None]), 0.0)
        need = (gap * gap).sum(-1) <= (rk[idx] ** 2)[:, None]
        tot += np.count_nonzero(need.any(0)) * 64 * len(idx)
    return tot / len(Q)


plo, phi = P.min(0), P.max(0)
pc = np.clip(((P - plo) / (phi - plo) * 16).astype(np.int64), 0, 15)
pcode = spread(pc[:, 0], 4) | (spread(pc[:, 1], 4) << 1) | (spread(pc[:, 2], 4) << 2)
Ps = P[np.argsort(pcode, kind='stable')]
T = (len(Ps) + 63) // 64
Ps = np.concatenate([Ps, np.repeat(Ps[-1:], T * 64 - len(Ps), 0)])
tl, th = Ps.reshape(T, 64, 3).min(1), Ps.reshape(T, 64, 3).max(1)
o_q = np.argsort(morton(Q, 4), kind='stable')
print(f"tile union, queries by own 12-bit Morton cell: {tile_union(o_q, tl, th):.0f} points per query")
Qc = np.clip(Q, plo, phi)   # each query's nearest point of the cloud's bounding box
lo_s, hi_s = lo, hi
lo, hi = plo, phi
for bits in (4, 6):
    o_c = np.lexsort((np.linalg.norm(Q - Qc, axis=1), morton(Qc, bits)))
    print(f"tile union, queries by the {3*bits}-bit Morton cell of their clamp to the cloud box: "
          f"{tile_union(o_c, tl, th):.0f} points per query")
lo, hi = lo_s, hi_s
