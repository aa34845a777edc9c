"""Synthetic cloud pairs; the real KITTI/ModelNet loaders are out of scope.

src ~ U[-1, 1]^3, R = RotX(tx) @ RotY(ty) @ RotZ(tz) with angles ~ U[0, 2pi) (utils.py:8-26,
KITTIDataset.py:67-81), t ~ U[-1, 1]^3, tgt = R @ src + t.  KITTI-like pairs are fp32 with
C_in = 3 (tgt rounded to fp32); ModelNet-like pairs are fp64 with C_in = 6 (random unit normals,
rotated with the points, ModelNet40Dataset.py:179-196).
"""
import math

import numpy as np
import torch


def rot_xyz(tx, ty, tz):
    cx, sx, cy, sy, cz, sz = math.cos(tx), math.sin(tx), math.cos(ty), math.sin(ty), math.cos(tz), math.sin(tz)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rx @ Ry @ Rz


def make_pairs(B, N, normals=False, seed=1234, scale=1.0):
    """Returns src (B, C, N), tgt (B, C, N), R (B, 3, 3) fp64, t (B, 3, 1) fp64 (CPU tensors)."""
    rng = np.random.default_rng(seed)
    src = rng.uniform(-1.0, 1.0, size=(B, 3, N)) * scale
    Rs, ts, tgts = [], [], []
    for b in range(B):
        R = rot_xyz(*rng.uniform(0.0, 2 * math.pi, size=3))
        t = rng.uniform(-1.0, 1.0, size=(3, 1))
        Rs.append(R)
        ts.append(t)
    R = np.stack(Rs)
    t = np.stack(ts)
    if normals:
        nrm = rng.normal(size=(B, 3, N))
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        src64 = np.concatenate([src, nrm], axis=1)
        tgt64 = np.concatenate([R @ src + t, R @ nrm], axis=1)
        return (torch.from_numpy(src64), torch.from_numpy(tgt64), torch.from_numpy(R), torch.from_numpy(t))
    src32 = src.astype(np.float32)
    tgt32 = (R @ src32.astype(np.float64) + t).astype(np.float32)
    return (torch.from_numpy(src32), torch.from_numpy(tgt32), torch.from_numpy(R), torch.from_numpy(t))
