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


def randomize_bn(model, seed=5):
    """Non-trivial eval-mode BatchNorm affine/statistics (default init is the identity)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                n = m.num_features
                m.weight.copy_(torch.rand(n, generator=g) + 0.5)
                m.bias.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_mean.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_var.copy_(torch.rand(n, generator=g) + 0.5)


def condition_weights(model, feats=None, wl_scale=10.0, target_std=2.0, seed=5):
    """Random init made well-conditioned for parity checks (every op and shape stays the
    reference's): BN statistics randomised; the weighting layer's fc1/fc2 weights drawn at
    `wl_scale` x the default scale; fc3 rescaled/shifted so that the pre-Softplus logit has mean 0
    and std `target_std` on `feats` (P x 32 FE features, any device).

    Why: with the default init the key-point scores are 0.62 +- 1e-4, so the top-k ORDER is
    decided by fp32 rounding noise (in the reference as much as here).  Conditioned, adjacent
    top-64 scores differ by ~1e-3 relative.  Load the resulting state_dict into every model
    compared (oracle and GPU) so they share identical weights."""
    randomize_bn(model, seed)
    wl = model.WL
    with torch.no_grad():
        for lin in (wl.fc1[0], wl.fc2[0]):
            lin.weight.mul_(wl_scale)
        if feats is not None:
            f = feats.reshape(-1, 32).double().cpu()
            h = torch.relu(f @ wl.fc1[0].weight.double().cpu().t() + wl.fc1[0].bias.double().cpu())
            h = torch.relu(h @ wl.fc2[0].weight.double().cpu().t() + wl.fc2[0].bias.double().cpu())
            z = h @ wl.fc3[0].weight.double().cpu().t()
            scale = target_std / max(float(z.std()), 1e-30)
            wl.fc3[0].weight.mul_(scale)
            wl.fc3[0].bias.fill_(-float(z.mean()) * scale)
    return model
