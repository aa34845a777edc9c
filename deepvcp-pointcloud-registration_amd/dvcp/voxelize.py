"""Candidate grid on the HIP path -- drop-in for voxelize.py:19-83.

cand[b, n, (ix*G + iy)*G + iz, a] = fp32(fma(s, i_a, (c_a - r) - s/2)), evaluated in fp64 like
torch's CPU arange (Q9: the grid is offset by -s/2, no sphere rejection).
"""
import math

import torch

from . import ops


def grid_side(r, s):
    """Per-axis arange length for a point at the origin (voxelize.py:62-64)."""
    return int(math.ceil(((0.0 + r) - ((0.0 - r) - s / 2)) / s))


def voxelize(point_clouds, r, s, check=True):
    """(B, N, 3) -> (B, N, C, 3) fp32."""
    G = grid_side(r, s)
    cand, err = ops.voxelize(point_clouds, r, s, G, pdim=1)
    if check and int(err.item()) != 0:
        raise RuntimeError("voxelize: a point's per-axis grid length differs from the others")
    return cand


def voxelize_point(point, search_radius, voxel_len):
    """voxelize.py:44-83 for one point (3,) -> (C, 3)."""
    return voxelize(point.reshape(1, 1, 3), search_radius, voxel_len)[0, 0]
