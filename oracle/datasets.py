"""CPU restatement of the reference's pair synthesis (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

KITTIDataset.py:11-16 (downsample), :39-49 (read + split), :64-81 (augment);
ModelNet40Dataset.py:38-41 (read), :58-85 (augment); utils.py:8-26 (RotX, RotY, RotZ as np.matrix).
numpy's global generator (and torch's for ModelNet's t) is drawn in the reference's order.
"""
import math

import numpy as np
import torch


def RotX(theta):
    return np.matrix([[1, 0, 0], [0, math.cos(theta), -math.sin(theta)], [0, math.sin(theta), math.cos(theta)]])


def RotY(theta):
    return np.matrix([[math.cos(theta), 0, math.sin(theta)], [0, 1, 0], [-math.sin(theta), 0, math.cos(theta)]])


def RotZ(theta):
    return np.matrix([[math.cos(theta), -math.sin(theta), 0], [math.sin(theta), math.cos(theta), 0], [0, 0, 1]])


def kitti_load(path, N):
    src = np.fromfile(path, dtype=np.float32, count=-1).reshape([-1, 4])
    idx = np.arange(src.shape[0])
    if src.shape[0] > N:
        idx = np.random.choice(src.shape[0], N, replace=False)
    src = src[idx, :]
    return src[:, :3], np.expand_dims(src[:, -1], axis=1)


def kitti_item(src_points):
    """src_points (N, 3) fp32 -> (src (3, N), target (3, N) fp64, R, t) as KITTIDataset.__getitem__."""
    src_points = src_points.T
    theta_x = np.random.uniform(0, np.pi * 2)
    theta_y = np.random.uniform(0, np.pi * 2)
    theta_z = np.random.uniform(0, np.pi * 2)
    t = np.random.uniform(-1.0, 1.0, (3, 1))
    R = RotX(theta_x) @ RotY(theta_y) @ RotZ(theta_z)
    target = R @ src_points + t
    return (torch.from_numpy(src_points), torch.from_numpy(np.asarray(target)), torch.from_numpy(np.asarray(R)),
            torch.from_numpy(t))


def modelnet_item(data):
    """data (N, 6) fp64 rows -> (src (6, N), target (6, N), R, t) as ModelNet40Dataset.__getitem__."""
    src_points, src_normals = data[:, :3].T, data[:, 3:].T
    theta_x = np.random.uniform(0, np.pi * 2)
    theta_y = np.random.uniform(0, np.pi * 2)
    theta_z = np.random.uniform(0, np.pi * 2)
    t = (1.0 - -1.0) * torch.rand(3, 1) + -1.0
    R = RotX(theta_x) @ RotY(theta_y) @ RotZ(theta_z)
    target_points = torch.from_numpy(np.asarray(R @ src_points)) + t
    target_normal = torch.from_numpy(np.asarray(R @ src_normals))
    src = torch.cat((torch.from_numpy(src_points), torch.from_numpy(src_normals)), dim=0)
    return src, torch.cat((target_points, target_normal), dim=0), torch.from_numpy(np.asarray(R)), t
