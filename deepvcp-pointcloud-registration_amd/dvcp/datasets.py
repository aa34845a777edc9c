"""On-disk formats and training-pair synthesis -- drop-in for
KITTIDataset.py and ModelNet40Dataset.py with the clouds resident in HBM.

What the reference does, and what is kept:
* KITTI velodyne scans are raw float32 (x, y, z, reflectance) rows (KITTIDataset.py:39); a scan with
  more than N points is downsampled with ``np.random.choice(num, N, replace=False)`` (:11-16).  The
  first 50 files of ``os.listdir`` of each of the sequences 00-03 are read (:33-36).
* ModelNet40 resampled shapes are comma-separated text rows (x, y, z, nx, ny, nz) read in fp64
  (ModelNet40Dataset.py:38-41); the file list comes from ``modelnet10_{split}.txt`` (or the
  ``_small_`` list) and ``<category>/<name>.txt``.
* ``__getitem__`` draws theta_x, theta_y, theta_z ~ U[0, 2 pi) and t with the same generators in the
  same order (numpy's global generator; ModelNet's t from ``torch.rand``), builds R = Rx Ry Rz
  (utils.py:8-26) on the host in fp64 exactly like the reference, and synthesises the target on the
  GPU (``dvcp_rigid_apply``): target = R src + t in fp64 (KITTI), points R src + t and normals R n
  (ModelNet).  A seeded run therefore yields the reference's R and t bit for bit and its target to
  fp64 rounding.

Clouds are uploaded once at construction (``device``) and every item is produced on the GPU;
there is no CPU fallback (the transform raises without a GPU, like every dvcp op).
"""
import math
import os

import numpy as np
import torch
from torch.utils.data import Dataset

from . import ops


def RotX(theta):
    return np.array([[1, 0, 0], [0, math.cos(theta), -math.sin(theta)], [0, math.sin(theta), math.cos(theta)]])


def RotY(theta):
    return np.array([[math.cos(theta), 0, math.sin(theta)], [0, 1, 0], [-math.sin(theta), 0, math.cos(theta)]])


def RotZ(theta):
    return np.array([[math.cos(theta), -math.sin(theta), 0], [math.sin(theta), math.cos(theta), 0], [0, 0, 1]])


def downsample(src, N):
    """KITTIDataset.py:11-16: a random subset of N rows (no replacement) when there are more."""
    num_src = src.shape[0]
    idx = np.arange(num_src)
    if num_src > N:
        idx = np.random.choice(num_src, N, replace=False)
    return src[idx, :]


def read_kitti_bin(path):
    """A velodyne scan: float32 rows (x, y, z, reflectance) (KITTIDataset.py:39)."""
    return np.fromfile(path, dtype=np.float32, count=-1).reshape([-1, 4])


def read_modelnet_txt(path):
    """A ModelNet40 resampled shape: comma-separated fp64 rows (x, y, z, nx, ny, nz) (ModelNet40Dataset.py:38)."""
    return np.loadtxt(path, delimiter=',', dtype=np.float64)


def _draw_pose():
    """The three angles then t, in the reference's order (KITTIDataset.py:67-75)."""
    tx = np.random.uniform(0, np.pi * 2)
    ty = np.random.uniform(0, np.pi * 2)
    tz = np.random.uniform(0, np.pi * 2)
    return RotX(tx) @ RotY(ty) @ RotZ(tz)


class KITTIDataset(Dataset):
    """KITTIDataset.py:18-95.  Items: (src (3, N) fp32, target (3, N) fp64, R (3, 3) fp64, t (3, 1) fp64),
    all on ``device``."""

    def __init__(self, root, augment=True, rotate=True, split="train", N=10000, device="cuda",
                 sequences=("00", "01", "02", "03"), files_per_sequence=50, verbose=False):
        self.root, self.split, self.augment, self.N = root, split, augment, N
        self.device = torch.device(device)
        self.files, self.points, self.reflectances = [], [], []
        for seq in sequences:
            path = f"{self.root}sequences/{seq}/velodyne/"
            for file in os.listdir(path)[:files_per_sequence]:
                if verbose:
                    print(f"Processing {file}")
                src = downsample(read_kitti_bin(path + file), self.N)
                self.files.append(file)
                self.points.append(torch.from_numpy(np.ascontiguousarray(src[:, :3].T)).to(self.device))
                self.reflectances.append(torch.from_numpy(np.ascontiguousarray(src[:, 3:].T)).to(self.device))
        if verbose:
            print('# Total clouds', len(self.points))

    def __len__(self):
        return len(self.points)

    def __getitem__(self, index):
        src = self.points[index]                                   # 3 x N fp32 (HBM)
        if not self.augment:
            raise NotImplementedError("KITTIDataset.py:96 returns an undefined target when augment=False")
        R = _draw_pose()
        t = np.random.uniform(-1.0, 1.0, (3, 1))
        Rd = torch.from_numpy(R).to(self.device)
        td = torch.from_numpy(t).to(self.device)
        target = ops.rigid_apply(src[None], Rd[None], td[None])[0]   # 3 x N fp64
        return src, target, Rd, td


class ModelNet40Dataset(Dataset):
    """ModelNet40Dataset.py:12-92.  Items: (src (6, N) fp64 = xyz + normals, target (6, N) fp64,
    R (3, 3) fp64, t (3, 1) fp32), all on ``device``."""

    def __init__(self, root, augment=True, rotate=True, full_dataset=True, split="train", device="cuda",
                 verbose=False):
        self.root, self.split, self.augment = root, split, augment
        self.device = torch.device(device)
        self.points, self.labels = [], []
        self.catfile = os.path.join(self.root, 'modelnet10_shape_names.txt')
        self.cat = [line.rstrip() for line in open(self.catfile)]
        lst = f'modelnet10_{split}.txt' if full_dataset else f'modelnet10_small_{split}.txt'
        names = np.atleast_1d(np.loadtxt(os.path.join(self.root, lst), dtype=str))
        for file in names:
            category, _ = file.split('_0')
            data = read_modelnet_txt(os.path.join(self.root, category, file) + '.txt')
            self.points.append(torch.from_numpy(np.ascontiguousarray(data[:, :6].T)).to(self.device))
            self.labels.append(file)
        self.verbose = verbose
        if verbose:
            print("# Total clouds", len(self.points))

    def __len__(self):
        return len(self.points)

    def __getitem__(self, index):
        src = self.points[index]                                   # 6 x N fp64 (HBM)
        if self.verbose:
            print('Processing file:', self.labels[index])
        if not self.augment:
            raise NotImplementedError("ModelNet40Dataset.py:80 uses an undefined target when augment=False")
        R = _draw_pose()
        t = (1.0 - -1.0) * torch.rand(3, 1) + -1.0                # fp32, ModelNet40Dataset.py:67-69
        Rd = torch.from_numpy(R).to(self.device)
        target = ops.rigid_apply(src[None], Rd[None], t.to(self.device)[None])[0]
        return src, target, Rd, t.to(self.device)
