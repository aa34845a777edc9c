"""Small helpers shared by the tests (no product code)."""
import os

import numpy as np
import torch

from conftest import GOLDEN


def randomize_bn(model, seed=5):
    """Non-trivial eval-mode BatchNorm statistics (same recipe as tests/golden/make_golden.py)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                n = m.num_features
                m.weight.copy_(torch.rand(n, generator=g) + 0.5)
                m.bias.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_mean.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_var.copy_(torch.rand(n, generator=g) + 0.5)


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def golden_state_dict(z):
    return {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w::")}
