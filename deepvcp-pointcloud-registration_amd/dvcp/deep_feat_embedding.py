"""Deep feature embedding on the HIP path -- drop-in for deep_feat_embedding.py:13-61.

Linear 35-32-32-32 with no nonlinearity (Q14, evaluated layer by layer, not collapsed) and a
max over the 32 neighbours.  ``forward(X, src)`` takes the materialised (B, K, 32, 35) or
(B, K, C, 32, 35) input like the reference; DeepVCP.forward instead uses the fused target
kernel (dvcp_dfe_tgt) that never materialises the target input.
"""
import torch
import torch.nn as nn

from . import autograd, ops
from ._params import cached_pack, linear_pack, linear_tensors
from .cpg import _wants_grad


class feat_embedding_layer(nn.Module):
    def __init__(self, K_nsample=32):
        super().__init__()
        self.K_nsample = 32
        self.fc1 = nn.Linear(35, 32, True)
        self.fc2 = nn.Linear(32, 32, True)
        self.fc3 = nn.Linear(32, 32, True)
        self.max_pool = nn.MaxPool1d(kernel_size=self.K_nsample)

    def packed_params(self):
        lins = [self.fc1, self.fc2, self.fc3]
        return cached_pack(self, "dfe", linear_tensors(*lins), lambda: linear_pack(*lins))

    def forward(self, X, src=True):
        expect = 4 if src else 5
        if X.dim() != expect:
            raise RuntimeError(f"feat_embedding_layer(src={src}) expects a {expect}-D input, got {tuple(X.shape)}")
        if _wants_grad(self, X):
            return autograd.dfe_rows(X, self)
        return ops.dfe(X, self.packed_params())
