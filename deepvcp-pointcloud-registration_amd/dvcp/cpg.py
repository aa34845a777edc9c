"""Corresponding point generation on the HIP path -- drop-in for cpg.py:14-60.

Cost volume (src - tgt)^2 with the reference's reshape of the permuted target (Q11), Conv3d
32-16-4-1 (k3, p1, no activations), softmax over the C = G^3 candidates, weighted mean of the
candidates.  One gfx950 workgroup per key point (dvcp_cpg).
"""
import torch
import torch.nn as nn

from . import autograd, ops
from ._params import cached_pack


class cpg(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv3d(in_channels=32, out_channels=16, kernel_size=3, stride=1, padding=1)
        self.conv2 = nn.Conv3d(in_channels=16, out_channels=4, kernel_size=3, stride=1, padding=1)
        self.conv3 = nn.Conv3d(in_channels=4, out_channels=1, kernel_size=3, stride=1, padding=1)
        self.softmax = nn.Softmax(dim=-1)

    def packed_params(self):
        convs = [self.conv1, self.conv2, self.conv3]
        tensors = [t for c in convs for t in (c.weight, c.bias)]
        return cached_pack(self, "cpg", tensors,
                           lambda: torch.cat([t.reshape(-1) for t in tensors]))

    def forward(self, src_dfe_feat, tgt_dfe_feat, candidates, r, s, return_weights=False):
        """src (B, N, 1, 32), tgt (B, N, 32, C), candidates (B, N, C, 3) -> vcp (B, N, 3)."""
        B, N, C, _ = candidates.shape
        grid_size = int((2 * r) / s + 1)
        assert C == grid_size * grid_size * grid_size
        if not return_weights and _wants_grad(self, src_dfe_feat, tgt_dfe_feat):
            return autograd.cpg(src_dfe_feat, tgt_dfe_feat, candidates, grid_size, self)
        return ops.cpg(src_dfe_feat, tgt_dfe_feat, candidates, grid_size, self.packed_params(),
                       want_weight=return_weights)


def _wants_grad(module, *inputs):
    """Autograd is on and something upstream of the output requires a gradient."""
    if not torch.is_grad_enabled():
        return False
    return any(p.requires_grad for p in module.parameters()) or any(t.requires_grad for t in inputs)
