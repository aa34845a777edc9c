"""Weighting layer on the HIP path -- drop-in for weighting_layer.py:8-33.

Linear 32-16-8-1 with ReLU, ReLU, Softplus (no BN, Q6), then top-K over the points, sorted
descending (ties to the lower index), flattened to (B*K,).
"""
import torch.nn as nn

from . import ops
from ._params import cached_pack, linear_pack, linear_tensors
from .pointnet2_utils import _inference_only


class weighting_layer(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Sequential(nn.Linear(32, 16, True), nn.ReLU())
        self.fc2 = nn.Sequential(nn.Linear(16, 8, True), nn.ReLU())
        self.fc3 = nn.Sequential(nn.Linear(8, 1, True), nn.Softplus())

    def packed_params(self):
        lins = [self.fc1[0], self.fc2[0], self.fc3[0]]
        return cached_pack(self, "wl", linear_tensors(*lins), lambda: linear_pack(*lins))

    def scores(self, X):
        """(B, S, 32) -> (B, S) saliency scores."""
        _inference_only(self)
        B, S, _ = X.shape
        return ops.weighting(X.reshape(B * S, 32).contiguous().float(), self.packed_params()).view(B, S)

    def forward(self, X, K=64):
        return ops.topk(self.scores(X), K).flatten()
