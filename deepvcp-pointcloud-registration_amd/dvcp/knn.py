"""Exact kNN on the HIP path -- replaces the un-vendored ``knn_cuda.KNN`` (REF-R R6).

Call surface of the reference's call sites (get_cat_feat_tgt.py:45,52; deepVCP_loss.py:70,72):
``KNN(k, transpose_mode)(ref, query) -> (dist, idx)``.  transpose_mode=True takes
(B, M, 3)/(B, Q, 3) and returns (B, Q, k); False takes (B, 3, M)/(B, 3, Q) and returns
(B, k, Q).  Inputs are read as fp32 (knn_cuda's ``.float()``); idx is int64, 0-based;
dist = sqrt of the fp32 squared distance; ties go to the lower index.
"""
import torch
import torch.nn as nn

from . import ops


class KNN(nn.Module):
    def __init__(self, k, transpose_mode=False):
        super().__init__()
        self.k = k
        self._t = transpose_mode

    def forward(self, ref, query):
        assert ref.size(0) == query.size(0), f"ref.shape={ref.shape} != query.shape={query.shape}"
        pdim = 1 if self._t else 2
        with torch.no_grad():
            dist, _, idx = ops.knn(ref, query, self.k, ref_pdim=pdim, qry_pdim=pdim)
        if not self._t:
            dist, idx = dist.transpose(1, 2), idx.transpose(1, 2)
        return dist, idx
