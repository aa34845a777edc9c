"""Get_Cat_Feat_Tgt -- drop-in for get_cat_feat_tgt.py:18-98 with REF-R R4 (per-batch gather)
and R5 (pass the target FE xyz as ``tgt_pts_xyz``).

Standalone module for API parity: it materialises the (B, K, C, 32, 35) fp64 tensor exactly as
the reference does (kNN on the HIP path, gathers as device ops).  DeepVCP.forward never builds
it -- dvcp_dfe_tgt gathers and weights each row in registers (Q10 weighting kept).
"""
import torch
import torch.nn as nn

from .knn import KNN


class Get_Cat_Feat_Tgt(nn.Module):
    def forward(self, candidate_pts, src_keypts, tgt_pts_xyz, tgt_deep_feat_pts):
        B = src_keypts.shape[0]
        k_nn = 32
        qry = torch.flatten(candidate_pts, 1, 2)
        dist, idx = KNN(k=k_nn, transpose_mode=True)(tgt_pts_xyz, qry)
        cand_rep = candidate_pts.unsqueeze(3).expand(*candidate_pts.shape[:3], k_nn, 3)
        w = dist / torch.sum(dist, dim=2, keepdim=True, dtype=torch.float64)
        wmap = w.unsqueeze(2).expand(B, qry.shape[1], k_nn, k_nn)
        nk, nc, nf = src_keypts.shape[1], candidate_pts.shape[2], tgt_deep_feat_pts.shape[2]
        bsel = torch.arange(B, device=idx.device).view(B, 1, 1).expand_as(idx)
        feat = tgt_deep_feat_pts[bsel, idx, :].view(B, nk, nc, k_nn, nf)
        pts = tgt_pts_xyz[bsel, idx, :].view(B, nk, nc, k_nn, 3)
        return torch.cat((pts - cand_rep, feat * wmap.reshape(B, nk, nc, k_nn, nf)), dim=4)
