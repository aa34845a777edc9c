"""Get_Cat_Feat_Src -- drop-in for get_cat_feat_src.py:16-55 (prints removed).

Standalone module for API parity, composed from device tensor ops.  DeepVCP.forward does not
call it: the same arithmetic runs fused inside the dvcp_src_keypoints HIP kernel.
"""
import torch
import torch.nn as nn


class Get_Cat_Feat_Src(nn.Module):
    def forward(self, src_keypts, src_keypts_grouped_pts, src_keyfeats):
        B, K, ns, nf = src_keyfeats.shape
        kp = src_keypts[:, :, :3].unsqueeze(2).expand(B, K, ns, 3)
        # PairwiseDistance(p=2, eps=1e-6): ||(a - b) + eps|| (Q5: a absolute, b local)
        dist = nn.PairwiseDistance(p=2, keepdim=True)(kp.reshape(-1, 3), src_keypts_grouped_pts[..., :3].reshape(-1, 3))
        dist = dist.view(B, K, ns, 1)
        w = dist / torch.sum(dist, dim=2, keepdim=True)
        local = src_keypts_grouped_pts[:, :, :, :3] - kp
        return torch.cat((local, src_keyfeats * w), dim=3)
