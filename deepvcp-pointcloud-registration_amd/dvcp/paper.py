"""Paper-faithful pose solve and loss (DeepVCP paper, Lu et al. ICCV 2019, Sec. 3.4-3.5; SURVEY.md
8(f) rank 4).  Not reference parity: the reference repository solves the pose with an unweighted
Kabsch and no reflection fix (deepVCP_loss.py:13-44), and its loss compares
the refit pose against the key points (deepVCP_loss.py:105-121).  The paper instead

  * weights each key point's correspondence by its weighting-layer score in the SVD,
  * corrects reflections, R = V diag(1, 1, sign det(V U^T)) U^T,
  * trains on  alpha * mean |R_gt x + t_gt - y*|  +  (1 - alpha) * mean |R_gt x + t_gt - (R x + t)|,

with y* the virtual corresponding points.  Both run in one HIP kernel per pair
(dvcp_paper_pose, fp64).  Forward only: use it to evaluate a model the paper's way
(DeepVCP.forward(..., return_weights=True) hands back the key points' scores).
"""
import torch

from . import _lib
from ._lib import call, ptr, stream


def _b3n(t):
    return t.double().contiguous()


def weighted_rigid_transform(x, y, w=None, reflection_fix=True):
    """Weighted Kabsch on (B, 3, n) point sets (fp64): -> R (B, 3, 3), t (B, 3, 1).  ``w`` (B, n)
    weights (None = uniform; with reflection_fix=False and w=None this is the reference's
    get_rigid_transform up to summation order)."""
    _lib.require_gpu(x, y, w)
    x, y = _b3n(x), _b3n(y)
    B, _, n = x.shape
    wc = None if w is None else w.double().reshape(B, n).contiguous()
    R = torch.empty(B, 3, 3, dtype=torch.float64, device=x.device)
    t = torch.empty(B, 3, 1, dtype=torch.float64, device=x.device)
    call("dvcp_paper_pose", ptr(x), ptr(y), ptr(wc), B, n, int(bool(reflection_fix)), None, None, ptr(R), ptr(t), None,
         stream())
    return R, t


def deepVCP_loss_paper(src_keypts, tgt_vcp, weights, R_true, t_true, alpha=0.5, reflection_fix=True):
    """The paper's loss on key points x = src_keypts (B, K, 3), virtual corresponding points
    y* = tgt_vcp (B, K, 3) and key-point weights (B, K) (None = uniform): -> (loss, R, t)."""
    _lib.require_gpu(src_keypts, tgt_vcp, R_true, t_true)
    x = src_keypts.permute(0, 2, 1).double().contiguous()
    y = tgt_vcp.permute(0, 2, 1).double().contiguous()
    B, _, n = x.shape
    Rt = R_true.double().expand(B, 3, 3).contiguous()
    tt = t_true.double().reshape(-1, 3, 1).expand(B, 3, 1).contiguous()
    wc = None if weights is None else weights.double().reshape(B, n).contiguous()
    R = torch.empty(B, 3, 3, dtype=torch.float64, device=x.device)
    t = torch.empty(B, 3, 1, dtype=torch.float64, device=x.device)
    partial = torch.empty(B, 2, dtype=torch.float64, device=x.device)
    call("dvcp_paper_pose", ptr(x), ptr(y), ptr(wc), B, n, int(bool(reflection_fix)), ptr(Rt), ptr(tt), ptr(R), ptr(t),
         ptr(partial), stream())
    denom = float(B * 3 * n)
    loss = alpha * partial[:, 0].sum() / denom + (1 - alpha) * partial[:, 1].sum() / denom
    return loss, R, t
