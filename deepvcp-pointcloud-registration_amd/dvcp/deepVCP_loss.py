"""Pose solve on the HIP path -- drop-in for deepVCP_loss.py:13-121.

get_rigid_transform: Kabsch in fp64 (R = V U^T, no reflection fix, Q13).
svd_optimization: SVD -> 1-NN inlier rejection (keep int(0.8 n)) -> SVD on (x1, R1 x1 + t1) (Q12).
deepVCP_loss: alpha * L1 + (1 - alpha) * |mean|, one workgroup per pair (dvcp_svd_optimization).
Set PRINT_LOSS = True to reproduce the reference's ``Loss: ...`` stdout line (:120), which the
reference's loss_vis.py scrapes; it forces a host sync, so it is off by default.
"""
import torch

from . import autograd, ops

PRINT_LOSS = False


def get_rigid_transform(x, y):
    """(B, 3, n) fp64 pairs -> R (B, 3, 3), t (B, 3, 1)."""
    return ops.rigid_transform(x, y)


def svd_optimization(x, y_pred, R_true, t_true):
    R2, t2, x1, y2, _ = ops.svd_optimization(x, y_pred, R_true, t_true)
    return R2, t2, x1, y2


def deepVCP_loss(x, y_pred, R_true, t_true, alpha):
    """x, y_pred (B, K, 3); R_true (B, 3, 3); t_true (B, 3, 1) -> (loss, R (B,3,3), t (B,3,1))."""
    # (B, 3, K) fp64 in one copy each (a permuted .double() left a strided tensor that the pose
    # kernels' operand preparation copied once more)
    x = x.transpose(1, 2).to(torch.float64, memory_format=torch.contiguous_format)
    y_pred = y_pred.transpose(1, 2).to(torch.float64, memory_format=torch.contiguous_format)
    if torch.is_grad_enabled() and y_pred.requires_grad:
        # train.py:121 loss.backward(): both Kabsch solves differentiated on the GPU
        loss, R, t = autograd.pose_loss(x, y_pred, R_true, t_true, alpha)
        if PRINT_LOSS:
            print(f"Loss: {loss}")
        return loss, R, t
    loss, R, t, _ = ops.deepvcp_loss(x, y_pred, R_true, t_true, alpha)   # one HIP solve + the scalar
    if PRINT_LOSS:
        print(f"Loss: {loss}")
    return loss, R, t
