"""Registration error metric of the reference's harness on the HIP path (train.py:112-120, :156-164).

The reference prints, per batch, the rotation error ||euler_xyz_deg(R_pred) - euler_xyz_deg(R_gt)||
(scipy Rotation.as_euler('xyz', degrees=True), nn.PairwiseDistance(p=2)) and the translation error
||t_pred - t_gt||.  Its translation line crashes as written (C8: PairwiseDistance on (B,3,1)
tensors gives (B,3) and .item() raises); REF-R takes the norm over the three components.
``registration_errors`` returns both per pair on the GPU (dvcp_registration_error), so a
multi-GPU job all-gathers them with the poses.
"""
from . import ops


def registration_errors(R_pred, t_pred, R_gt, t_gt):
    """-> (rot_err (B,) degrees, trans_err (B,)) fp64 on the device."""
    return ops.registration_error(R_pred, t_pred, R_gt, t_gt)
