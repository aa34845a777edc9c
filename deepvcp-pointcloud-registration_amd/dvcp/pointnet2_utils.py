"""PointNet++ primitives on the HIP path -- drop-in for the reference's pointnet2_utils.py.

Same names, arguments and outputs as pointnet2_utils.py:19-202 (the part the DeepVCP forward
uses); the work runs in hand-written gfx950 kernels (dvcp_fps, dvcp_ball_query,
dvcp_sa_group_mlp, dvcp_square_distance).  Training mode uses batch-statistics BatchNorm
(dvcp/batchnorm.py); the backward runs through dvcp.autograd.feat_extraction.
"""
import torch
import torch.nn as nn

from . import batchnorm, ops
from ._params import bn_affine, cached_pack

__all__ = ["square_distance", "index_points", "farthest_point_sample", "query_ball_point", "sample_and_group",
           "PointNetSetAbstraction"]


def square_distance(src, dst):
    """pointnet2_utils.py:19-40: (B, S, 3), (B, N, 3) -> (B, S, N), expansion form."""
    return ops.square_distance(src, dst)


def index_points(points, idx):
    """pointnet2_utils.py:43-60: out[b, ...] = points[b, idx[b, ...], :] (a device gather)."""
    B = points.shape[0]
    view = [B] + [1] * (idx.dim() - 1)
    bidx = torch.arange(B, device=points.device).view(view).expand_as(idx)
    return points[bidx, idx, :]


def farthest_point_sample(xyz, npoint, start=None):
    """pointnet2_utils.py:63-84: (B, N, 3) -> (B, npoint) int64.  The start index is drawn
    with torch.randint on the CPU generator exactly as the reference does (:75)."""
    B, N, _ = xyz.shape
    if start is None:
        start = torch.randint(0, N, (B,), dtype=torch.long)
    idx, _ = ops.fps(xyz, npoint, start.to(xyz.device), pdim=1)
    return idx


def query_ball_point(radius, nsample, xyz, new_xyz):
    """pointnet2_utils.py:87-107: (B, N, 3), (B, S, 3) -> (B, S, min(nsample, N)) int64."""
    ns = min(int(nsample), xyz.shape[1])
    _, _, pad = ops.ball_query(xyz, new_xyz, radius, ns, pdim=1, cdim_pts=1, compact=False, padded=True)
    return pad


def sample_and_group(npoint, radius, nsample, xyz, points, returnidx=False, start=None):
    """pointnet2_utils.py:110-138."""
    B, N, C = xyz.shape
    fps_idx = farthest_point_sample(xyz, npoint, start=start)
    new_xyz = index_points(xyz, fps_idx)
    idx = query_ball_point(radius, nsample, xyz, new_xyz)
    grouped = index_points(xyz, idx) - new_xyz.view(B, npoint, 1, C)
    if points is not None:
        grouped = torch.cat([grouped, index_points(points, idx)], dim=-1)
    if returnidx:
        return new_xyz, grouped, idx
    return new_xyz, grouped


def _inference_only(module):
    if module.training:
        raise NotImplementedError(f"dvcp: {type(module).__name__}.forward in training mode needs autograd "
                                  "(train through DeepVCP.forward with gradients enabled) or .eval()")


class PointNetSetAbstraction(nn.Module):
    """pointnet2_utils.py:161-202 (group_all=False).  Same parameters and state_dict keys
    (mlp_convs.i.weight/bias, mlp_bns.i.*); the forward is fused FPS -> ball query ->
    grouped MLP + max on the GPU, evaluating the MLP once per distinct ball-query hit."""

    def __init__(self, npoint, radius, nsample, in_channel, mlp, group_all=False):
        super().__init__()
        if group_all:
            raise NotImplementedError("group_all=True is dead code in the reference forward")
        self.npoint, self.radius, self.nsample = npoint, radius, nsample
        self.mlp_convs = nn.ModuleList()
        self.mlp_bns = nn.ModuleList()
        last = in_channel
        for width in mlp:
            self.mlp_convs.append(nn.Conv2d(last, width, 1))
            self.mlp_bns.append(nn.BatchNorm2d(width))
            last = width
        self.chans = [in_channel] + list(mlp)
        self.group_all = group_all

    def packed_params(self):
        tensors = []
        for conv, bn in zip(self.mlp_convs, self.mlp_bns):
            tensors += [conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var]

        def build():
            parts = []
            for conv, bn in zip(self.mlp_convs, self.mlp_bns):
                scale, shift = bn_affine(bn)
                parts += [conv.weight.reshape(-1), conv.bias, scale, shift]
            return torch.cat(parts)

        return cached_pack(self, "sa", tensors, build)

    def forward(self, xyz, points, start=None):
        """xyz (B, 3, N), points (B, D, N) or None -> new_xyz (B, 3, S), features (B, D', S).
        In training mode the BatchNorms use batch statistics and update their running statistics.
        This module has no autograd path of its own (its backward runs inside
        dvcp.autograd.feat_extraction, i.e. through feat_extraction_layer / DeepVCP): with
        gradients enabled and a trainable parameter it raises instead of returning features that
        silently carry no gradient."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError(
                "dvcp: PointNetSetAbstraction.forward is not differentiable on its own; train it through "
                "feat_extraction_layer / DeepVCP (dvcp.autograd.feat_extraction), or call it under torch.no_grad()")
        B, _, N = xyz.shape
        if start is None:
            start = torch.randint(0, N, (B,), dtype=torch.long)
        _, new_xyz = ops.fps(xyz, self.npoint, start.to(xyz.device), pdim=2)
        ns = min(int(self.nsample), N)
        count, lst, _ = ops.ball_query(xyz, new_xyz, self.radius, ns, pdim=2, cdim_pts=2)
        if self.training:
            out, _ = batchnorm.train_forward(self, xyz, new_xyz, points, count, lst, ns)
            return new_xyz, out.permute(0, 2, 1)
        out = ops.sa_group_mlp(xyz, new_xyz, points, count, lst, ns, self.chans, self.packed_params(),
                               xyz_pdim=2, feat_ddim=1, feat_pdim=2)
        return new_xyz, out.permute(0, 2, 1)
