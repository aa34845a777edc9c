"""Paper-faithful mode (DeepVCP paper, Lu et al. ICCV 2019).  Not reference
parity: the reference repository implements a different network and none of
what follows runs in it.  Everything here is opt-in -- the reference path (dvcp.DeepVCP,
dvcp.deepVCP_loss) is untouched by it.  The checker is oracle/paper.py; DESIGN.md 4.6 lists the
choices the paper leaves open.

  * ``deepVCP_loss_paper`` / ``weighted_rigid_transform`` -- Sec. 3.4-3.5: weighted Kabsch with the
    key points' weights, reflection fix, the outlier rejection (the 20 % pairs with the largest
    residual under the first solve are dropped and the rest solved again) and the two-term L1
    loss.  Differentiable in the virtual corresponding points and the weights: the backward is
    HIP (dvcp_paper_pose_backward).
  * ``PointNetFeaturePropagation`` -- the reference's own dead layer (pointnet2_utils.py:265-315),
    one HIP kernel (dvcp_feature_propagation).
  * ``PaperFeatExtraction`` -- Sec. 3.1 + supplement: PointNet++ with three set-abstraction layers
    (4096 / 1024 / 256 samples) and three feature-propagation layers back to every input point,
    then a 32-unit fully connected layer (fused into the last propagation launch).
  * ``DeepVCPPaper`` -- the whole network with duplication (Sec. 3.6): a shared feature extractor
    and two cascaded stages, the second fed with the first's pose and generating candidates on a
    z line scored by a 1-D CNN (dvcp_cpg1d).  Inference (eval, no_grad).
"""
import torch
import torch.nn as nn

from . import _lib, ops
from ._params import bn_affine, cached_pack
from .cpg import cpg as _cpg3d
from .deep_feat_embedding import feat_embedding_layer
from .pointnet2_utils import PointNetSetAbstraction, _inference_only


def _b3n(t):
    return t.double().contiguous()


def weighted_rigid_transform(x, y, w=None, reflection_fix=True, inlier_ratio=1.0):
    """Weighted Kabsch on (B, 3, n) point sets (fp64): -> R (B, 3, 3), t (B, 3, 1).  ``w`` (B, n)
    weights (None = uniform; with reflection_fix=False, w=None and inlier_ratio=1 this is the
    reference's get_rigid_transform up to summation order); inlier_ratio < 1: the paper's
    rejection step."""
    return ops.paper_pose(x, y, w, reflection_fix=reflection_fix, inlier_ratio=inlier_ratio)


class _PaperLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, w, Rt, tt, alpha, reflection_fix, inlier_ratio):
        R, t, partial = ops.paper_pose(x, y, w, reflection_fix, inlier_ratio, Rt, tt)
        B, _, n = x.shape
        denom = float(B * 3 * n)
        loss = alpha * partial[:, 0].sum() / denom + (1 - alpha) * partial[:, 1].sum() / denom
        ctx.save_for_backward(x, y, w, Rt, tt)
        ctx.cfg = (alpha, reflection_fix, inlier_ratio)
        ctx.mark_non_differentiable(R, t)
        return loss, R, t

    @staticmethod
    def backward(ctx, g_loss, g_R, g_t):
        x, y, w, Rt, tt = ctx.saved_tensors
        alpha, refl, ratio = ctx.cfg
        gy, gw = ops.paper_pose_backward(x, y, w, Rt, tt, alpha, g_loss, refl, ratio, want_w=ctx.needs_input_grad[2])
        return None, gy, gw, None, None, None, None, None


def deepVCP_loss_paper(src_keypts, tgt_vcp, weights, R_true, t_true, alpha=0.5, reflection_fix=True,
                       inlier_ratio=1.0):
    """The paper's loss on key points x = src_keypts (B, K, 3), virtual corresponding points
    y* = tgt_vcp (B, K, 3) and key-point weights (B, K) (None = uniform): -> (loss, R, t).
    inlier_ratio = 0.8 is the paper's rejection step.  Differentiable in tgt_vcp and weights."""
    _lib.require_gpu(src_keypts, tgt_vcp, R_true, t_true)
    x = src_keypts.detach().permute(0, 2, 1).double().contiguous()
    y = tgt_vcp.permute(0, 2, 1).double()
    B, _, n = x.shape
    Rt = R_true.detach().double().expand(B, 3, 3).contiguous()
    tt = t_true.detach().double().reshape(-1, 3, 1).expand(B, 3, 1).contiguous()
    w = None if weights is None else weights.double().reshape(B, n)
    loss, R, t = _PaperLoss.apply(x, y.contiguous(), None if w is None else w.contiguous(), Rt, tt, float(alpha),
                                  bool(reflection_fix), float(inlier_ratio))
    return loss, R, t


# ------------------------------------------------------------------------------ feature extractor
class PointNetFeaturePropagation(nn.Module):
    """pointnet2_utils.py:265-315 (same parameters and state_dict keys: mlp_convs.i, mlp_bns.i);
    forward(xyz1 (B, 3, N), xyz2 (B, 3, S), points1 (B, D1, N) or None, points2 (B, D2, S)) ->
    (B, D', N), one HIP launch (eval-mode BN folded; inference only)."""

    def __init__(self, in_channel, mlp):
        super().__init__()
        self.mlp_convs = nn.ModuleList()
        self.mlp_bns = nn.ModuleList()
        last = in_channel
        for out in mlp:
            self.mlp_convs.append(nn.Conv1d(last, out, 1))
            self.mlp_bns.append(nn.BatchNorm1d(out))
            last = out
        self.chans = [in_channel] + list(mlp)

    def packed_params(self, fc=None):
        """W | b | scale | shift per layer (BN folded), then the optional fc as a plain layer."""
        tensors = [t for conv, bn in zip(self.mlp_convs, self.mlp_bns)
                   for t in (conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var)]
        if fc is not None:
            tensors += [fc.weight, fc.bias]

        def build():
            parts = []
            for conv, bn in zip(self.mlp_convs, self.mlp_bns):
                scale, shift = bn_affine(bn)
                parts += [conv.weight.reshape(-1), conv.bias, scale, shift]
            if fc is not None:
                n = fc.weight.shape[0]
                parts += [fc.weight.reshape(-1), fc.bias, torch.ones(n, device=fc.weight.device),
                          torch.zeros(n, device=fc.weight.device)]
            return torch.cat(parts)

        return cached_pack(self, "fp" if fc is None else "fp_fc", tensors, build)

    def run(self, xyz1, xyz2, p1, p2_rows, fc=None):
        """-> (B, N, C) rows; p2_rows (B, S, D2) fp32 row-major, p1 (B, D1, N) view or None."""
        chans = self.chans + ([fc.weight.shape[0]] if fc is not None else [])
        relu = [1] * len(self.mlp_convs) + ([0] if fc is not None else [])
        return ops.feature_propagation(xyz1, xyz2, p2_rows, p1, chans, relu, self.packed_params(fc))

    def forward(self, xyz1, xyz2, points1, points2):
        _inference_only(self)
        rows = self.run(xyz1, xyz2, points1, points2.permute(0, 2, 1).contiguous().float())
        return rows.permute(0, 2, 1)


def paper_fe_config(use_normal=False, npoints=(4096, 1024, 256), radii=(0.1, 0.2, 0.4), nsample=32):
    """Supplement Sec. 1 (see oracle/paper.py)."""
    d0 = 3 if use_normal else 0
    sa = [dict(npoint=npoints[0], radius=radii[0], nsample=nsample, in_channel=3 + d0, mlp=[32, 32]),
          dict(npoint=npoints[1], radius=radii[1], nsample=nsample, in_channel=32 + 3, mlp=[32, 64]),
          dict(npoint=npoints[2], radius=radii[2], nsample=nsample, in_channel=64 + 3, mlp=[64, 64])]
    fp = [dict(in_channel=64 + 64, mlp=[64, 64]), dict(in_channel=32 + 64, mlp=[32, 32]),
          dict(in_channel=d0 + 32, mlp=[32, 32, 32])]
    return sa, fp


class PaperFeatExtraction(nn.Module):
    """Paper Sec. 3.1: per-point features (B, N, 32) for every input point.  forward(pts (B, C, N),
    starts=None (3, B) FPS starts, drawn like the reference's sample_and_group when None)."""

    def __init__(self, use_normal=False, **cfg):
        super().__init__()
        self.use_normal = use_normal
        sa, fp = paper_fe_config(use_normal, **cfg)
        self.sa1, self.sa2, self.sa3 = (PointNetSetAbstraction(**c) for c in sa)
        self.fp3, self.fp2, self.fp1 = (PointNetFeaturePropagation(**c) for c in fp)
        self.fc = nn.Linear(32, 32)

    def draw_starts(self, B, N):
        return torch.stack([torch.randint(0, n, (B,), dtype=torch.long)
                            for n in (N, self.sa1.npoint, self.sa2.npoint)])

    def forward(self, pts, starts=None):
        _inference_only(self)
        B, _, N = pts.shape
        if starts is None:
            starts = self.draw_starts(B, N)
        xyz = pts[:, :3, :]
        feat = pts[:, 3:, :] if self.use_normal else None
        levels = [(xyz, feat)]
        f_rows = None
        for sa, st in zip((self.sa1, self.sa2, self.sa3), starts):
            pxyz, pf = levels[-1]
            _, c = ops.fps(pxyz, sa.npoint, st.to(pts.device), pdim=2)
            ns = min(int(sa.nsample), pxyz.shape[2])
            count, lst, _ = ops.ball_query(pxyz, c, sa.radius, ns, pdim=2, cdim_pts=2)
            f_rows = ops.sa_group_mlp(pxyz, c, pf, count, lst, ns, sa.chans, sa.packed_params(), xyz_pdim=2,
                                      feat_ddim=1, feat_pdim=2)          # (B, S, C)
            levels.append((c, f_rows.permute(0, 2, 1)))
        (x0, f0), (x1, f1), (x2, f2), (x3, f3) = levels
        g2 = self.fp3.run(x2, x3, f2, f3.permute(0, 2, 1))                # (B, 1024, 64)
        g1 = self.fp2.run(x1, x2, f1, g2)                                 # (B, 4096, 32)
        return self.fp1.run(x0, x1, f0, g1, fc=self.fc)                   # (B, N, 32) incl. fc


class PaperWeighting(nn.Module):
    """Paper Sec. 3.2: FC 16 (BN, ReLU), FC 8 (BN, ReLU), FC 1 softplus; eval BN folded into the
    linear layers, one HIP launch (dvcp_weighting)."""

    def __init__(self):
        super().__init__()
        self.fc1, self.bn1 = nn.Linear(32, 16), nn.BatchNorm1d(16)
        self.fc2, self.bn2 = nn.Linear(16, 8), nn.BatchNorm1d(8)
        self.fc3 = nn.Linear(8, 1)

    def packed_params(self):
        tensors = [self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, self.fc3.weight, self.fc3.bias]
        tensors += [t for bn in (self.bn1, self.bn2) for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)]

        def build():
            parts = []
            for lin, bn in ((self.fc1, self.bn1), (self.fc2, self.bn2)):
                s, h = bn_affine(bn)
                parts += [(lin.weight * s[:, None]).reshape(-1), lin.bias * s + h]
            return torch.cat(parts + [self.fc3.weight.reshape(-1), self.fc3.bias])

        return cached_pack(self, "pwl", tensors, build)

    def forward(self, f):
        """(B, N, 32) -> (B, N) scores."""
        _inference_only(self)
        B, N, _ = f.shape
        return ops.weighting(f.reshape(B * N, 32).contiguous().float(), self.packed_params()).view(B, N)


class CPG1D(nn.Module):
    """Paper Sec. 3.6: the back network's CPG, Conv1d 32-16-4-1 (k 3, p 1) over a z line of
    candidates, softmax, weighted candidate mean (one wave per key point, dvcp_cpg1d)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv1d(32, 16, 3, padding=1)
        self.conv2 = nn.Conv1d(16, 4, 3, padding=1)
        self.conv3 = nn.Conv1d(4, 1, 3, padding=1)

    def packed_params(self):
        tensors = [t for c in (self.conv1, self.conv2, self.conv3) for t in (c.weight, c.bias)]
        return cached_pack(self, "cpg1d", tensors, lambda: torch.cat([t.reshape(-1) for t in tensors]))

    def forward(self, src, tgt, cand):
        _inference_only(self)
        return ops.cpg1d(src, tgt, cand, self.packed_params())


class _Stage(nn.Module):
    def __init__(self, one_d):
        super().__init__()
        self.WL = PaperWeighting()
        self.DFE = feat_embedding_layer()
        self.cpg = CPG1D() if one_d else _cpg3d()
        self.one_d = one_d


def centred_grid(G, s, device, dtype=torch.float64):
    ax = (torch.arange(G, dtype=dtype, device=device) - (G - 1) / 2.0) * s
    return torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)


class DeepVCPPaper(nn.Module):
    """The paper's network with duplication (Sec. 3, 3.6; oracle/paper.py DeepVCPPaper is its
    checker; same submodule names and state_dict keys).  forward(src (B, C, N), tgt, R_init
    (B|1, 3, 3), t_init (B|1, 3[, 1])) -> list of per-stage dicts (keypts, vcp, weights, R, t, ...).
    ``starts``: (2, 3, B) FPS starts of the two FE calls; ``keypoint_idx``: optional per-stage
    (B, K) key-point overrides for stage-decoupled parity tests."""

    def __init__(self, use_normal=False, K=64, r=2.0, s=0.4, s_z=0.25, d=1.0, nsample=32, duplication=True,
                 inlier_ratio=0.8, **fe_cfg):
        super().__init__()
        self.FE = PaperFeatExtraction(use_normal, **fe_cfg)
        self.stages = nn.ModuleList([_Stage(False)] + ([_Stage(True)] if duplication else []))
        self.K, self.r, self.s, self.s_z, self.d, self.ns = K, r, s, s_z, d, nsample
        self.inlier_ratio = inlier_ratio

    def forward(self, src, tgt, R_init, t_init, starts=None, keypoint_idx=None):
        _inference_only(self)
        _lib.require_gpu(src, tgt)
        B, _, N = src.shape
        dev = src.device
        if starts is None:
            starts = torch.stack([self.FE.draw_starts(B, N), self.FE.draw_starts(B, tgt.shape[2])])
        f_src, f_tgt = self.FE(src, starts[0]), self.FE(tgt, starts[1])
        xs, xt = src[:, :3, :], tgt[:, :3, :]
        xs_rows = xs.permute(0, 2, 1)
        Rc = R_init.to(dev, torch.float64).expand(B, 3, 3)
        tc = t_init.to(dev, torch.float64).reshape(-1, 3).expand(B, 3)
        out = []
        for si, st in enumerate(self.stages):
            score = st.WL(f_src)
            top = ops.topk(score, self.K) if keypoint_idx is None else keypoint_idx[si].to(dev, torch.int64)
            w = torch.gather(score, 1, top)
            kp = torch.gather(xs_rows, 1, top[..., None].expand(B, self.K, 3)).contiguous()   # (B, K, 3)
            ns_src = min(self.ns, N)
            cnt, lst, _ = ops.ball_query(xs, kp, self.d, ns_src, pdim=2, cdim_pts=1)
            rows = ops.group_rows(kp, xs, f_src, cnt, lst, self.ns, self.d)
            src_dfe = ops.dfe(rows, st.DFE.packed_params())                                  # (B, K, 32)
            moved = torch.einsum("bij,bkj->bki", Rc, kp.double()) + tc[:, None, :]
            if st.one_d:
                G = int(2 * self.r / self.s_z + 1)
                off = torch.zeros(G, 3, dtype=torch.float64, device=dev)
                off[:, 2] = (torch.arange(G, dtype=torch.float64, device=dev) - (G - 1) / 2.0) * self.s_z
            else:
                G = int(2 * self.r / self.s + 1)
                off = centred_grid(G, self.s, dev)
            cand = (moved[:, :, None, :] + off[None, None]).float().contiguous()            # (B, K, C, 3)
            C = cand.shape[2]
            qry = cand.view(B, self.K * C, 3)
            ns_tgt = min(self.ns, xt.shape[2])
            cnt, lst, _ = ops.ball_query(xt, qry, self.d, ns_tgt, pdim=2, cdim_pts=1)
            trows = ops.group_rows(qry, xt, f_tgt, cnt, lst, self.ns, self.d)
            tgt_dfe = ops.dfe(trows, st.DFE.packed_params()).view(B, self.K, C, 32)
            if st.one_d:
                vcp = ops.cpg1d(src_dfe, tgt_dfe, cand, st.cpg.packed_params())
            else:
                # cpg.py:34's reshape of a (B, K, 32, C) view whose row-major order is the
                # candidates' own: the 3-D grid without the reference's Q11 scramble
                vcp = ops.cpg(src_dfe, tgt_dfe.contiguous().view(B, self.K, 32, C), cand, G,
                              st.cpg.packed_params())
            R, t = ops.paper_pose(kp.permute(0, 2, 1), vcp.permute(0, 2, 1), w, True, self.inlier_ratio)
            Rc, tc = R, t.reshape(B, 3)
            out.append(dict(keypts=kp, vcp=vcp, weights=w, R=R, t=t, topk=top, cand=cand, src_dfe=src_dfe,
                            tgt_dfe=tgt_dfe, score=score))
        return out


__all__ = ["deepVCP_loss_paper", "weighted_rigid_transform", "PointNetFeaturePropagation", "PaperFeatExtraction",
           "PaperWeighting", "CPG1D", "DeepVCPPaper", "paper_fe_config"]
