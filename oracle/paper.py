"""Checker for the paper-faithful mode (dvcp.paper).

TEST INFRASTRUCTURE ONLY (the checker for dvcp.paper, never called by the product path).  The
DeepVCP paper (Lu et al., ICCV 2019, vendored as DeepVCP_W.Lu_S.Song_ICCV2019.pdf) describes a
network the reference repository does not implement; this module restates it in numpy / plain
torch CPU ops so the HIP paper mode can be checked:

  * the pose solve and loss (Sec. 3.4-3.5): weighted Kabsch with the key points' weights,
    reflection-corrected, an outlier-rejection step that drops the 20 % pairs with the largest
    residual under the first estimate and solves again, and the two-term L1 loss;
  * the per-point feature extractor (Sec. 3.1 + supplement Sec. 1): PointNet++ with three
    set-abstraction layers (4096 / 1024 / 256 samples, MLPs 32-32, 32-64, 64-64) and three
    feature-propagation layers (64-64, 32-32, 32-32-32) back to every input point, then a 32-unit
    fully connected layer.  The feature-propagation layer is the reference's own (dead)
    PointNetFeaturePropagation (pointnet2_utils.py:265-315), restated line by line;
  * the weighting layer with batch norm on its first two layers (Sec. 3.2);
  * the deep feature embedding on ball-query neighbourhoods of radius d = 1 (Sec. 3.3, K = 32,
    duplicated when fewer, local coordinates normalised by d);
  * the corresponding point generation on a centred candidate grid (Sec. 3.4, no Q11 scramble);
  * duplication (Sec. 3.6): a second network sharing the feature extractor, fed with the first
    network's pose, whose CPG is a 1-D CNN over candidates along z only.

Where the paper leaves a choice open it is fixed here and in dvcp.paper alike:
set-abstraction radii 0.1 / 0.2 / 0.4 with 32 neighbours, DFE activations as the reference's
feat_embedding_layer (none), candidates with no neighbour inside d give all-zero rows, the
z line has s_z = 0.25 and the same half-width r.  There is no reference implementation of any of
this, so it is "parity unpinned" against the reference; it is pinned by its own known-answer
tests (tests/test_oracle_kat.py: exact rotations under weights, zero-weight outliers, mirrored
sets, rejection of planted outliers, interpolation of constant and linear fields, the 1-D CPG on
a planted peak)."""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ref_r as R_


# ---------------------------------------------------------------------------------------- pose
def weighted_rigid_transform(x, y, w=None, reflection_fix=True):
    """x, y (3, n) float64, w (n,) -> R (3, 3), t (3,)."""
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    w = np.ones(x.shape[1]) if w is None else np.asarray(w, np.float64)
    cx = (x * w).sum(1) / w.sum()
    cy = (y * w).sum(1) / w.sum()
    H = ((x - cx[:, None]) * w) @ (y - cy[:, None]).T
    U, S, Vt = np.linalg.svd(H)
    V = Vt.T
    d = np.sign(np.linalg.det(V @ U.T)) if reflection_fix else 1.0
    R = V @ np.diag([1.0, 1.0, d]) @ U.T
    return R, cy - R @ cx


def paper_pose(x, y, w=None, inlier_ratio=0.8, reflection_fix=True):
    """Paper Sec. 3.5: weighted Kabsch, then reject the (1 - inlier_ratio) share of pairs with
    the largest residual |R x + t - y| (ties: the lower index is kept) and solve again on the
    rest.  inlier_ratio >= 1: one solve.  -> R, t, kept indices."""
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    n = x.shape[1]
    w = np.ones(n) if w is None else np.asarray(w, np.float64)
    R, t = weighted_rigid_transform(x, y, w, reflection_fix)
    m = int(inlier_ratio * n)
    if m >= n:
        return R, t, np.arange(n)
    res = np.linalg.norm(R @ x + t[:, None] - y, axis=0)
    keep = np.sort(np.argsort(res, kind="stable")[:m])
    R, t = weighted_rigid_transform(x[:, keep], y[:, keep], w[keep], reflection_fix)
    return R, t, keep


def deepvcp_loss_paper(x, y, w, R_true, t_true, alpha=0.5, reflection_fix=True, inlier_ratio=1.0):
    """x, y (B, 3, n), w (B, n) or None -> (loss, R (B,3,3), t (B,3))."""
    Rs, ts, s1, s2, cnt = [], [], 0.0, 0.0, 0
    for b in range(x.shape[0]):
        R, t, _ = paper_pose(x[b], y[b], None if w is None else w[b], inlier_ratio, reflection_fix)
        ygt = R_true[b] @ x[b] + t_true[b].reshape(3, 1)
        s1 += np.abs(ygt - y[b]).sum()
        s2 += np.abs(ygt - (R @ x[b] + t.reshape(3, 1))).sum()
        cnt += x[b].size
        Rs.append(R)
        ts.append(t)
    return alpha * s1 / cnt + (1 - alpha) * s2 / cnt, np.stack(Rs), np.stack(ts)


def _kabsch_torch(x, y, w, reflection_fix=True):
    """Differentiable weighted Kabsch on (3, n) fp64 tensors (torch.linalg.svd's backward)."""
    W = w.sum()
    cx = (x * w).sum(1) / W
    cy = (y * w).sum(1) / W
    H = ((x - cx[:, None]) * w) @ (y - cy[:, None]).T
    U, S, Vh = torch.linalg.svd(H)
    V = Vh.T
    d = torch.sign(torch.det(V @ U.T)).detach() if reflection_fix else torch.ones((), dtype=x.dtype)
    D = torch.diag(torch.stack([torch.ones((), dtype=x.dtype), torch.ones((), dtype=x.dtype), d]))
    R = V @ D @ U.T
    return R, cy - R @ cx


def deepvcp_loss_paper_torch(x, y, w, R_true, t_true, alpha=0.5, reflection_fix=True, inlier_ratio=0.8):
    """The paper loss in torch fp64 (autograd in y and w: the backward's checker).  x, y (B, 3, n),
    w (B, n).  The rejection's selection carries no gradient; the second solve does."""
    losses1, losses2, Rs, ts = [], [], [], []
    B, _, n = x.shape
    for b in range(B):
        R1, t1 = _kabsch_torch(x[b], y[b], w[b], reflection_fix)
        m = int(inlier_ratio * n)
        if m < n:
            res = torch.linalg.norm(R1 @ x[b] + t1[:, None] - y[b], dim=0).detach().numpy()
            keep = torch.from_numpy(np.sort(np.argsort(res, kind="stable")[:m]))
            R, t = _kabsch_torch(x[b][:, keep], y[b][:, keep], w[b][keep], reflection_fix)
        else:
            R, t = R1, t1
        ygt = R_true[b] @ x[b] + t_true[b].reshape(3, 1)
        losses1.append((ygt - y[b]).abs().sum())
        losses2.append((ygt - (R @ x[b] + t[:, None])).abs().sum())
        Rs.append(R)
        ts.append(t)
    cnt = float(B * 3 * n)
    loss = alpha * torch.stack(losses1).sum() / cnt + (1 - alpha) * torch.stack(losses2).sum() / cnt
    return loss, torch.stack(Rs), torch.stack(ts)


# ------------------------------------------------------------------------ feature propagation
class PointNetFeaturePropagation(nn.Module):
    """pointnet2_utils.py:265-315 (the reference defines it but never calls it): 3-NN inverse-
    distance interpolation of points2 (at xyz2) onto xyz1 with square_distance (expansion form)
    and a sort, concatenation with points1, then [Conv1d 1x1, BN1d, ReLU] per MLP layer."""

    def __init__(self, in_channel, mlp):
        super().__init__()
        self.mlp_convs = nn.ModuleList()
        self.mlp_bns = nn.ModuleList()
        last = in_channel
        for out in mlp:
            self.mlp_convs.append(nn.Conv1d(last, out, 1))
            self.mlp_bns.append(nn.BatchNorm1d(out))
            last = out

    def forward(self, xyz1, xyz2, points1, points2):
        xyz1 = xyz1.permute(0, 2, 1)
        xyz2 = xyz2.permute(0, 2, 1)
        points2 = points2.permute(0, 2, 1)
        B, N, C = xyz1.shape
        _, S, _ = xyz2.shape
        if S == 1:
            interpolated = points2.repeat(1, N, 1)
        else:
            dists = R_.square_distance(xyz1, xyz2)
            dists, idx = dists.sort(dim=-1, stable=True)       # ties: the lower index first
            dists, idx = dists[:, :, :3], idx[:, :, :3]
            dist_recip = 1.0 / (dists + 1e-8)
            norm = torch.sum(dist_recip, dim=2, keepdim=True)
            weight = dist_recip / norm
            interpolated = torch.sum(R_.index_points(points2, idx) * weight.view(B, N, 3, 1), dim=2)
        if points1 is not None:
            new_points = torch.cat([points1.permute(0, 2, 1), interpolated], dim=-1)
        else:
            new_points = interpolated
        new_points = new_points.permute(0, 2, 1)
        for conv, bn in zip(self.mlp_convs, self.mlp_bns):
            new_points = F.relu(bn(conv(new_points.float())))
        return new_points


def paper_fe_config(use_normal=False, npoints=(4096, 1024, 256), radii=(0.1, 0.2, 0.4), nsample=32):
    """Supplement Sec. 1: SA 4096 / 1024 / 256 samples with MLPs 32-32, 32-64, 64-64; FP MLPs
    64-64, 32-32, 32-32-32; then a 32-unit fully connected layer."""
    d0 = 3 if use_normal else 0
    sa = [dict(npoint=npoints[0], radius=radii[0], nsample=nsample, in_channel=3 + d0, mlp=[32, 32]),
          dict(npoint=npoints[1], radius=radii[1], nsample=nsample, in_channel=32 + 3, mlp=[32, 64]),
          dict(npoint=npoints[2], radius=radii[2], nsample=nsample, in_channel=64 + 3, mlp=[64, 64])]
    fp = [dict(in_channel=64 + 64, mlp=[64, 64]), dict(in_channel=32 + 64, mlp=[32, 32]),
          dict(in_channel=d0 + 32, mlp=[32, 32, 32])]
    return sa, fp


class PaperFeatExtraction(nn.Module):
    """Per-point features (B, N, 32) for every input point (paper Sec. 3.1)."""

    def __init__(self, use_normal=False, **cfg):
        super().__init__()
        self.use_normal = use_normal
        sa, fp = paper_fe_config(use_normal, **cfg)
        self.sa1, self.sa2, self.sa3 = (R_.PointNetSetAbstraction(**c) for c in sa)
        self.fp3, self.fp2, self.fp1 = (PointNetFeaturePropagation(**c) for c in fp)
        self.fc = nn.Linear(32, 32)

    def forward(self, pts):
        l0_xyz = pts[:, :3, :]
        l0_pts = pts[:, 3:, :] if self.use_normal else None
        l1_xyz, l1_pts = self.sa1(l0_xyz, l0_pts)
        l2_xyz, l2_pts = self.sa2(l1_xyz, l1_pts)
        l3_xyz, l3_pts = self.sa3(l2_xyz, l2_pts)
        l2_pts = self.fp3(l2_xyz, l3_xyz, l2_pts, l3_pts)
        l1_pts = self.fp2(l1_xyz, l2_xyz, l1_pts, l2_pts)
        l0 = self.fp1(l0_xyz, l1_xyz, l0_pts.float() if l0_pts is not None else None, l1_pts)
        return self.fc(l0.permute(0, 2, 1))               # dropout (keep 0.7) is identity in eval


class PaperWeighting(nn.Module):
    """Paper Sec. 3.2: FC 16 (BN, ReLU), FC 8 (BN, ReLU), FC 1 softplus."""

    def __init__(self):
        super().__init__()
        self.fc1, self.bn1 = nn.Linear(32, 16), nn.BatchNorm1d(16)
        self.fc2, self.bn2 = nn.Linear(16, 8), nn.BatchNorm1d(8)
        self.fc3 = nn.Linear(8, 1)

    def forward(self, f):                                  # (B, N, 32) -> (B, N)
        B, N, _ = f.shape
        h = F.relu(self.bn1(self.fc1(f.reshape(B * N, 32))))
        h = F.relu(self.bn2(self.fc2(h)))
        return F.softplus(self.fc3(h)).view(B, N)


def group_rows(centres, xyz, feats, radius, nsample):
    """Sec. 3.3 neighbourhoods: the first nsample points (ascending index) within radius of each
    centre (query_ball_point, pointnet2_utils.py:87-107, padded with the first hit), rows
    [(p - c) / radius, f(p)] -> (B, Q, nsample, 3 + D).  A centre with no point in range gets
    all-zero rows."""
    B, Q, _ = centres.shape
    N = xyz.shape[1]
    ns = min(nsample, N)
    g = R_.query_ball_point(radius, ns, xyz, centres)               # (B, Q, ns), N where empty
    empty = g[:, :, :1] >= N
    gi = torch.where(g >= N, torch.zeros_like(g), g)
    local = (R_.index_points(xyz, gi) - centres[:, :, None, :]) / radius
    rows = torch.cat([local.float(), R_.index_points(feats, gi).float()], -1)
    rows = torch.where(empty[..., None], torch.zeros_like(rows), rows)
    if ns < nsample:
        rows = torch.cat([rows, rows[:, :, :1].expand(B, Q, nsample - ns, rows.shape[-1])], 2)
    return rows


def centred_grid(G, s, dtype=torch.float64):
    ax = (torch.arange(G, dtype=dtype) - (G - 1) / 2.0) * s
    return torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)


class CPG1D(nn.Module):
    """Sec. 3.6 duplication: the back network's CPG, a 1-D CNN over the Gz candidates along z
    (Conv1d 32-16-4-1, k 3, p 1, no activations, like cpg.py's 3-D chain), softmax over them and
    the weighted candidate sum (cpg.py:53-58)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv1d(32, 16, 3, padding=1)
        self.conv2 = nn.Conv1d(16, 4, 3, padding=1)
        self.conv3 = nn.Conv1d(4, 1, 3, padding=1)

    def forward(self, src, tgt, cand):
        """src (B, K, 32), tgt (B, K, Gz, 32), cand (B, K, Gz, 3) -> vcp (B, K, 3)."""
        B, K, Gz, _ = tgt.shape
        cost = (src[:, :, None, :] - tgt) ** 2                          # (B, K, Gz, 32)
        x = cost.reshape(B * K, Gz, 32).permute(0, 2, 1)
        x = self.conv3(self.conv2(self.conv1(x))).reshape(B, K, Gz)
        w = F.softmax(x, dim=2)
        return torch.sum(w[..., None] * cand, 2) / torch.sum(w, 2)[..., None]


class _Stage(nn.Module):
    """One network of the cascade: weighting layer, DFE and a CPG (3-D or the 1-D z line)."""

    def __init__(self, one_d):
        super().__init__()
        self.WL = PaperWeighting()
        self.DFE = R_.feat_embedding_layer()
        self.cpg = CPG1D() if one_d else R_.cpg()
        self.one_d = one_d


class DeepVCPPaper(nn.Module):
    """Paper-faithful DeepVCP with duplication (Sec. 3, 3.6): shared per-point FE; stage 1 =
    weighting + top-K, DFE on radius-d neighbourhoods, a centred (2r/s+1)^3 candidate grid around
    the key points moved by (R_init, t_init), 3-D CPG, pose with rejection; stage 2 (the same with
    its own weights) is moved by stage 1's pose and generates candidates on a z line of
    2r/s_z + 1 points with the 1-D CPG.  forward -> list of per-stage dicts (keypts, vcp, weights,
    R, t)."""

    def __init__(self, use_normal=False, K=64, r=2.0, s=0.4, s_z=0.25, d=1.0, nsample=32, duplication=True,
                 inlier_ratio=0.8, **fe_cfg):
        super().__init__()
        self.FE = PaperFeatExtraction(use_normal, **fe_cfg)
        self.stages = nn.ModuleList([_Stage(False)] + ([_Stage(True)] if duplication else []))
        self.K, self.r, self.s, self.s_z, self.d, self.ns = K, r, s, s_z, d, nsample
        self.inlier_ratio = inlier_ratio

    def forward(self, src, tgt, R_init, t_init):
        B = src.shape[0]
        f_src, f_tgt = self.FE(src), self.FE(tgt)
        xs, xt = src[:, :3].permute(0, 2, 1), tgt[:, :3].permute(0, 2, 1)
        Rc, tc = R_init.double().expand(B, 3, 3), t_init.double().reshape(-1, 3).expand(B, 3)
        out = []
        for st in self.stages:
            score = st.WL(f_src)
            w, top = torch.topk(score, self.K, dim=1)
            kp = R_.index_points(xs, top)                                  # (B, K, 3)
            rows = group_rows(kp, xs, f_src, self.d, self.ns)
            src_dfe = st.DFE(rows, src=True)                               # (B, K, 32)
            moved = torch.einsum("bij,bkj->bki", Rc, kp.double()) + tc[:, None, :]
            if st.one_d:
                G = int(2 * self.r / self.s_z + 1)
                ax = (torch.arange(G, dtype=torch.float64) - (G - 1) / 2.0) * self.s_z
                off = torch.zeros(G, 3, dtype=torch.float64)
                off[:, 2] = ax
            else:
                G = int(2 * self.r / self.s + 1)
                off = centred_grid(G, self.s)
            cand = (moved[:, :, None, :] + off[None, None]).float()        # (B, K, C, 3)
            C = cand.shape[2]
            trows = group_rows(cand.reshape(B, self.K * C, 3), xt, f_tgt, self.d, self.ns)
            tgt_dfe = st.DFE(trows.reshape(B, self.K, C, self.ns, -1), src=False)  # (B, K, C, 32)
            if st.one_d:
                vcp = st.cpg(src_dfe, tgt_dfe, cand)
            else:
                # the reference cpg's reshape (cpg.py:34) of a (B, K, 32, C) view whose row-major
                # order is the candidates' own: the 3-D grid without the Q11 scramble
                vcp = st.cpg(src_dfe.unsqueeze(2), tgt_dfe.contiguous().view(B, self.K, 32, C), cand, self.r,
                             self.s)
            Rs, ts = [], []
            for b in range(B):
                Rb, tb, _ = paper_pose(kp[b].double().T.numpy(), vcp[b].double().T.numpy(),
                                       w[b].double().numpy(), self.inlier_ratio)
                Rs.append(torch.from_numpy(Rb))
                ts.append(torch.from_numpy(tb))
            Rc, tc = torch.stack(Rs), torch.stack(ts)
            out.append(dict(keypts=kp, vcp=vcp, weights=w, R=Rc, t=tc, topk=top, cand=cand, src_dfe=src_dfe,
                            tgt_dfe=tgt_dfe, score=score))
        return out
