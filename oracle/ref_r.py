"""REF-R: the reference DeepVCP forward + pose solve, restated in plain torch CPU ops.

TEST INFRASTRUCTURE ONLY -- see ``oracle/__init__.py``.  PARITY UNPINNED: the
reference holds no golden vectors and could not be imported here; this module is
pinned by the hand KATs in ``tests/test_oracle_kat.py``.

Every function names the reference file:line it restates.  The same torch ops run
in the same order as the reference so dtype promotion, BLAS rounding and
tie-breaking are inherited rather than re-derived.  Deviations are only the crash
repairs of SURVEY.md Appendix A.2:

  R1  FE chains sa1 -> sa2 -> sa3 on the previous layer's features and applies
      ``fc`` (deep_feat_extraction.py:26-32); sa2/sa3 in_channel = 35 / 67.
  R2  key points are gathered from the FE xyz with the FE-space top-k indices
      (deepVCP.py:44-46).
  R3  R_init is used as-is when it already has B rows (deepVCP.py:87).
  R4  per-batch gather in Get_Cat_Feat_Tgt (get_cat_feat_tgt.py:78-88).
  R5  kNN reference set = target FE xyz (get_cat_feat_tgt.py:50-52,85).
  R6  ``knn_cuda.KNN`` -> :class:`KNN` below (exact brute force, contract in
      SURVEY.md 8(c)): fp32 d2 = (dx*dx + dy*dy) + dz*dz, ascending, ties to the
      lower index, dist = sqrt(d2), 0-based int64 idx.
  R7  K, r, s are parameters (defaults reproduce the literals K=64, r=1, s=0.4).
  R8  voxelize.py:23 ``.view(-1, 3)`` -> ``.reshape(-1, 3)`` (the permuted key
      points from deepVCP.py:91 are non-contiguous, so ``view`` raises for B>1).
  R9  query_ball_point pads with ``gidx.shape[2]`` columns of the first hit instead of
      ``nsample`` (pointnet2_utils.py:104 repeats to nsample).  The two agree whenever
      nsample <= N; for nsample > N (the key-point grouping with K < 32, deepVCP.py:54,
      or tiny test clouds) the reference's mask ``group_idx == N`` has N columns while
      the repeated head has nsample, and the boolean index raises.  The repair keeps
      the first min(nsample, N) slots, i.e. the rows the reference would have
      produced had the shapes matched.

The optional ``chunk`` arguments only bound peak memory (row blocks of the same
ops); results are row-independent.
"""
import math
from contextlib import contextmanager

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "square_distance", "index_points", "farthest_point_sample", "query_ball_point",
    "sample_and_group", "PointNetSetAbstraction", "feat_extraction_layer",
    "weighting_layer", "Get_Cat_Feat_Src", "Get_Cat_Feat_Tgt", "voxelize",
    "voxelize_point", "feat_embedding_layer", "cpg", "DeepVCP", "KNN",
    "get_rigid_transform", "svd_optimization", "deepVCP_loss", "tracing", "fps_starts",
    "fe_config", "registration_errors",
]

# ---------------------------------------------------------------------------
# stage tracing (oracle-only): intermediate outputs recorded for the
# stage-decoupled GPU parity tests.
_TRACE = None


@contextmanager
def tracing():
    """Record intermediate stage outputs into a list of (name, tensor) pairs."""
    global _TRACE
    prev, _TRACE = _TRACE, []
    try:
        yield _TRACE
    finally:
        _TRACE = prev


# Optional injected FPS start indices (oracle-only): when set, farthest_point_sample pops its
# start from this list instead of drawing from the CPU generator, so the oracle can replay the
# exact starts a GPU run used.  None = draw like the reference (pointnet2_utils.py:75).
_START_QUEUE = None


@contextmanager
def fps_starts(starts):
    """Replay the given (calls, B) start indices in call order."""
    global _START_QUEUE
    prev, _START_QUEUE = _START_QUEUE, [s for s in starts]
    try:
        yield
    finally:
        _START_QUEUE = prev


def _rec(name, value):
    if _TRACE is not None:
        _TRACE.append((name, value.detach().clone() if torch.is_tensor(value) else value))


# ---------------------------------------------------------------------------
# L1 geometric primitives -- pointnet2_utils.py

def square_distance(src, dst):
    """pointnet2_utils.py:19-40.  Expansion form in this order:
    (-2 * src @ dst^T) + |src|^2 + |dst|^2  (the matmul is BLAS-rounded)."""
    nb, ns, _ = src.shape
    nd = dst.shape[1]
    out = -2 * torch.matmul(src, dst.permute(0, 2, 1))
    out += torch.sum(src ** 2, -1).view(nb, ns, 1)
    out += torch.sum(dst ** 2, -1).view(nb, 1, nd)
    return out


def index_points(points, idx):
    """pointnet2_utils.py:43-60: out[b, ...] = points[b, idx[b, ...], :]."""
    nb = points.shape[0]
    shape = [nb] + [1] * (idx.dim() - 1)
    rep = [1] + list(idx.shape[1:])
    bidx = torch.arange(nb, dtype=torch.long).view(shape).repeat(rep)
    return points[bidx, idx, :]


def farthest_point_sample(xyz, npoint, start=None):
    """pointnet2_utils.py:63-84.

    The running minimum lives in the default dtype (fp32) even for fp64 xyz
    (:74,:82); the update is a strict ``<`` (:81); argmax takes the first index
    of the maximum (:83).  The start index is drawn from the *CPU* generator
    exactly as the reference does (:75) unless ``start`` is given.
    """
    nb, n, _ = xyz.shape
    chosen = torch.zeros(nb, npoint, dtype=torch.long)
    running = torch.ones(nb, n) * 1e10
    if start is None and _START_QUEUE:
        start = _START_QUEUE.pop(0)
    if start is None:
        cur = torch.randint(0, n, (nb,), dtype=torch.long)
    else:
        cur = start.clone().long()
    rows = torch.arange(nb, dtype=torch.long)
    for step in range(npoint):
        chosen[:, step] = cur
        centre = xyz[rows, cur, :].view(nb, 1, 3)
        d = torch.sum((xyz - centre) ** 2, -1)
        upd = d < running
        running[upd] = d[upd].float()
        cur = torch.max(running, -1)[1]
    return chosen


def query_ball_point(radius, nsample, xyz, new_xyz, chunk=2048):
    """pointnet2_utils.py:87-107: first ``nsample`` ascending indices whose
    expansion-form d2 is not ``> radius**2``, padded with the first hit."""
    nb, n, _ = xyz.shape
    s_total = new_xyz.shape[1]
    parts = []
    for s0 in range(0, s_total, chunk):
        ctr = new_xyz[:, s0:s0 + chunk, :]
        s = ctr.shape[1]
        gidx = torch.arange(n, dtype=torch.long).view(1, 1, n).repeat([nb, s, 1])
        d2 = square_distance(ctr, xyz)
        gidx[d2 > radius ** 2] = n
        gidx = gidx.sort(dim=-1)[0][:, :, :nsample]
        # R9: pad to the sliced width (= nsample unless nsample > N, where :104 raises)
        head = gidx[:, :, 0].view(nb, s, 1).repeat([1, 1, gidx.shape[2]])
        miss = gidx == n
        gidx[miss] = head[miss]
        parts.append(gidx)
        del d2
    return torch.cat(parts, dim=1)


def sample_and_group(npoint, radius, nsample, xyz, points, returnidx=False, start=None):
    """pointnet2_utils.py:110-138."""
    nb, _, c = xyz.shape
    fidx = farthest_point_sample(xyz, npoint, start=start)
    _rec("fps_idx", fidx)
    centres = index_points(xyz, fidx)
    gidx = query_ball_point(radius, nsample, xyz, centres)
    _rec("ball_idx", gidx)
    local = index_points(xyz, gidx) - centres.view(nb, npoint, 1, c)
    if points is not None:
        grouped = torch.cat([local, index_points(points, gidx)], dim=-1)
    else:
        grouped = local
    if returnidx:
        return centres, grouped, gidx
    return centres, grouped


class PointNetSetAbstraction(nn.Module):
    """pointnet2_utils.py:161-202 (group_all=False path; the only one the
    forward uses, deep_feat_extraction.py:10-13)."""

    def __init__(self, npoint, radius, nsample, in_channel, mlp, group_all=False):
        super().__init__()
        self.npoint, self.radius, self.nsample = npoint, radius, nsample
        self.mlp_convs = nn.ModuleList()
        self.mlp_bns = nn.ModuleList()
        last = in_channel
        for width in mlp:
            self.mlp_convs.append(nn.Conv2d(last, width, 1))
            self.mlp_bns.append(nn.BatchNorm2d(width))
            last = width
        assert not group_all
        self.group_all = group_all

    def forward(self, xyz, points):
        xyz = xyz.permute(0, 2, 1)
        if points is not None:
            points = points.permute(0, 2, 1)
        centres, grouped = sample_and_group(self.npoint, self.radius, self.nsample, xyz, points)
        x = grouped.permute(0, 3, 2, 1)                      # (B, C+D, ns, S)  :195
        for conv, bn in zip(self.mlp_convs, self.mlp_bns):
            x = F.relu(bn(conv(x.float())))                  # :198
        x = torch.max(x, 2)[0]                               # :200
        _rec("sa_out", x)
        return centres.permute(0, 2, 1), x


def fe_config(use_normal=True, npoint=10000):
    """SA table of deep_feat_extraction.py:10-13 (+R1 channel repair).
    ``npoint`` defaults to the literal 10000 (Q1); smaller values only serve
    fast tests."""
    c_in = 6 if use_normal else 3
    return [
        dict(npoint=npoint, radius=0.1, nsample=256, in_channel=c_in, mlp=[16, 16, 32]),
        dict(npoint=npoint, radius=0.2, nsample=128, in_channel=32 + 3, mlp=[32, 64]),
        dict(npoint=npoint, radius=0.4, nsample=64, in_channel=64 + 3, mlp=[64, 64]),
    ]


class feat_extraction_layer(nn.Module):
    """deep_feat_extraction.py:5-32 with R1: sa2/sa3 consume the previous
    layer's (xyz, features) and ``fc`` maps 64 -> 32."""

    def __init__(self, use_normal=True, npoint=10000):
        super().__init__()
        self.use_normal = use_normal
        cfg = fe_config(use_normal, npoint)
        self.sa1 = PointNetSetAbstraction(**cfg[0])
        self.sa2 = PointNetSetAbstraction(**cfg[1])
        self.sa3 = PointNetSetAbstraction(**cfg[2])
        self.fc = nn.Linear(64, 32)

    def forward(self, pts):
        if self.use_normal:
            xyz, feat = pts[:, :3, :], pts[:, 3:, :]
        else:
            xyz, feat = pts, None
        xyz, feat = self.sa1(xyz, feat)
        xyz, feat = self.sa2(xyz, feat)
        xyz, feat = self.sa3(xyz, feat)
        out_xyz = xyz.permute(0, 2, 1)
        out_feat = self.fc(feat.permute(0, 2, 1))
        _rec("fe_xyz", out_xyz)
        _rec("fe_feat", out_feat)
        return out_xyz, out_feat


class weighting_layer(nn.Module):
    """weighting_layer.py:8-33: Linear 32-16-8-1 (ReLU, ReLU, Softplus), then
    top-k (sorted, descending) over dim 1, flattened to (B*K,)."""

    def __init__(self):
        super().__init__()
        self.fc1 = nn.Sequential(nn.Linear(32, 16, True), nn.ReLU())
        self.fc2 = nn.Sequential(nn.Linear(16, 8, True), nn.ReLU())
        self.fc3 = nn.Sequential(nn.Linear(8, 1, True), nn.Softplus())

    def forward(self, X, K=64):
        score = self.fc3(self.fc2(self.fc1(X)))
        _rec("wl_score", score)
        return torch.topk(score, K, dim=1).indices.flatten()


class Get_Cat_Feat_Src(nn.Module):
    """get_cat_feat_src.py:16-55 (prints removed).  Quirk Q5: the distance
    compares the absolute key point with the *local* grouped coordinates."""

    def forward(self, src_keypts, src_keypts_grouped_pts, src_keyfeats):
        nb, nk, ns, nf = src_keyfeats.shape
        kp = src_keypts[:, :, :3].unsqueeze(2).repeat(1, 1, ns, 1)
        pd = nn.PairwiseDistance(p=2, keepdim=True)
        dist = pd(torch.flatten(kp, 0, 2), torch.flatten(src_keypts_grouped_pts[:, :, :, :3], 0, 2))
        dist = dist.view(nb, nk, ns, 1)
        wnorm = dist / torch.sum(dist, dim=2, keepdim=True)
        wnorm = wnorm.view(nb, nk, ns).unsqueeze(3).repeat(1, 1, 1, nf)
        local = src_keypts_grouped_pts[:, :, :, :3] - kp
        return torch.cat((local, src_keyfeats * wnorm), dim=3)


def _knn_rows(ref, qry, k, chunk=2048):
    """Exact kNN (R6 contract): ref (M,3) f32, qry (Q,3) f32 -> (Q,k) dist, idx."""
    m = ref.shape[0]
    ar = torch.arange(m, dtype=torch.int64)
    dists, idxs = [], []
    for q0 in range(0, qry.shape[0], chunk):
        q = qry[q0:q0 + chunk]
        diff = ref.unsqueeze(0) - q.unsqueeze(1)                     # (Qc, M, 3)
        d2 = (diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]) + diff[..., 2] * diff[..., 2]
        key = d2.contiguous().view(torch.int32).to(torch.int64) * (1 << 32) + ar
        best = torch.topk(key, k, dim=1, largest=False, sorted=True).values
        sel = best & 0xFFFFFFFF
        # correctly rounded sqrt (the contract; knn_cuda's CUDA sqrtf is IEEE): torch's fp32
        # CPU sqrt is up to 1 ulp off, its fp64 sqrt narrowed to fp32 is exact
        dists.append(torch.sqrt(torch.gather(d2, 1, sel).double()).float())
        idxs.append(sel)
    return torch.cat(dists, 0), torch.cat(idxs, 0)


class KNN:
    """Stand-in for the un-vendored ``knn_cuda.KNN`` (R6).  Same call surface as
    get_cat_feat_tgt.py:45,52 and deepVCP_loss.py:70,72: ``KNN(k, transpose_mode)
    (ref, query) -> (dist, idx)``; transpose_mode=True takes (B, M, D)/(B, Q, D)
    and returns (B, Q, k); False takes (B, D, M)/(B, D, Q) and returns (B, k, Q).
    Inputs are cast to fp32 and evaluated under no_grad, per batch."""

    def __init__(self, k, transpose_mode=False):
        self.k = k
        self.transpose_mode = transpose_mode

    def __call__(self, ref, query):
        assert ref.size(0) == query.size(0)
        with torch.no_grad():
            ds, ix = [], []
            for b in range(ref.size(0)):
                r = ref[b] if self.transpose_mode else ref[b].t()
                q = query[b] if self.transpose_mode else query[b].t()
                d, i = _knn_rows(r.float().contiguous(), q.float().contiguous(), self.k)
                if not self.transpose_mode:
                    d, i = d.t(), i.t()
                ds.append(d)
                ix.append(i)
            return torch.stack(ds, 0), torch.stack(ix, 0)


class Get_Cat_Feat_Tgt(nn.Module):
    """get_cat_feat_tgt.py:18-98 with R4 (per-batch gather) and R5 (the kNN
    reference set is the FE xyz).  Quirk Q10: the normalised distance weight
    is indexed by the feature channel."""

    def forward(self, candidate_pts, src_keypts, tgt_pts_xyz, tgt_deep_feat_pts):
        nb = src_keypts.shape[0]
        k_nn = 32
        qry = torch.flatten(candidate_pts, 1, 2)
        dist, idx = KNN(k=k_nn, transpose_mode=True)(tgt_pts_xyz, qry)
        _rec("knn_dist", dist)
        _rec("knn_idx", idx)
        cand_rep = candidate_pts.unsqueeze(3).repeat(1, 1, 1, k_nn, 1)
        dsum = torch.sum(dist, dim=2, keepdim=True, dtype=float)
        wnorm = dist / dsum
        wmap = wnorm.unsqueeze(2).repeat(1, 1, k_nn, 1)
        nk, nc, nf = src_keypts.shape[1], candidate_pts.shape[2], tgt_deep_feat_pts.shape[2]
        bsel = torch.arange(nb).view(nb, 1, 1).expand(nb, idx.shape[1], k_nn).flatten()
        isel = idx.flatten()
        feat_sel = tgt_deep_feat_pts[bsel, isel, :].view(nb, nk, nc, k_nn, nf)
        pts_sel = tgt_pts_xyz[bsel, isel, :].view(nb, nk, nc, k_nn, 3)
        local = pts_sel - cand_rep
        wmap = wmap.view(nb, nk, nc, k_nn, nf)
        return torch.cat((local, feat_sel * wmap), dim=4)


def voxelize_point(point, search_radius, voxel_len):
    """voxelize.py:44-83, literal: bbox from a cartesian product, per-axis
    ``torch.arange(min - s/2, max, s)`` (default fp32 values, accumulated in
    double), meshgrid 'ij', no sphere rejection (Q9)."""
    cx, cy, cz = point
    tx = torch.tensor([cx - search_radius, cx + search_radius])
    ty = torch.tensor([cy - search_radius, cy + search_radius])
    tz = torch.tensor([cz - search_radius, cz + search_radius])
    corners = torch.cartesian_prod(tx, ty, tz)
    lo = torch.min(corners, axis=0)
    hi = torch.max(corners, axis=0)
    axes = [torch.arange(lo.values[a] - voxel_len / 2, hi.values[a], voxel_len) for a in range(3)]
    gx, gy, gz = torch.meshgrid(axes[0], axes[1], axes[2], indexing="ij")
    grid = torch.stack((gx, gy, gz), axis=-1)
    return torch.stack([row for row in grid.reshape(-1, grid.shape[-1])])


def voxelize(point_clouds, r, s):
    """voxelize.py:19-29: (B, N, 3) -> (B, N, C, 3)."""
    nb, n, _ = point_clouds.shape
    # R8: the reference's ``.view(-1, 3)`` (voxelize.py:23) raises for B>1 on the
    # non-contiguous permuted key points (deepVCP.py:91); reshape gives the same rows.
    out = torch.stack([voxelize_point(p, r, s) for p in point_clouds.reshape(-1, 3)])
    return torch.reshape(out, (nb, n, -1, 3))


class feat_embedding_layer(nn.Module):
    """deep_feat_embedding.py:13-61: Linear 35-32-32-32 with no nonlinearity
    (Q14), MaxPool1d(32) over the neighbour axis."""

    def __init__(self, K_nsample=32):
        super().__init__()
        self.K_nsample = 32
        self.fc1 = nn.Linear(35, 32, True)
        self.fc2 = nn.Linear(32, 32, True)
        self.fc3 = nn.Linear(32, 32, True)
        self.max_pool = nn.MaxPool1d(kernel_size=self.K_nsample)

    def forward(self, X, src=True, chunk=None):
        X = X.float()
        if src:
            nb, nk, _, _ = X.shape
            X = self.fc3(self.fc2(self.fc1(X)))
            X = torch.flatten(X.permute(0, 1, 3, 2), 1, 2)
            return self.max_pool(X).view(nb, nk, 32, 1).squeeze(3)
        nb, nk, nc, _, _ = X.shape
        X = self.fc3(self.fc2(self.fc1(X)))
        X = torch.flatten(X.permute(0, 1, 2, 4, 3), 1, 3)
        return self.max_pool(X).view(nb, nk, nc, 32, 1).squeeze(4)


class cpg(nn.Module):
    """cpg.py:14-60: cost volume (src - scrambled tgt)^2 (Q11), Conv3d
    32-16-4-1 (k3, p1, no activations), softmax over C, weighted mean."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv3d(32, 16, kernel_size=3, stride=1, padding=1)
        self.conv2 = nn.Conv3d(16, 4, kernel_size=3, stride=1, padding=1)
        self.conv3 = nn.Conv3d(4, 1, kernel_size=3, stride=1, padding=1)
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, src_dfe_feat, tgt_dfe_feat, candidates, r, s):
        nb, nk, nc, _ = candidates.shape
        g = int((2 * r) / s + 1)
        assert nc == g * g * g
        src_vol = src_dfe_feat.reshape(nb, nk, 1, 1, 1, 32).repeat(1, 1, g, g, g, 1)
        tgt_vol = tgt_dfe_feat.reshape(nb, nk, g, g, g, 32)
        cost = torch.square(src_vol - tgt_vol)
        x = cost.permute(0, 1, 5, 2, 3, 4).flatten(start_dim=0, end_dim=1)
        x = self.conv3(self.conv2(self.conv1(x)))
        w = self.softmax(x.reshape(nb, nk, nc))
        _rec("cpg_weight", w)
        w = w.unsqueeze(-1).repeat(1, 1, 1, 3)
        vcp = torch.sum(torch.mul(w, candidates), -2)
        vcp /= torch.sum(w, -2)
        return vcp


class DeepVCP(nn.Module):
    """deepVCP.py:16-110 with R2, R3, R5, R7; prints/timers removed."""

    def __init__(self, use_normal, K=64, r=1.0, s=0.4, fe_npoint=10000):
        super().__init__()
        self.FE1 = feat_extraction_layer(use_normal=use_normal, npoint=fe_npoint)
        self.WL = weighting_layer()
        self.DFE = feat_embedding_layer()
        self.cpg = cpg()
        self.K, self.r, self.s = K, r, s

    def forward(self, src_pts, tgt_pts, R_init, t_init):
        nb = src_pts.shape[0]
        K, r, s = self.K, self.r, self.s
        src_xyz, src_feat = self.FE1(src_pts)
        top = self.WL(src_feat, K)
        _rec("topk_idx", top.view(nb, K))
        src_keypts = index_points(src_xyz, top.view(nb, K))                 # R2
        _rec("keypts", src_keypts)
        _, g_local, picked = sample_and_group(npoint=K, radius=1, nsample=32,
                                              xyz=src_keypts[:, :, :3], points=None,
                                              returnidx=True)
        src_cat = Get_Cat_Feat_Src()(src_keypts, g_local, index_points(src_feat, picked))
        _rec("src_cat", src_cat)
        tgt_xyz, tgt_feat = self.FE1(tgt_pts)
        R_rep = R_init if R_init.shape[0] == nb else R_init.repeat(nb, 1, 1)  # R3
        kT = src_keypts.permute(0, 2, 1)[:, :3, :]
        moved = torch.matmul(R_rep, kT.double()).permute(0, 2, 1)
        _rec("moved", moved)
        cand = voxelize(moved, r, s)
        _rec("candidates", cand)
        tgt_cat = Get_Cat_Feat_Tgt()(cand, src_keypts, tgt_xyz, tgt_feat)  # R5
        src_dfe = self.DFE(src_cat, src=True)
        tgt_dfe = self.DFE(tgt_cat, src=False)
        del tgt_cat
        _rec("src_dfe", src_dfe)
        _rec("tgt_dfe", tgt_dfe)
        vcp = self.cpg(src_dfe.unsqueeze(2), tgt_dfe.permute(0, 1, 3, 2), cand, r, s)
        return src_keypts[:, :, :3], vcp


# ---------------------------------------------------------------------------
# L4 pose solve -- deepVCP_loss.py

def get_rigid_transform(x, y):
    """deepVCP_loss.py:13-44: Kabsch, R = V U^T with no reflection fix (Q13;
    the det/Z lines :36-40 are dead code)."""
    cx = torch.mean(x, dim=2, keepdim=True)
    cy = torch.mean(y, dim=2, keepdim=True)
    H = torch.matmul(torch.sub(x, cx), torch.sub(y, cy).permute(0, 2, 1))
    u, _, v = torch.svd(H)
    R = torch.matmul(v, u.permute(0, 2, 1))
    t = cy + torch.matmul(-R, cx)
    return R, t


def svd_optimization(x, y_pred, R_true, t_true):
    """deepVCP_loss.py:57-90: SVD, 1-NN of y_true against R1 x + t1, keep the
    int(0.8 n) closest, SVD again on (x1, R1 x1 + t1) (Q12)."""
    y_true = torch.matmul(R_true, x) + t_true
    y_pred = y_pred.double()
    n = y_pred.shape[2]
    R1, t1 = get_rigid_transform(x, y_pred)
    y1 = torch.matmul(R1, x) + t1
    d, _ = KNN(k=1, transpose_mode=False)(y1, y_true)
    keep = torch.topk(d, k=int(n * 0.8), dim=-1, largest=False, sorted=True).indices
    keep = keep.repeat(1, 3, 1)
    y1 = torch.gather(y1, dim=-1, index=keep)
    x1 = torch.gather(x, dim=-1, index=keep)
    R2, t2 = get_rigid_transform(x1, y1)
    return R2, t2, x1, torch.matmul(R2, x1) + t2


def deepVCP_loss(x, y_pred, R_true, t_true, alpha):
    """deepVCP_loss.py:105-121 (the ``Loss:`` print kept off)."""
    x = x.permute(0, 2, 1).double()
    y_pred = y_pred.permute(0, 2, 1).double()
    R, t, x_in, y_opt = svd_optimization(x, y_pred, R_true, t_true)
    y_true_in = torch.matmul(R_true, x_in) + t_true
    l2 = torch.abs(torch.mean(torch.sub(y_opt, y_true_in)))
    loss = alpha * nn.L1Loss(reduction="mean")(y_true_in, y_opt) + (1 - alpha) * l2
    return loss, R, t


def registration_errors(R_pred, t_pred, R_gt, t_gt):
    """train.py:112-120 per pair, C8 fixed (translation norm over the 3 components):
    rot_err = PairwiseDistance(euler_xyz_deg(R_pred), euler_xyz_deg(R_gt)) via scipy, trans_err =
    PairwiseDistance(t_pred, t_gt).  scipy raises for det <= 0 (Q13 reflections); NaN there."""
    import numpy as np
    from scipy.spatial.transform import Rotation
    B = R_pred.shape[0]
    Rp = R_pred.double().reshape(B, 3, 3).numpy()
    Rg = R_gt.double().reshape(-1, 3, 3).expand(B, 3, 3).numpy()
    pdist = nn.PairwiseDistance(p=2)
    rot = []
    for b in range(B):
        try:
            ep = torch.tensor(Rotation.from_matrix(Rp[b]).as_euler('xyz', degrees=True)).reshape(1, 3)
            eg = torch.tensor(Rotation.from_matrix(Rg[b]).as_euler('xyz', degrees=True)).reshape(1, 3)
            rot.append(float(pdist(ep, eg).item()))
        except ValueError:
            rot.append(float("nan"))
    tp = t_pred.double().reshape(B, 3)
    tg = t_gt.double().reshape(-1, 3).expand(B, 3)
    return torch.tensor(rot, dtype=torch.float64), pdist(tp, tg)
