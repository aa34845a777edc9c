"""Hand-derived known-answer tests pinning the CPU oracle to the reference semantics.

The reference ships no tests or golden vectors and could not be imported here (SURVEY.md 4,
8(c)), so each expected value below is derived by hand from the cited reference lines.
"""
import math

import numpy as np
import pytest
import torch

import oracle as O


def test_fps_collinear_order_and_tail():
    """pointnet2_utils.py:63-84 on x = 0..4 from index 0: distances 0,1,4,9,16 -> 4; then
    min-dists 0,1,4,1,0 -> 2; then 0,1,0,1,0 -> first max 1; then 3; all zero -> index 0."""
    xyz = torch.tensor([[[0.0, 0, 0], [1, 0, 0], [2, 0, 0], [3, 0, 0], [4, 0, 0]]])
    idx = O.farthest_point_sample(xyz, 7, start=torch.tensor([0]))
    assert idx.tolist() == [[0, 4, 2, 1, 3, 0, 0]]


def test_fps_first_index_tie_break():
    xyz = torch.tensor([[[-1.0, 0, 0], [0, 0, 0], [1, 0, 0]]])
    assert O.farthest_point_sample(xyz, 3, start=torch.tensor([1])).tolist() == [[1, 0, 2]]


def test_fps_running_min_is_fp32_for_fp64_input():
    # two fp64 distances that differ only below fp32 resolution: the fp32 running minimum
    # (pointnet2_utils.py:74,82) makes them tie, so the first index wins
    a = 1.0
    b = 1.0 + 1e-12
    xyz = torch.tensor([[[0.0, 0, 0], [a, 0, 0], [-math.sqrt(b * b), 0, 0]]], dtype=torch.float64)
    assert O.farthest_point_sample(xyz, 2, start=torch.tensor([0])).tolist() == [[0, 1]]


def test_ball_query_boundary_inclusive_and_padding():
    """:102 excludes only d2 > r^2: points at exactly r are kept; :104-106 pad with the first."""
    xyz = torch.tensor([[[0.0, 0, 0], [0.5, 0, 0], [1.0, 0, 0], [1.5, 0, 0]]])
    ctr = torch.tensor([[[0.0, 0, 0]]])
    assert O.query_ball_point(1.0, 3, xyz, ctr).tolist() == [[[0, 1, 2]]]
    assert O.query_ball_point(1.0, 5, xyz, ctr).tolist() == [[[0, 1, 2, 0]]]  # nsample > N: N columns


def test_ball_query_lowest_indices_not_nearest():
    xyz = torch.tensor([[[0.9, 0, 0], [0.8, 0, 0], [0.0, 0, 0], [0.1, 0, 0]]])
    ctr = torch.tensor([[[0.0, 0, 0]]])
    assert O.query_ball_point(1.0, 2, xyz, ctr).tolist() == [[[0, 1]]]  # Q2


def test_ball_query_no_hit_gives_N():
    xyz = torch.zeros(1, 3, 3)
    ctr = torch.full((1, 1, 3), 9.0)
    assert O.query_ball_point(1.0, 4, xyz, ctr).tolist() == [[[3, 3, 3]]]  # nsample > N -> N columns


def test_square_distance_rounds_like_mkl_fma_chain():
    g = torch.Generator().manual_seed(0)
    a, b = torch.rand(1, 64, 3, generator=g), torch.rand(1, 80, 3, generator=g)
    d = O.square_distance(a, b)[0].numpy()
    an, bn = a[0].numpy(), b[0].numpy()

    def fma(x, y, z):
        return (x.astype(np.float64) * y.astype(np.float64) + z.astype(np.float64)).astype(np.float32)

    dot = fma(an[:, None, 2], bn[None, :, 2], fma(an[:, None, 1], bn[None, :, 1], an[:, None, 0] * bn[None, :, 0]))
    ss = lambda p: (p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1]) + p[:, 2] * p[:, 2]  # noqa: E731
    want = ((np.float32(-2) * dot) + ss(an)[:, None]) + ss(bn)[None, :]
    assert np.array_equal(d, want)


def test_voxel_grid_origin_r1():
    """voxelize.py:62-77 at c = 0, r = 1, s = 0.4: axis = arange(-1.2, 1.0, 0.4) =
    {-1.2, -0.8, -0.4, 0.0, 0.4, 0.8} (offset by -s/2, Q9), C = 6^3, ix-major order."""
    cand = O.voxelize_point(torch.zeros(3, dtype=torch.float64), 1.0, 0.4)
    # torch's arange evaluates fma(step, i, start) in fp64: at i = 3 that is 1.11e-16, where the
    # unfused start + step*i would give 2.22e-16
    from fractions import Fraction
    axis = [np.float32(float(Fraction(0.4) * i + Fraction(-1.0 - 0.2))) for i in range(6)]
    assert axis[3] == np.float32(1.1102230246251565e-16)
    assert cand.shape == (216, 3) and cand.dtype == torch.float32
    np.testing.assert_array_equal(cand[:6, 2].numpy(), axis)          # iz fastest
    np.testing.assert_array_equal(cand[::36, 0].numpy(), axis)        # ix slowest
    assert abs(axis[0] + 1.2) < 1e-6


def test_voxel_grid_r2_is_11_cubed():
    cand = O.voxelize(torch.tensor([[[3.25, -1.5, 0.1]]], dtype=torch.float64), 2.0, 0.4)
    assert cand.shape == (1, 1, 1331, 3)
    assert int((2 * 2.0) / 0.4 + 1) ** 3 == 1331   # cpg.py:29-30 agrees


def test_knn_ties_go_to_lower_index():
    ref = torch.tensor([[[1.0, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]]])
    d, i = O.KNN(k=3, transpose_mode=True)(ref, torch.zeros(1, 1, 3))
    assert i.tolist() == [[[0, 1, 2]]] and d.tolist() == [[[1.0, 1.0, 1.0]]]
    d, i = O.KNN(k=2, transpose_mode=False)(ref.transpose(1, 2), torch.zeros(1, 3, 1))
    assert i.shape == (1, 2, 1) and i[0, :, 0].tolist() == [0, 1]


def test_pairwise_distance_formula():
    """get_cat_feat_src.py:36: PairwiseDistance = sqrt(fma chain of ((a - b) + 1e-6)^2)."""
    a = torch.tensor([[0.3, -0.7, 1.1]])
    b = torch.tensor([[0.1, 0.2, -0.4]])
    d = torch.nn.PairwiseDistance(p=2, keepdim=True)(a, b)
    e = ((a - b) + 1e-6).double()
    assert abs(float(d) - math.sqrt(float((e * e).sum()))) < 1e-6


def test_kabsch_exact_rotation():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, 3, 20, generator=g, dtype=torch.float64)
    c, s = math.cos(0.7), math.sin(0.7)
    R = torch.tensor([[[c, -s, 0], [s, c, 0], [0, 0, 1]]], dtype=torch.float64)
    t = torch.tensor([[[1.0], [2.0], [-3.0]]], dtype=torch.float64)
    Rg, tg = O.get_rigid_transform(x, R @ x + t)
    assert torch.allclose(Rg, R, atol=1e-12) and torch.allclose(tg, t, atol=1e-12)


def test_kabsch_no_reflection_fix():
    """Q13: deepVCP_loss.py:36-40 computes the det sign but never applies it."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(1, 3, 20, generator=g, dtype=torch.float64)
    F = torch.diag(torch.tensor([1.0, 1.0, -1.0], dtype=torch.float64))[None]
    Rg, _ = O.get_rigid_transform(x, F @ x)
    assert torch.allclose(Rg, F, atol=1e-12) and float(torch.det(Rg)) < 0


def test_inlier_count_and_refit():
    """deepVCP_loss.py:76: int(0.8 * 64) = 51 inliers; Q12: the refit uses R1 x + t1."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 3, 64, generator=g, dtype=torch.float64)
    y = x + 0.1 * torch.randn(2, 3, 64, generator=g, dtype=torch.float64)
    R2, t2, x1, y2 = O.svd_optimization(x, y, torch.eye(3, dtype=torch.float64).expand(2, 3, 3),
                                        torch.zeros(2, 3, 1, dtype=torch.float64))
    R1, t1 = O.get_rigid_transform(x, y)
    assert x1.shape == (2, 3, 51) and y2.shape == (2, 3, 51)
    assert torch.allclose(R2, R1, atol=1e-10) and torch.allclose(t2, t1, atol=1e-10)


def test_cpg_target_scramble_map():
    """Q11: cpg.py:34 reshapes the permuted (B,K,32,C) target, so volume element (g, f') is
    tgt_dfe[c = l % C, f = l // C] with l = g*32 + f'."""
    B, K, G = 1, 1, 3
    C = G ** 3
    tgt = torch.arange(C * 32, dtype=torch.float32).view(B, K, C, 32)     # value = c*32 + f
    vol = tgt.permute(0, 1, 3, 2).reshape(B, K, G, G, G, 32).reshape(C, 32)
    for g_ in range(C):
        for fp in range(32):
            l = g_ * 32 + fp
            assert vol[g_, fp] == (l % C) * 32 + l // C


def test_weighting_topk_sorted_descending():
    torch.manual_seed(0)
    wl = O.weighting_layer()
    X = torch.randn(2, 500, 32)
    idx = wl(X, K=10).view(2, 10)
    with torch.no_grad():
        s = wl.fc3(wl.fc2(wl.fc1(X)))[..., 0]
    for b in range(2):
        v = s[b, idx[b]]
        assert (v[1:] <= v[:-1]).all()
        assert torch.equal(torch.sort(idx[b]).values, torch.sort(torch.topk(s[b], 10).indices).values)


def test_e2e_shapes_and_dtypes_small():
    torch.manual_seed(0)
    m = O.DeepVCP(use_normal=True, K=32, r=1.0, s=0.4, fe_npoint=64).eval()
    g = torch.Generator().manual_seed(4)
    src = torch.rand(1, 6, 200, generator=g, dtype=torch.float64)
    with torch.no_grad():
        kp, vcp = m(src, src.clone(), torch.eye(3, dtype=torch.float64)[None], torch.zeros(1, 3))
    assert kp.shape == (1, 32, 3) and kp.dtype == torch.float64     # ModelNet: fp64 key points
    assert vcp.shape == (1, 32, 3) and vcp.dtype == torch.float32   # CPG is fp32 (A.4)


# ------------------------------------------------------------------ registration error (harness)
def test_registration_error_kat():
    """train.py:112-120 (C8 fixed): identity vs identity leaves only PairwiseDistance's eps in each
    component; Rx(10 deg) vs identity differs by 10 deg in the first Euler angle; a reflection is
    rejected by scipy (NaN)."""
    import math
    import oracle as O
    I = torch.eye(3, dtype=torch.float64)[None]
    z = torch.zeros(1, 3, 1, dtype=torch.float64)
    rot, tr = O.registration_errors(I, z, I, z)
    assert abs(rot.item() - math.sqrt(3) * 1e-6) < 1e-15 and abs(tr.item() - math.sqrt(3) * 1e-6) < 1e-15
    a = math.radians(10.0)
    Rx = torch.tensor([[1, 0, 0], [0, math.cos(a), -math.sin(a)], [0, math.sin(a), math.cos(a)]],
                      dtype=torch.float64)[None]
    t = torch.tensor([[[3.0], [4.0], [0.0]]], dtype=torch.float64)
    rot, tr = O.registration_errors(Rx, t, I, z)
    want = math.sqrt((10.0 + 1e-6) ** 2 + 2e-12)
    assert abs(rot.item() - want) < 1e-9
    assert abs(tr.item() - math.sqrt((3 + 1e-6) ** 2 + (4 + 1e-6) ** 2 + 1e-12)) < 1e-12
    refl = torch.diag(torch.tensor([1.0, 1.0, -1.0], dtype=torch.float64))[None]
    rot, _ = O.registration_errors(refl, z, I, z)
    assert math.isnan(rot.item())


def test_paper_pose_checker_kats():
    """oracle/paper.py (the checker of the paper-faithful pose solve): an exact rotation is
    recovered with any positive weights; zero weights drop points; a reflected point set gives
    det(R) = -1 without the fix and a proper rotation with it."""
    import numpy as np
    from oracle import paper as OP
    rng = np.random.default_rng(7)
    x = rng.standard_normal((3, 20))
    th = 0.7
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1.0]])
    t = np.array([0.3, -1.2, 2.0])
    y = Rz @ x + t[:, None]
    w = rng.random(20) + 0.1
    R, tt = OP.weighted_rigid_transform(x, y, w)
    assert np.allclose(R, Rz, atol=1e-12) and np.allclose(tt, t, atol=1e-12)
    y_bad = y.copy()
    y_bad[:, :5] += 10.0                              # corrupted points with zero weight
    w0 = w.copy()
    w0[:5] = 0.0
    R, tt = OP.weighted_rigid_transform(x, y_bad, w0)
    assert np.allclose(R, Rz, atol=1e-12) and np.allclose(tt, t, atol=1e-12)
    M = np.diag([1.0, 1.0, -1.0])                     # a mirror image: the unconstrained fit reflects
    R0, _ = OP.weighted_rigid_transform(x, M @ x, None, reflection_fix=False)
    R1, _ = OP.weighted_rigid_transform(x, M @ x, None, reflection_fix=True)
    assert np.isclose(np.linalg.det(R0), -1.0) and np.isclose(np.linalg.det(R1), 1.0)


def test_paper_rejection_and_fp_kats():
    """oracle/paper.py, the rest of the paper mode's checker:
    * the rejection step (Sec. 3.5): 20 % planted outliers are exactly the rejected pairs and the
      second solve recovers the exact rotation (the first, contaminated one does not);
    * feature propagation (pointnet2_utils.py:265-315): a constant field interpolates to itself,
      a point coinciding with an xyz2 point takes (to 1e-6) that point's value (weight 1/1e-8);
    * group_rows: a centre with no neighbour in range gives zero rows, fewer neighbours than
      nsample are padded with the first hit;
    * the 1-D CPG with zero conv weights scores every candidate alike: vcp = the line's mean."""
    import numpy as np
    from oracle import paper as OP
    rng = np.random.default_rng(11)
    n = 50
    x = rng.standard_normal((3, n))
    th = 1.1
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1.0]])
    t = np.array([0.5, 0.2, -0.7])
    y = Rz @ x + t[:, None]
    bad = rng.choice(n, 10, replace=False)
    y[:, bad] += rng.standard_normal((3, 10)) * 3.0
    w = rng.random(n) + 0.1
    R1, _ = OP.weighted_rigid_transform(x, y, w)
    R, tt, keep = OP.paper_pose(x, y, w, inlier_ratio=0.8)
    assert not np.allclose(R1, Rz, atol=1e-3)
    assert sorted(set(range(n)) - set(keep.tolist())) == sorted(bad.tolist())
    assert np.allclose(R, Rz, atol=1e-12) and np.allclose(tt, t, atol=1e-12)

    torch.manual_seed(0)
    fp = OP.PointNetFeaturePropagation(in_channel=4, mlp=[4]).eval()
    with torch.no_grad():
        fp.mlp_convs[0].weight.copy_(torch.eye(4)[:, :, None])
        fp.mlp_convs[0].bias.zero_()
    xyz1 = torch.rand(1, 3, 20)
    xyz2 = torch.rand(1, 3, 7)
    xyz2[0, :, 3] = xyz1[0, :, 5]
    p2 = torch.arange(28, dtype=torch.float32).view(1, 4, 7) * 0.1
    const = torch.full((1, 4, 7), 2.5)
    with torch.no_grad():
        out_c = fp(xyz1, xyz2, None, const)
        out = fp(xyz1, xyz2, None, p2)
    bn_scale = 1.0 / math.sqrt(1.0 + 1e-5)                # eval BatchNorm1d at its init
    assert torch.allclose(out_c, torch.full_like(out_c, 2.5 * bn_scale), rtol=1e-6)
    assert torch.allclose(out[0, :, 5], p2[0, :, 3] * bn_scale, rtol=1e-6, atol=1e-6)

    xyz = torch.tensor([[[0.0, 0.0, 0.0], [0.1, 0.0, 0.0], [5.0, 5.0, 5.0]]])
    feats = torch.tensor([[[1.0], [2.0], [3.0]]])
    ctr = torch.tensor([[[0.0, 0.0, 0.0], [20.0, 20.0, 20.0]]])
    rows = OP.group_rows(ctr, xyz, feats, 0.5, 4)
    assert rows.shape == (1, 2, 4, 4)
    assert torch.equal(rows[0, 1], torch.zeros(4, 4))
    assert torch.equal(rows[0, 0, :, 3], torch.tensor([1.0, 2.0, 1.0, 1.0]))
    assert torch.allclose(rows[0, 0, 1, :3], torch.tensor([0.2, 0.0, 0.0]))

    c1 = OP.CPG1D()
    with torch.no_grad():
        for c in (c1.conv1, c1.conv2, c1.conv3):
            c.weight.zero_()
            c.bias.zero_()
        cand = torch.zeros(1, 2, 9, 3)
        cand[..., 2] = torch.arange(9, dtype=torch.float32) * 0.25 - 1.0
        cand[:, 1, :, 0] = 3.0
        vcp = c1(torch.rand(1, 2, 32), torch.rand(1, 2, 9, 32), cand)
    assert torch.allclose(vcp, cand.mean(2), atol=1e-6)
