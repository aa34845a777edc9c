"""BASELINE.json's other configurations at their full sizes (C3 is bench.py's and
test_gpu_e2e.py's):

* C2 -- ModelNet40-like, 32 pairs x 2048 points with normals (C_in = 6, fp64), K = 32: the whole
  batch in one forward; pairs 0, 13 and 31 each equal their own single-pair run (pairs are
  independent in eval mode) and match the oracle (key points exact, R, t within
  1e-4).
* C5 -- synthetic 65536-point clouds, K = 256: the first FPS (65536 -> 10000, the split select
  above the register-resident limit) is bit-exact against the oracle, and the full forward +
  pose solve runs with its structural properties intact, with the reference's fp32 features and
  with BASELINE's fp16 feature storage (DeepVCP(feat_dtype=torch.float16): same key points, vcp
  and R, t within the features' fp16 rounding of the fp32 run).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _calibrated_pair(use_normal, K, r, s, src0, fe_npoint=10000):
    import oracle as O
    import dvcp
    from dvcp.synthetic import condition_weights, randomize_bn
    torch.manual_seed(0)
    ref = O.DeepVCP(use_normal=use_normal, K=K, r=r, s=s, fe_npoint=fe_npoint).eval()
    randomize_bn(ref)
    with torch.no_grad():
        _, calib = ref.FE1(src0)
    condition_weights(ref, feats=calib)
    mine = dvcp.DeepVCP(use_normal=use_normal, K=K, r=r, s=s, fe_npoint=fe_npoint).eval()
    mine.load_state_dict(ref.state_dict())
    return ref, mine


C2_PAIRS = (0, 4, 9, 13, 18, 22, 27, 31)   # 8 of the 32, spread over the batch


@pytest.fixture(scope="module")
def c2_batch(cuda):
    """C2 in one batch (32 ModelNet-like pairs with normals, fp64, N = 2048, K = 32)."""
    import dvcp
    from dvcp.synthetic import make_pairs
    B, N, K, r, s = 32, 2048, 32, 1.0, 0.4
    src, tgt, R_gt, t_gt = make_pairs(B, N, normals=True, seed=202)   # fp64, C_in = 6
    ref, mine = _calibrated_pair(True, K, r, s, src[:1])
    mine.to(cuda)
    starts = mine.draw_starts(B, N, N)
    tr = {}
    with torch.no_grad():
        kp, vcp = mine(src.to(cuda), tgt.to(cuda), R_gt.to(cuda), torch.zeros(1, 3), starts=starts, trace=tr)
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt.to(cuda), t_gt.to(cuda), 0.5)
    assert kp.shape == (B, K, 3) and vcp.shape == (B, K, 3) and torch.isfinite(loss)
    return dict(ref=ref, mine=mine, data=(src, tgt, R_gt, t_gt), starts=starts, trace=tr, out=(kp, vcp, R, t), K=K)


@pytest.mark.parametrize("b", C2_PAIRS)
def test_c2_pair_equals_single_pair_run(cuda, c2_batch, b):
    """Pairs are independent: pair b of the batch equals its own single-pair run."""
    import dvcp
    c = c2_batch
    src, tgt, R_gt, t_gt = c["data"]
    kp, vcp, R, t = c["out"]
    with torch.no_grad():
        kp1, vcp1 = c["mine"](src[b:b + 1].to(cuda), tgt[b:b + 1].to(cuda), R_gt[b:b + 1].to(cuda),
                              torch.zeros(1, 3), starts=c["starts"][:, b:b + 1])
        _, R1, t1 = dvcp.deepVCP_loss(kp1, vcp1, R_gt[b:b + 1].to(cuda), t_gt[b:b + 1].to(cuda), 0.5)
    assert torch.equal(kp1[0], kp[b]), b
    torch.testing.assert_close(vcp1[0], vcp[b], rtol=0, atol=1e-6)
    torch.testing.assert_close(R1[0], R[b], rtol=0, atol=1e-9)
    torch.testing.assert_close(t1[0], t[b], rtol=0, atol=1e-9)


@pytest.mark.parametrize("b", C2_PAIRS)
def test_c2_pair_vs_oracle(cuda, c2_batch, b):
    """Pair b of the C2 batch end to end against the oracle with the GPU's own top-k, checked rank
    by rank (tests_helpers.topk_parity).  Should a near-tie block reorder the top-k, the pair is
    re-run from the oracle's top-k and key points, R, t must still match: the R, t <= 1e-4 check is
    asserted on every path, never skipped."""
    import oracle as O
    import dvcp
    from tests_helpers import topk_parity
    c = c2_batch
    src, tgt, R_gt, t_gt = c["data"]
    kp, vcp, R, t = c["out"]
    tr, K, starts = c["trace"], c["K"], c["starts"]
    sl = slice(b, b + 1)
    with torch.no_grad(), O.fps_starts(list(starts[:, sl])), O.tracing() as trace:
        kp_o, vcp_o = c["ref"](src[sl], tgt[sl], R_gt[sl], torch.zeros(1, 3))
        _, R_o, t_o = O.deepVCP_loss(kp_o, vcp_o, R_gt[sl], t_gt[sl], 0.5)
    d = dict(trace)
    want = d["wl_score"][..., 0]
    exact, n_amb = topk_parity(tr["topk"][sl], tr["score"][sl], d["topk_idx"], want, K)
    print(f"C2 pair {b}: GPU top-k == oracle top-k: {exact} ({n_amb} near-tie rank boundaries)")
    if exact:
        kp0, R0, t0 = kp[sl], R[sl], t[sl]
    else:   # a near-tie block reordered: the back half from the oracle's top-k
        with torch.no_grad():
            kp0, vcp0 = c["mine"](src[sl].to(cuda), tgt[sl].to(cuda), R_gt[sl].to(cuda), torch.zeros(1, 3),
                                  starts=starts[:, sl], keypoint_idx=d["topk_idx"])
            _, R0, t0 = dvcp.deepVCP_loss(kp0, vcp0, R_gt[sl].to(cuda), t_gt[sl].to(cuda), 0.5)
    assert torch.equal(kp0.cpu(), kp_o.to(kp0.dtype))
    torch.testing.assert_close(R0.cpu(), R_o, rtol=0, atol=1e-4)
    torch.testing.assert_close(t0.cpu(), t_o, rtol=0, atol=1e-4)


def test_c5_first_fps_full_size_vs_oracle(cuda):
    """65536 -> 10000 (sa1 of C5): the default FPS path (round 6: the split select, 8 workgroups
    per cloud), bit-exact against the oracle's FPS."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(505)
    xyz = torch.rand(1, 65536, 3, generator=g) * 2 - 1
    start = torch.tensor([40000])
    want = O.farthest_point_sample(xyz, 10000, start)
    got, _ = ops.fps(xyz.to(cuda), 10000, start.to(cuda), pdim=1)
    assert torch.equal(got.cpu(), want)


def test_c5_forward_properties(cuda):
    """C5 shape end to end (N = 65536, K = 256, r = 2.0, s = 0.4): key points are rows of the
    source cloud, the virtual corresponding points are finite and inside the candidate grids'
    hull, R is a rotation (R_init = R_gt, Q13's reflection aside) and the loss is finite."""
    import dvcp
    from dvcp.synthetic import make_pairs
    B, N, K, r, s = 1, 65536, 256, 2.0, 0.4
    src, tgt, R_gt, t_gt = make_pairs(B, N, seed=555)
    torch.manual_seed(0)
    mine = dvcp.DeepVCP(use_normal=False, K=K, r=r, s=s).eval().to(cuda)
    tr = {}
    with torch.no_grad():
        kp, vcp = mine(src.to(cuda), tgt.to(cuda), R_gt.to(cuda), torch.zeros(1, 3), trace=tr)
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt.to(cuda), t_gt.to(cuda), 0.5)
    assert kp.shape == (B, K, 3) and vcp.shape == (B, K, 3)
    pts = src[0].t().to(cuda)                                     # (N, 3)
    member = (kp[0][:, None, :] == pts[None, :, :]).all(-1).any(-1)
    assert bool(member.all())                                     # every key point is a source point
    assert torch.isfinite(vcp).all()
    lo = tr["cand"].amin(dim=2)
    hi = tr["cand"].amax(dim=2)
    assert bool(((vcp >= lo - 1e-5) & (vcp <= hi + 1e-5)).all())  # convex combination of candidates
    det = torch.linalg.det(R)
    assert torch.isfinite(loss) and bool(torch.isfinite(R).all())
    torch.testing.assert_close(R @ R.transpose(1, 2), torch.eye(3, dtype=R.dtype, device=cuda).expand_as(R),
                               rtol=0, atol=1e-9)
    assert float(det.abs().min()) == pytest.approx(1.0, abs=1e-9)


def test_c5_fp16_features_vs_fp32(cuda):
    """C5 with BASELINE's "fp16 features" (the target feature table stored as fp16, gathered by
    dvcp_dfe_tgt_f16) against the same forward on fp32 features: identical key points and
    candidates, vcp within 1e-2 (fp16 rounding of the features, through the CPG softmax), R, t
    within 1e-3."""
    import dvcp
    from dvcp.synthetic import make_pairs
    B, N, K, r, s = 1, 65536, 256, 2.0, 0.4
    src, tgt, R_gt, t_gt = [x.to(cuda) for x in make_pairs(B, N, seed=556)]
    torch.manual_seed(0)
    m32 = dvcp.DeepVCP(use_normal=False, K=K, r=r, s=s).eval().to(cuda)
    m16 = dvcp.DeepVCP(use_normal=False, K=K, r=r, s=s, feat_dtype=torch.float16).eval().to(cuda)
    m16.load_state_dict(m32.state_dict())
    starts = m32.draw_starts(B, N, N)
    out = []
    with torch.no_grad():
        for m in (m32, m16):
            tr = {}
            kp, vcp = m(src, tgt, R_gt, torch.zeros(1, 3), starts=starts, trace=tr)
            _, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt, t_gt, 0.5)
            out.append((kp, vcp, R, t, tr["cand"]))
    (kp0, v0, R0, t0, c0), (kp1, v1, R1, t1, c1) = out
    assert torch.equal(kp0, kp1) and torch.equal(c0, c1)
    print(f"C5 fp16 vs fp32 features: vcp max|d| {float((v0 - v1).abs().max()):.2e}, "
          f"R max|d| {float((R0 - R1).abs().max()):.2e}, t max|d| {float((t0 - t1).abs().max()):.2e}")
    torch.testing.assert_close(v1, v0, rtol=0, atol=1e-2)
    torch.testing.assert_close(R1, R0, rtol=0, atol=1e-3)
    torch.testing.assert_close(t1, t0, rtol=0, atol=1e-3)


def test_c5_feature_extractor_full_size_vs_oracle(cuda):
    """C5's feature extractor at full size against the oracle, as test_e2e_c3_pair_vs_oracle does at C3:
    one 65536-point pair, K = 256, the GPU's own outputs of one forward (extract_features + top-k):
    * the FPS index sequences of all three layers of both clouds bit-exact (65536 -> 10000 -> 10000
      -> 10000; pointnet2_utils.py:63-84);
    * the six ball-query lists in the reference's padded form (pointnet2_utils.py:87-107; sa1
      scans all 65536 points for each of its 10000 centres) exact, except rows whose differing
      points sit within 4 ulp of r^2 (the oracle's BLAS-rounded square_distance; counted);
    * FE geometry exact, FE features (deep_feat_extraction.py:18-32) within rtol 1e-4, scores
      within 1e-3 relative (the conditioned WL's logit gain), and the K = 256 top-k rank by rank
      (tests_helpers.topk_parity; weighting_layer.py:26-33)."""
    import os

    import oracle as O
    from dvcp import ops
    from dvcp.synthetic import make_pairs
    from tests_helpers import ball_rows_mismatch_ok, padded_ball_rows, topk_parity
    B, N, K, r, s = 1, 65536, 256, 2.0, 0.4
    src, tgt, _, _ = make_pairs(B, N, seed=558)
    ref, mine = _calibrated_pair(False, K, r, s, src)
    mine = mine.to(cuda)
    torch.manual_seed(2)
    starts = mine.draw_starts(B, N, N)
    tr = {}
    with torch.no_grad():
        f = mine.extract_features(src.to(cuda), tgt.to(cuda), starts, trace=tr)
        top = ops.topk(f["score"], K)
    torch.cuda.synchronize()
    layers = tr["fe_layers"]
    radii = [mine.FE1.sa1.radius, mine.FE1.sa2.radius, mine.FE1.sa3.radius]
    n_boundary = 0
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    for side, (cloud, o0, key_xyz, key_feat) in enumerate(((src, 0, "src_xyz", "src_feat"),
                                                          (tgt, 4, "tgt_xyz", "tgt_feat"))):
        with torch.no_grad(), O.fps_starts([starts[o0 + i] for i in range(3)]), O.tracing() as trace:
            xyz_o, feat_o = ref.FE1(cloud)
            if side == 0:
                top_o = ref.WL(feat_o, K).view(B, K)
        d = dict(trace)
        fps_o = [v for n, v in trace if n == "fps_idx"]
        ball_o = [v for n, v in trace if n == "ball_idx"]
        pts = cloud[0].t().contiguous()
        for lvl, layer in enumerate(layers):
            fidx = fps_o[lvl][0]
            assert torch.equal(layer["idx"][side].cpu(), fidx), (side, lvl)
            ctr = pts[fidx]
            got = padded_ball_rows(layer, side)
            n_boundary += ball_rows_mismatch_ok(pts[None], ctr[None], got[None], ball_o[lvl], radii[lvl])
            pts = ctr
        assert torch.equal(f[key_xyz].transpose(1, 2).cpu(), xyz_o)
        torch.testing.assert_close(f[key_feat].cpu(), feat_o, rtol=1e-4, atol=1e-5)
        if side == 0:
            want = d["wl_score"][..., 0]
            torch.testing.assert_close(f["score"].cpu(), want, rtol=1e-3, atol=1e-5)
            exact, n_amb = topk_parity(top, f["score"], top_o, want, K)
    print(f"C5 FE: 6 FPS sequences exact, {n_boundary} ball rows differing only at r^2 rounding; GPU top-{K} == "
          f"oracle top-{K}: {exact} ({n_amb} near-tie rank boundaries)")


def test_c5_head_stage_decoupled_vs_oracle(cuda):
    """C5's head at full size, stage-decoupled: the GPU's feature extractor on
    a 65536-point pair, its K = 256 key points moved by R_init, then every head stage against the
    oracle fed the SAME inputs:
    * candidate grid (voxelize.py:19-83) of all 256 key points: exact;
    * kNN (get_cat_feat_tgt.py:44-52) of all 340,736 candidates, run at full size: indices and
      distances bit-exact on a 16-key-point slice (21,296 queries, the oracle's chunked brute force);
    * the fused target gather + DFE (get_cat_feat_tgt.py:54-96 + deep_feat_embedding.py:47-60) on
      the fp32 table, and on BASELINE's fp16 table against the oracle on the same rounded values:
      within 1e-5;
    * the source DFE (all key points) within 1e-5;
    * CPG (cpg.py:27-60) on the oracle's own DFE outputs for the slice: vcp within 1e-5."""
    import oracle as O
    import dvcp
    from dvcp import ops
    from dvcp.synthetic import make_pairs, randomize_bn
    B, N, K, r, s = 1, 65536, 256, 2.0, 0.4
    G = int((2 * r) / s + 1)
    src, tgt, R_gt, _ = make_pairs(B, N, seed=557)
    torch.manual_seed(0)
    mine = dvcp.DeepVCP(use_normal=False, K=K, r=r, s=s).eval().to(cuda)
    randomize_bn(mine)
    starts = mine.draw_starts(B, N, N)
    with torch.no_grad():
        f = mine.extract_features(src.to(cuda), tgt.to(cuda), starts)
        top = ops.topk(f["score"], K)
        keypts, src_cat, moved = ops.src_keypoints(f["src_xyz"], f["src_feat"], top, f["starts"][3], R_gt.to(cuda))
        src_dfe = ops.dfe(src_cat, mine.DFE.packed_params())
        cand, _ = ops.voxelize(moved, r, s, G, pdim=1)
        qry = cand.view(B, K * G ** 3, 3)
        dist, idx, _ = ops.knn(f["tgt_xyz"], qry, 32, ref_pdim=2, qry_pdim=1, want_idx64=False)
        tgt_dfe = ops.dfe_tgt(f["tgt_xyz"], f["tgt_feat"], qry, dist, idx, mine.DFE.packed_params(), ref_pdim=2)
        tgt_dfe16 = ops.dfe_tgt(f["tgt_xyz"], f["tgt_feat"].half(), qry, dist, idx, mine.DFE.packed_params(),
                                ref_pdim=2)
    torch.cuda.synchronize()
    dfe_o, cpg_o = O.feat_embedding_layer(), O.cpg()
    dfe_o.load_state_dict({k: v.cpu() for k, v in mine.DFE.state_dict().items()})
    cpg_o.load_state_dict({k: v.cpu() for k, v in mine.cpg.state_dict().items()})
    cand_o = O.voxelize(moved.cpu(), r, s)
    assert torch.equal(cand.cpu(), cand_o)
    with torch.no_grad():
        src_dfe_o = dfe_o(src_cat.cpu(), src=True)
    torch.testing.assert_close(src_dfe.cpu(), src_dfe_o, rtol=1e-5, atol=1e-5)
    tx, tf = f["tgt_xyz"].transpose(1, 2).cpu(), f["tgt_feat"].cpu()
    sl = slice(120, 136)                                   # 16 key points of 256
    C = G ** 3
    kp_sl = keypts[:, sl].cpu()
    wants = []
    for table, got_dfe in ((tf, tgt_dfe), (tf.half().float(), tgt_dfe16)):
        with torch.no_grad(), O.tracing() as trace:
            cat_o = O.Get_Cat_Feat_Tgt()(cand_o[:, sl], kp_sl, tx, table)
            want_dfe = dfe_o(cat_o, src=False)
            del cat_o
        d = dict(trace)
        q = slice(sl.start * C, sl.stop * C)
        assert torch.equal(idx[:, q].cpu().long(), d["knn_idx"]), "C5 kNN indices differ from the oracle"
        assert torch.equal(dist[:, q].cpu(), d["knn_dist"]), "C5 kNN distances differ from the oracle"
        torch.testing.assert_close(got_dfe[:, q].cpu().view(want_dfe.shape), want_dfe, rtol=1e-5, atol=1e-5)
        wants.append(want_dfe)
    # CPG on the oracle's own stage inputs (the fp32 table's DFE of the slice)
    with torch.no_grad():
        vcp_o = cpg_o(src_dfe_o[:, sl].unsqueeze(2), wants[0].permute(0, 1, 3, 2), cand_o[:, sl], r, s)
        vcp = ops.cpg(src_dfe_o[:, sl].to(cuda), wants[0].to(cuda).permute(0, 1, 3, 2), cand_o[:, sl].to(cuda), G,
                      mine.cpg.packed_params())
    torch.testing.assert_close(vcp.cpu(), vcp_o, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype,N,npoint,B", [(torch.float32, 40000, 3000, 3), (torch.float64, 20000, 2000, 2)])
def test_split_fps_vs_oracle(cuda, dtype, N, npoint, B):
    """The per-step split FPS (S workgroups per cloud, ragged last chunk, several clouds per
    launch; parts=1 -- the default above 16384 fp32 points is the split select) is bit-exact
    against the oracle's FPS."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(N + B)
    xyz = (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dtype)
    start = torch.randint(0, N, (B,), generator=g)
    want = O.farthest_point_sample(xyz, npoint, start)
    got, ctr = ops.fps(xyz.to(cuda), npoint, start.to(cuda), pdim=1, parts=1)
    assert torch.equal(got.cpu(), want)
    assert torch.equal(ctr.cpu(), torch.gather(xyz, 1, want[..., None].expand(B, npoint, 3)).transpose(1, 2))


def test_dense_fps_vs_oracle(cuda):
    """Clouds beyond the split kernel's 16 workgroups (here fp64, 140000 points > 16 x 8192) take
    the one-workgroup dense kernel: bit-exact against the oracle."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(77)
    B, N, npoint = 1, 140000, 300
    xyz = torch.rand(B, N, 3, generator=g, dtype=torch.float64) * 2 - 1
    start = torch.randint(0, N, (B,), generator=g)
    got, _ = ops.fps(xyz.to(cuda), npoint, start.to(cuda), pdim=1)
    assert torch.equal(got.cpu(), O.farthest_point_sample(xyz, npoint, start))


def test_split_fps_guard_raises(cuda):
    """The split FPS's bounded wait: with one workgroup of the last cloud withheld from the grid,
    that cloud's other workgroups give up after spin_cap polls and raise the error word; their
    indices stay in range (never -1), the centres they could not compute are the start point's
    coordinates (finite, never the uninitialised buffer), and the complete clouds are still exact."""
    import ctypes

    import oracle as O
    from dvcp import _lib
    g = torch.Generator().manual_seed(78)
    B, N, npoint = 3, 40000, 200                       # S = 3 workgroups per fp32 cloud
    xyz = torch.rand(B, N, 3, generator=g) * 2 - 1
    start = torch.randint(0, N, (B,), generator=g)
    x, st = xyz.to(cuda), start.to(cuda)
    idx = torch.full((B, npoint), -7, dtype=torch.int64, device=cuda)
    ctr = torch.full((B, 3, npoint), float("nan"), dtype=torch.float32, device=cuda)
    ws = torch.empty(B, N, dtype=torch.float32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    _lib.call("dvcp_fps_split_probe", _lib.F32, _lib.ptr(x), N * 3, 1, 3, B, N, npoint, _lib.ptr(st), _lib.ptr(idx),
              _lib.ptr(ctr), _lib.ptr(ws), _lib.ptr(err), ctypes.c_uint32(2000), 1, _lib.stream())
    torch.cuda.synchronize()
    assert int(err.item()) == 1
    got, c = idx.cpu(), ctr.cpu()
    assert bool(((got >= 0) & (got < N)).all())
    assert bool(torch.isfinite(c).all())
    # every centre is the point its index names; the unfinished steps hold the start point
    assert torch.equal(c, torch.gather(xyz, 1, got[..., None].expand(B, npoint, 3)).transpose(1, 2))
    last = got[B - 1]
    assert int(last[-1]) == int(start[B - 1])
    want = O.farthest_point_sample(xyz[:B - 1], npoint, start[:B - 1])
    assert torch.equal(got[:B - 1], want)
    # the same launch with the full grid completes and leaves the word clear
    err.zero_()
    _lib.call("dvcp_fps_split_probe", _lib.F32, _lib.ptr(x), N * 3, 1, 3, B, N, npoint, _lib.ptr(st), _lib.ptr(idx),
              _lib.ptr(ctr), _lib.ptr(ws), _lib.ptr(err), ctypes.c_uint32(1 << 22), 0, _lib.stream())
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(idx.cpu(), O.farthest_point_sample(xyz, npoint, start))


def test_device_flag_check_raises(cuda):
    """A set error word surfaces as RuntimeError from dvcp.check_device_flags (the path the split
    FPS guard and the voxel-grid length check take)."""
    import dvcp
    from dvcp import _lib
    dvcp.check_device_flags(block=True)
    _lib.defer_flag_check("probe flag", torch.ones(1, dtype=torch.int32, device=cuda))
    with pytest.raises(RuntimeError, match="probe flag"):
        dvcp.check_device_flags(block=True)
    dvcp.check_device_flags(block=True)   # reported once


def test_device_flags_deferred_to_step_end(cuda):
    """Inside ``deferred_flags`` (DeepVCP.forward's scope) the words are copied once when the block
    closes, on the stream each was flagged on: a set word still raises (after the block), and the
    clear words of the same block do not."""
    import dvcp
    from dvcp import _lib
    dvcp.check_device_flags(block=True)
    side = torch.cuda.Stream(device=cuda)
    with _lib.deferred_flags():
        _lib.defer_flag_check("clear word", torch.zeros(1, dtype=torch.int32, device=cuda))
        with torch.cuda.stream(side):
            w = torch.zeros(1, dtype=torch.int32, device=cuda)
            w.fill_(3)
            _lib.defer_flag_check("deferred probe", w)
        assert not _lib._PENDING_FLAGS        # nothing copied yet
    assert len(_lib._PENDING_FLAGS) == 2      # one copy per stream, one entry per word
    with pytest.raises(RuntimeError, match="deferred probe"):
        dvcp.check_device_flags(block=True)
    dvcp.check_device_flags(block=True)
