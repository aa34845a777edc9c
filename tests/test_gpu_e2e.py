"""End-to-end parity: dvcp.DeepVCP + deepVCP_loss on the GPU vs REF-R (oracle).

Checked stage by stage so that fp32 drift upstream cannot hide a discrete mismatch (SURVEY.md
section 4: stage-decoupled): FE xyz (pure FPS geometry) bit-exact; FE features rtol 1e-4;
key points exact unless the oracle's own ranking is a near tie at the measured precision
(flagged, and then the back half still runs from the oracle's top-k); candidates, kNN indices
and distances bit-exact; vcp atol 1e-5; R, t atol 1e-4 (the north_star bar).
"""
import numpy as np
import pytest
import torch

from tests_helpers import golden, golden_state_dict, topk_parity

pytestmark = pytest.mark.gpu


def _load_model(cuda, z, dfe_literal=False):
    import dvcp
    model = dvcp.DeepVCP(use_normal=bool(z["normals"]), K=int(z["K"]), r=float(z["r"]), s=float(z["s"]),
                         fe_npoint=int(z["fe_npoint"]), dfe_literal=dfe_literal).eval()
    model.load_state_dict(golden_state_dict(z))
    return model.to(cuda)


def _forward(cuda, model, z, keypoint_idx=None):
    import dvcp
    src, tgt = torch.from_numpy(z["src"]).to(cuda), torch.from_numpy(z["tgt"]).to(cuda)
    R_gt, t_gt = torch.from_numpy(z["R_gt"]).to(cuda), torch.from_numpy(z["t_gt"]).to(cuda)
    tr = {}
    with torch.no_grad():
        kp, vcp = model(src, tgt, R_gt, torch.zeros(1, 3), starts=torch.from_numpy(z["starts"]), trace=tr,
                        keypoint_idx=keypoint_idx)
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt, t_gt, 0.5)
    return tr, kp, vcp, loss, R, t


@pytest.mark.parametrize("name", ["e2e_c3small", "e2e_c1"])
def test_e2e_fixture_front(cuda, name):
    """Own pipeline up to the key points: FE geometry exact, features/scores close, and the
    GPU's own top-k equals the oracle's wherever the oracle's ranking is determined at the
    precision the two fp32 pipelines agree to."""
    z = golden(name)
    K = int(z["K"])
    tr, kp, vcp, loss, R, t = _forward(cuda, _load_model(cuda, z), z)
    assert torch.equal(tr["src_xyz"].transpose(1, 2).cpu(), torch.from_numpy(z["fe_xyz_src"]))
    assert torch.equal(tr["tgt_xyz"].transpose(1, 2).cpu(), torch.from_numpy(z["fe_xyz_tgt"]))
    torch.testing.assert_close(tr["src_feat"].cpu(), torch.from_numpy(z["fe_feat_src"]), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["tgt_feat"].cpu(), torch.from_numpy(z["fe_feat_tgt"]), rtol=1e-4, atol=1e-5)
    # the conditioned WL centres its logits, which amplifies the ~1e-6 relative fp32 feature
    # noise by mean/std of the raw logit (~100x); scores agree to 1e-3 relative
    want = torch.from_numpy(z["score"])
    torch.testing.assert_close(tr["score"].cpu(), want, rtol=1e-3, atol=1e-5)
    exact, n_amb = topk_parity(tr["topk"], tr["score"], torch.from_numpy(z["topk"]), want, K)
    print(f"{name}: GPU top-k == oracle top-k: {exact} ({n_amb} near-tie rank boundaries)")
    if exact or torch.equal(kp.cpu(), torch.from_numpy(z["keypts_out"])):
        # the GPU's own top-k drives the back half: the whole forward against the fixture
        torch.testing.assert_close(kp.cpu(), torch.from_numpy(z["keypts_out"]), rtol=0, atol=0)
        torch.testing.assert_close(vcp.cpu(), torch.from_numpy(z["vcp"]), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(R.cpu(), torch.from_numpy(z["R"]), rtol=0, atol=1e-4)
        torch.testing.assert_close(t.cpu(), torch.from_numpy(z["t"]), rtol=0, atol=1e-4)
    # otherwise the order differs only inside near-tie blocks (asserted above) and the back
    # half is checked from the oracle's top-k in test_e2e_fixture_back


@pytest.mark.parametrize("dfe", ["collapsed", "literal"])
@pytest.mark.parametrize("name", ["e2e_c3small", "e2e_c1"])
def test_e2e_fixture_back(cuda, name, dfe):
    """Stage-decoupled back half: the oracle's top-k indices are fed in, then key points,
    candidates and kNN indices must be exact and vcp / R / t / loss within tolerance -- with the
    product's collapsed DFE map and with the literal fc1 -> fc2 -> fc3 chain (SURVEY App. A.3 Q14's
    parity path, DeepVCP(dfe_literal=True))."""
    z = golden(name)
    tr, kp, vcp, loss, R, t = _forward(cuda, _load_model(cuda, z, dfe_literal=dfe == "literal"), z,
                                       keypoint_idx=torch.from_numpy(z["topk"]))
    B = kp.shape[0]
    assert torch.equal(kp.cpu(), torch.from_numpy(z["keypts_out"]))
    torch.testing.assert_close(tr["src_cat"].cpu(), torch.from_numpy(z["src_cat"]).float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["moved"].cpu(), torch.from_numpy(z["moved"]), rtol=0, atol=1e-12)
    nq = z["knn_idx_head"].shape[1]
    assert torch.equal(tr["knn_idx"][:, :nq].cpu(), torch.from_numpy(z["knn_idx_head"]))
    assert torch.equal(tr["knn_dist"][:, :nq].cpu(), torch.from_numpy(z["knn_dist_head"]))
    torch.testing.assert_close(tr["src_dfe"].cpu(), torch.from_numpy(z["src_dfe"]), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["tgt_dfe"].reshape(B, -1, 32)[:, :nq].cpu(), torch.from_numpy(z["tgt_dfe_head"]),
                               rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(vcp.cpu(), torch.from_numpy(z["vcp"]), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(R.cpu(), torch.from_numpy(z["R"]), rtol=0, atol=1e-4)
    torch.testing.assert_close(t.cpu(), torch.from_numpy(z["t"]), rtol=0, atol=1e-4)
    torch.testing.assert_close(loss.cpu(), torch.from_numpy(z["loss"]), rtol=1e-4, atol=1e-6)


def _oracle_threads():
    """The oracle's CPU threads: the cores this process may use, capped at the GPU box's CPU
    share (16 per GPU)."""
    import os
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(n, 16))


C3_B = 8


@pytest.fixture(scope="module")
def c3_lanes(cuda):
    """BASELINE C3 as bench.py runs it: B = 8 pairs, N = 16384, K = 64, r = 2.0, s = 0.4, FE npoint
    10000, with two more 8-pair batches in flight on their own streams.  The lane-0 batch (with its
    stage trace: FE layers' FPS indices and ball-query lists, features, scores, top-k, candidates,
    kNN) and the same batch run alone."""
    import oracle as O
    import dvcp
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn
    B, N, K, r, s = C3_B, 16384, 64, 2.0, 0.4
    lanes_data = [make_pairs(B, N, seed=777 + 101 * lane) for lane in range(3)]
    torch.manual_seed(0)
    ref = O.DeepVCP(use_normal=False, K=K, r=r, s=s).eval()
    randomize_bn(ref)
    mine = dvcp.DeepVCP(use_normal=False, K=K, r=r, s=s).eval().to(cuda)
    mine.load_state_dict(ref.state_dict())
    src = lanes_data[0][0]
    with torch.no_grad():
        _, calib, _ = mine.FE1.run(src[:1].to(cuda))
    condition_weights(ref, feats=calib)     # separated key-point scores (dvcp/synthetic.py)
    mine.load_state_dict(ref.state_dict())
    torch.manual_seed(1)
    starts = [mine.draw_starts(B, N, N) for _ in lanes_data]
    dev_data = [tuple(x.to(cuda) for x in d) for d in lanes_data]

    def run(lane, trace=None):
        s_, g_, R_, t_ = dev_data[lane]
        kp, vcp = mine(s_, g_, R_, torch.zeros(1, 3), starts=starts[lane], trace=trace)
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_, t_, 0.5)
        return kp, vcp, loss, R, t

    streams = [torch.cuda.Stream(device=cuda) for _ in lanes_data]
    tr = {}
    with torch.no_grad():
        outs = []
        for lane, st in enumerate(streams):
            with torch.cuda.stream(st):
                outs.append(run(lane, trace=tr if lane == 0 else None))
        torch.cuda.synchronize()
        alone = run(0)
        torch.cuda.synchronize()
    return dict(ref=ref, mine=mine, data=lanes_data[0], starts=starts[0], trace=tr, outs=outs, alone=alone,
                K=K)


def test_e2e_c3_lanes_equal_alone(c3_lanes):
    """The lane-0 batch run alongside two other batches equals the same batch run alone, bit for bit."""
    for a, b in zip(c3_lanes["outs"][0], c3_lanes["alone"]):
        assert torch.equal(a, b), "a batch run alongside others differs from the same batch run alone"


@pytest.mark.parametrize("b", range(C3_B))
def test_e2e_c3_pair_vs_oracle(cuda, c3_lanes, b):
    """Every pair of the C3 batch against the live oracle (REF-R, oracle/ref_r.py), stage by stage
    with the GPU's OWN outputs of the batched run:
    * all 7 FPS index sequences bit-exact (src / tgt sa1-sa3 at 16384 -> 10000 -> 10000 -> 10000);
    * the six FE ball-query lists (pointnet2_utils.py:87-107, padded form) -- exact except rows
      whose differing points sit within 4 ulp of r^2 (BLAS rounding of square_distance; counted);
    * FE geometry exact, FE features (src and tgt) within rtol 1e-4;
    * top-k per rank (tests_helpers.topk_parity), key points and candidates exact;
    * the kNN (get_cat_feat_tgt.py:44-52) of all 85184 candidates: indices AND distances bit-exact;
    * target DFE features within rtol 1e-4, vcp within 1e-5, R, t within the north_star's 1e-4.
    Should a near-tie block reorder the top-k, the back half (key points, candidates, kNN, DFE,
    vcp, R, t) is re-run from the oracle's top-k at full size and checked the same way."""
    import oracle as O
    from tests_helpers import ball_rows_mismatch_ok, padded_ball_rows
    c = c3_lanes
    ref, mine, K, tr = c["ref"], c["mine"], c["K"], c["trace"]
    src, tgt, R_gt, t_gt = c["data"]
    starts = c["starts"]
    kp, vcp, loss, R, t = (x.cpu() for x in c["outs"][0])
    B = src.shape[0]
    torch.set_num_threads(_oracle_threads())
    with torch.no_grad(), O.fps_starts([x[b:b + 1] for x in starts]), O.tracing() as trace:
        kp_o, vcp_o = ref(src[b:b + 1], tgt[b:b + 1], R_gt[b:b + 1], torch.zeros(1, 3))
        loss_o, R_o, t_o = O.deepVCP_loss(kp_o, vcp_o, R_gt[b:b + 1], t_gt[b:b + 1], 0.5)
    d = dict(trace)
    fps_o = [v for n, v in trace if n == "fps_idx"]    # src sa1-3, key points, tgt sa1-3
    ball_o = [v for n, v in trace if n == "ball_idx"]
    feat_o = [v for n, v in trace if n == "fe_feat"]
    fe_x = [v for n, v in trace if n == "fe_xyz"]
    radii = [mine.FE1.sa1.radius, mine.FE1.sa2.radius, mine.FE1.sa3.radius]
    n_boundary = 0
    for side, (row, o0, cloud) in enumerate(((b, 0, src), (B + b, 4, tgt))):
        pts = cloud[b].t().contiguous()                       # (N, 3)
        for lvl, layer in enumerate(tr["fe_layers"]):
            fidx = fps_o[o0 + lvl][0]
            assert torch.equal(layer["idx"][row].cpu(), fidx), (side, lvl)
            ctr = pts[fidx]
            got = padded_ball_rows(layer, row)
            n_boundary += ball_rows_mismatch_ok(pts[None], ctr[None], got[None], ball_o[o0 + lvl], radii[lvl])
            pts = ctr
    assert torch.equal(tr["src_xyz"][b:b + 1].transpose(1, 2).cpu(), fe_x[0])
    assert torch.equal(tr["tgt_xyz"][b:b + 1].transpose(1, 2).cpu(), fe_x[1])
    torch.testing.assert_close(tr["src_feat"][b:b + 1].cpu(), feat_o[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["tgt_feat"][b:b + 1].cpu(), feat_o[1], rtol=1e-4, atol=1e-5)
    want = d["wl_score"][..., 0]
    torch.testing.assert_close(tr["score"][b:b + 1].cpu(), want, rtol=1e-3, atol=1e-5)
    exact, n_amb = topk_parity(tr["topk"][b:b + 1], tr["score"][b:b + 1], d["topk_idx"], want, K)
    print(f"C3 pair {b}: 7 FPS exact, {n_boundary} ball rows differing only at r^2 rounding; GPU top-k == oracle "
          f"top-k: {exact} ({n_amb} near-tie rank boundaries), max|dR| {float((R[b] - R_o[0]).abs().max()):.2e}, "
          f"max|dt| {float((t[b] - t_o[0]).abs().max()):.2e}")
    if exact:
        back = dict(kp=kp[b:b + 1], vcp=vcp[b:b + 1], R=R[b:b + 1], t=t[b:b + 1], cand=tr["cand"][b:b + 1],
                    knn_idx=tr["knn_idx"][b:b + 1], knn_dist=tr["knn_dist"][b:b + 1], tgt_dfe=tr["tgt_dfe"][b:b + 1])
    else:   # near-tie block reordered: the back half from the oracle's top-k
        one = tuple(x[b:b + 1].to(cuda) for x in c["data"])
        tr1 = {}
        with torch.no_grad():
            kp1, vcp1, _, R1, t1 = _run_pair(mine, one, [x[b:b + 1] for x in starts], d["topk_idx"], trace=tr1)
        back = dict(kp=kp1, vcp=vcp1, R=R1, t=t1, cand=tr1["cand"], knn_idx=tr1["knn_idx"], knn_dist=tr1["knn_dist"],
                    tgt_dfe=tr1["tgt_dfe"])
    back = {k: v.cpu() for k, v in back.items()}
    assert torch.equal(back["kp"], kp_o)
    assert torch.equal(back["cand"], d["candidates"])
    assert torch.equal(back["knn_idx"].long(), d["knn_idx"]), "kNN indices differ from the oracle"
    assert torch.equal(back["knn_dist"], d["knn_dist"]), "kNN distances differ from the oracle"
    torch.testing.assert_close(back["tgt_dfe"].reshape(d["tgt_dfe"].shape), d["tgt_dfe"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(back["vcp"], vcp_o, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(back["R"], R_o, rtol=0, atol=1e-4)
    torch.testing.assert_close(back["t"], t_o, rtol=0, atol=1e-4)


def _run_pair(model, data, starts, keypoint_idx, trace=None):
    import dvcp
    s_, g_, R_, t_ = data
    kp, vcp = model(s_, g_, R_, torch.zeros(1, 3), starts=torch.stack(starts), keypoint_idx=keypoint_idx, trace=trace)
    loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_, t_, 0.5)
    return kp, vcp, loss, R, t


def test_module_surface_errors(cuda):
    import dvcp
    m = dvcp.DeepVCP(use_normal=False).to(cuda)   # training mode by default, like nn.Module
    x = torch.zeros(1, 3, 64, device=cuda)
    with torch.no_grad(), pytest.raises(NotImplementedError):   # training mode needs autograd
        m(x, x, torch.eye(3, dtype=torch.float64, device=cuda)[None], torch.zeros(1, 3))
    m.eval()
    with pytest.raises(RuntimeError, match="float64"):
        m(x, x, torch.eye(3, device=cuda)[None], torch.zeros(1, 3))
    c = dvcp.cpg().eval().to(cuda)
    with pytest.raises(AssertionError):
        c(torch.zeros(1, 1, 1, 32, device=cuda), torch.zeros(1, 1, 32, 100, device=cuda),
          torch.zeros(1, 1, 100, 3, device=cuda), 1.0, 0.4)


def test_return_weights_and_paper_loss(cuda):
    """forward(..., return_weights=True) also returns the key points' weighting-layer scores
    (score[topk], descending like torch.topk), and the paper's weighted loss runs on them."""
    import dvcp
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn
    src, tgt, R, t = make_pairs(2, 2048, seed=41)
    torch.manual_seed(0)
    m = dvcp.DeepVCP(use_normal=False, K=32, r=1.0, s=0.4, fe_npoint=512).eval().to(cuda)
    randomize_bn(m)
    with torch.no_grad():
        _, calib, _ = m.FE1.run(src.to(cuda))
    condition_weights(m, feats=calib)
    starts = m.draw_starts(2, 2048, 2048)
    tr = {}
    with torch.no_grad():
        kp, vcp, w = m(src.to(cuda), tgt.to(cuda), R.to(cuda), torch.zeros(1, 3), starts=starts, trace=tr,
                       return_weights=True)
        kp2, vcp2 = m(src.to(cuda), tgt.to(cuda), R.to(cuda), torch.zeros(1, 3), starts=starts)
        loss, Rp, tp = dvcp.paper.deepVCP_loss_paper(kp, vcp, w, R.to(cuda), t.to(cuda), 0.5)
    assert torch.equal(kp, kp2) and torch.equal(vcp, vcp2)
    assert torch.equal(w, torch.gather(tr["score"], 1, tr["topk"]))
    assert (w[:, 1:] <= w[:, :-1]).all() and (w > 0).all()
    assert torch.isfinite(loss) and (torch.linalg.det(Rp) > 0).all()


def test_dfe_weight_change_between_eval_forwards(cuda):
    """The packed DFE parameters are formed on the calling stream before the source-row DFE forks
    to the side stream, and both DFE launches read that one buffer: after a DFE weight
    changes between two eval forwards, the second forward equals a fresh model's with the new
    weights, bit for bit (a stale or half-rebuilt pack would differ)."""
    z = golden("e2e_c1")
    model = _load_model(cuda, z)
    _forward(cuda, model, z)  # builds and caches the pack
    with torch.no_grad():
        model.DFE.fc2.weight.mul_(1.5)
        model.DFE.fc3.bias.add_(0.25)
    _, kp1, vcp1, _, R1, t1 = _forward(cuda, model, z)
    fresh = _load_model(cuda, z)
    fresh.load_state_dict(model.state_dict())
    _, kp2, vcp2, _, R2, t2 = _forward(cuda, fresh, z)
    assert torch.equal(kp1, kp2) and torch.equal(vcp1, vcp2) and torch.equal(R1, R2) and torch.equal(t1, t2)
    # and the change did reach the kernels: the pose moved against the fixture's weights
    _, _, vcp0, _, _, _ = _forward(cuda, _load_model(cuda, z), z)
    assert not torch.equal(vcp0, vcp1)


def test_captured_step_equals_eager(cuda):
    """dvcp.graphs.CapturedStep: the forward + pose solve + registration error captured once as a
    HIP graph and replayed with new FPS starts equals the eager step with those starts, bit for bit
    (two replays with different starts; the graph's error words are checked after each)."""
    import dvcp
    from dvcp import _lib
    from dvcp.graphs import CapturedStep
    z = golden("e2e_c1")
    model = _load_model(cuda, z)
    src, tgt = torch.from_numpy(z["src"]).to(cuda), torch.from_numpy(z["tgt"]).to(cuda)
    R_gt, t_gt = torch.from_numpy(z["R_gt"]).to(cuda), torch.from_numpy(z["t_gt"]).to(cuda)
    B = src.shape[0]
    g = CapturedStep(model, src, tgt, R_gt, t_gt, alpha=0.5, starts=torch.from_numpy(z["starts"]))
    gen = torch.Generator().manual_seed(77)
    for _ in range(2):
        sizes = (src.shape[2], model.FE1.sa1.npoint, model.FE1.sa2.npoint, model.K, tgt.shape[2],
                 model.FE1.sa1.npoint, model.FE1.sa2.npoint)
        starts = torch.stack([torch.randint(0, n, (B,), generator=gen) for n in sizes])
        R, t, rot, trans = g.replay(starts)
        torch.cuda.synchronize()
        R, t, rot, trans = R.clone(), t.clone(), rot.clone(), trans.clone()
        with torch.no_grad():
            kp, vcp = model(src, tgt, R_gt, torch.zeros(1, 3), starts=starts)
            _, R2, t2 = dvcp.deepVCP_loss(kp, vcp, R_gt, t_gt, 0.5)
            rot2, trans2 = dvcp.registration_errors(R2, t2, R_gt, t_gt)
        assert torch.equal(R, R2) and torch.equal(t, t2)
        assert torch.equal(rot, rot2) and torch.equal(trans, trans2)
    _lib.check_device_flags(block=True)
