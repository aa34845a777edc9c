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

from tests_helpers import golden, golden_state_dict

pytestmark = pytest.mark.gpu


def _near_tie(score, K, rel):
    """True if two distinct values among the oracle's top K+1 scores are closer than `rel`
    (relative): the top-k order/set is then not determined at the precision both sides agree
    to.  Exactly equal scores come from duplicated FE points (N < npoint, Q1) and are
    value-identical, so they are not counted."""
    for row in score.double():
        s = torch.unique(torch.sort(row, descending=True).values[: K + 1])
        if s.numel() > 1 and bool(((s[1:] - s[:-1]) / s[1:].abs().clamp_min(1e-30) < rel).any()):
            return True
    return False


def _score_noise(got, want):
    return float(((got.double() - want.double()).abs() / want.double().abs().clamp_min(1e-30)).max())


def _load_model(cuda, z):
    import dvcp
    model = dvcp.DeepVCP(use_normal=bool(z["normals"]), K=int(z["K"]), r=float(z["r"]), s=float(z["s"]),
                         fe_npoint=int(z["fe_npoint"])).eval()
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
    noise = _score_noise(tr["score"].cpu(), want)
    if _near_tie(want, K, rel=max(1e-5, 10 * noise)):
        pytest.skip(f"oracle top-{K} not determined at the agreed precision ({noise:.1e}); the back half is "
                    "checked with the oracle's top-k in test_e2e_fixture_back")
    torch.testing.assert_close(kp.cpu(), torch.from_numpy(z["keypts_out"]), rtol=0, atol=0)


@pytest.mark.parametrize("name", ["e2e_c3small", "e2e_c1"])
def test_e2e_fixture_back(cuda, name):
    """Stage-decoupled back half: the oracle's top-k indices are fed in, then key points,
    candidates and kNN indices must be exact and vcp / R / t / loss within tolerance."""
    z = golden(name)
    tr, kp, vcp, loss, R, t = _forward(cuda, _load_model(cuda, z), z, keypoint_idx=torch.from_numpy(z["topk"]))
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


def test_e2e_live_full_size_pair(cuda):
    """One C3 pair at full size (N=16384, K=64, r=2.0, npoint 10000) against the live oracle,
    end to end with the GPU's own top-k (R, t within the north_star's 1e-4)."""
    import oracle as O
    import dvcp
    from dvcp.synthetic import condition_weights, make_pairs, randomize_bn
    src, tgt, R_gt, t_gt = make_pairs(1, 16384, seed=777)
    torch.manual_seed(0)
    ref = O.DeepVCP(use_normal=False, K=64, r=2.0, s=0.4).eval()
    randomize_bn(ref)
    with torch.no_grad():
        _, calib = ref.FE1(src)
    condition_weights(ref, feats=calib)
    mine = dvcp.DeepVCP(use_normal=False, K=64, r=2.0, s=0.4).eval()
    mine.load_state_dict(ref.state_dict())
    mine.to(cuda)
    torch.manual_seed(1)
    with torch.no_grad(), O.tracing() as trace:
        kp_o, vcp_o = ref(src, tgt, R_gt, torch.zeros(1, 3))
        loss_o, R_o, t_o = O.deepVCP_loss(kp_o, vcp_o, R_gt, t_gt, 0.5)
    torch.manual_seed(1)
    tr = {}
    with torch.no_grad():
        kp, vcp = mine(src.to(cuda), tgt.to(cuda), R_gt.to(cuda), torch.zeros(1, 3), trace=tr)
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt.to(cuda), t_gt.to(cuda), 0.5)
    d = dict(trace)
    fe_x = [v for n, v in trace if n == "fe_xyz"]
    assert torch.equal(tr["src_xyz"].transpose(1, 2).cpu(), fe_x[0])
    assert torch.equal(tr["tgt_xyz"].transpose(1, 2).cpu(), fe_x[1])
    want = d["wl_score"][..., 0]
    noise = _score_noise(tr["score"].cpu(), want)
    if _near_tie(want, 64, rel=max(1e-5, 10 * noise)):
        pytest.skip(f"top-k not determined at the agreed precision ({noise:.1e})")
    torch.testing.assert_close(kp.cpu(), kp_o, rtol=0, atol=0)
    assert torch.equal(tr["cand"].cpu(), d["candidates"])
    torch.testing.assert_close(vcp.cpu(), vcp_o, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(R.cpu(), R_o, rtol=0, atol=1e-4)
    torch.testing.assert_close(t.cpu(), t_o, rtol=0, atol=1e-4)
    torch.testing.assert_close(loss.cpu(), loss_o, rtol=1e-4, atol=1e-6)


def test_module_surface_errors(cuda):
    import dvcp
    m = dvcp.DeepVCP(use_normal=False).to(cuda)   # training mode by default, like nn.Module
    x = torch.zeros(1, 3, 64, device=cuda)
    with pytest.raises(NotImplementedError):
        m(x, x, torch.eye(3, dtype=torch.float64, device=cuda)[None], torch.zeros(1, 3))
    m.eval()
    with pytest.raises(RuntimeError, match="float64"):
        m(x, x, torch.eye(3, device=cuda)[None], torch.zeros(1, 3))
    c = dvcp.cpg().eval().to(cuda)
    with pytest.raises(AssertionError):
        c(torch.zeros(1, 1, 1, 32, device=cuda), torch.zeros(1, 1, 32, 100, device=cuda),
          torch.zeros(1, 1, 100, 3, device=cuda), 1.0, 0.4)
