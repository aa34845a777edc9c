"""End-to-end parity: dvcp.DeepVCP + deepVCP_loss on the GPU vs REF-R (oracle).

Checked stage by stage so that fp32 drift upstream cannot hide a discrete mismatch:
FE xyz (pure FPS geometry) bit-exact; FE features rtol 1e-4; scores rtol 1e-4; key-point set
exact unless the oracle's 64th/65th score gap is a near tie (< 1e-5 relative, flagged);
candidates bit-exact; kNN indices exact; vcp atol 1e-5; R, t atol 1e-4 (north_star bar).
"""
import numpy as np
import pytest
import torch

from tests_helpers import golden, golden_state_dict

pytestmark = pytest.mark.gpu


def _near_tie(score, K, rel=1e-5):
    """True if two distinct values among the oracle's top K+1 scores are closer than `rel`
    (relative): then the reference's own top-k order/set is decided by fp32 rounding.  Exactly
    equal scores come from duplicated FE points (N < npoint, Q1) and are value-identical."""
    for row in score.double():
        s = torch.unique(torch.sort(row, descending=True).values[: K + 1])
        if s.numel() > 1 and bool(((s[1:] - s[:-1]) / s[1:].abs().clamp_min(1e-30) < rel).any()):
            return True
    return False


def _run_fixture(cuda, name):
    import dvcp
    z = golden(name)
    normals = bool(z["normals"])
    K, r, s, npt = int(z["K"]), float(z["r"]), float(z["s"]), int(z["fe_npoint"])
    model = dvcp.DeepVCP(use_normal=normals, K=K, r=r, s=s, fe_npoint=npt).eval()
    model.load_state_dict(golden_state_dict(z))
    model.to(cuda)
    src, tgt = torch.from_numpy(z["src"]).to(cuda), torch.from_numpy(z["tgt"]).to(cuda)
    R_gt, t_gt = torch.from_numpy(z["R_gt"]).to(cuda), torch.from_numpy(z["t_gt"]).to(cuda)
    tr = {}
    with torch.no_grad():
        kp, vcp = model(src, tgt, R_gt, torch.zeros(1, 3), starts=torch.from_numpy(z["starts"]), trace=tr)
        loss, R, t = dvcp.deepVCP_loss(kp, vcp, R_gt, t_gt, 0.5)
    return z, tr, kp, vcp, loss, R, t


@pytest.mark.parametrize("name", ["e2e_c3small", "e2e_c1"])
def test_e2e_fixture(cuda, name):
    z, tr, kp, vcp, loss, R, t = _run_fixture(cuda, name)
    K = int(z["K"])
    assert torch.equal(tr["src_xyz"].transpose(1, 2).cpu(), torch.from_numpy(z["fe_xyz_src"]))
    assert torch.equal(tr["tgt_xyz"].transpose(1, 2).cpu(), torch.from_numpy(z["fe_xyz_tgt"]))
    torch.testing.assert_close(tr["src_feat"].cpu(), torch.from_numpy(z["fe_feat_src"]), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["tgt_feat"].cpu(), torch.from_numpy(z["fe_feat_tgt"]), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["score"].cpu(), torch.from_numpy(z["score"]), rtol=1e-4, atol=1e-6)
    if _near_tie(torch.from_numpy(z["score"]), K):
        pytest.skip("oracle top-k boundary is a near tie; key-point set legitimately ambiguous")
    # key points: same coordinates (tied duplicate points may swap order, values agree)
    torch.testing.assert_close(kp.cpu(), torch.from_numpy(z["keypts_out"]), rtol=0, atol=0)
    torch.testing.assert_close(tr["src_cat"].cpu(), torch.from_numpy(z["src_cat"]).float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(tr["moved"].cpu(), torch.from_numpy(z["moved"]), rtol=0, atol=1e-12)
    nq = z["knn_idx_head"].shape[1]
    assert torch.equal(tr["knn_idx"][:, :nq].cpu(), torch.from_numpy(z["knn_idx_head"]))
    torch.testing.assert_close(tr["src_dfe"].cpu(), torch.from_numpy(z["src_dfe"]), rtol=1e-4, atol=1e-5)
    B = kp.shape[0]
    torch.testing.assert_close(tr["tgt_dfe"].reshape(B, -1, 32)[:, :nq].cpu(), torch.from_numpy(z["tgt_dfe_head"]),
                               rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(vcp.cpu(), torch.from_numpy(z["vcp"]), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(R.cpu(), torch.from_numpy(z["R"]), rtol=0, atol=1e-4)
    torch.testing.assert_close(t.cpu(), torch.from_numpy(z["t"]), rtol=0, atol=1e-4)
    torch.testing.assert_close(loss.cpu(), torch.from_numpy(z["loss"]), rtol=1e-4, atol=1e-6)


def test_e2e_live_full_size_pair(cuda):
    """One C3 pair at full size (N=16384, K=64, r=2.0, npoint 10000) against the live oracle."""
    import oracle as O
    import dvcp
    from dvcp.synthetic import make_pairs
    from dvcp.synthetic import condition_weights, randomize_bn
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
    if _near_tie(d["wl_score"][..., 0], 64):
        pytest.skip("near-tie at the top-k boundary")
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
