"""numpy restatement of the paper-faithful pose solve (test infrastructure only: the checker for
dvcp.paper / dvcp_paper_pose).  DeepVCP paper (Lu et al., ICCV 2019) Sec. 3.4-3.5: weighted
Kabsch with the key points' weights, reflection-corrected, and the two-term L1 loss.  There is
no reference implementation of it (the repository's deepVCP_loss.py:13-44 is unweighted with no
reflection fix), so this restatement is "parity unpinned" against the reference and pinned by
its own known-answer cases (tests/test_oracle_kat.py)."""
import numpy as np


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


def deepvcp_loss_paper(x, y, w, R_true, t_true, alpha=0.5, reflection_fix=True):
    """x, y (B, 3, n), w (B, n) or None -> (loss, R (B,3,3), t (B,3))."""
    Rs, ts, s1, s2, cnt = [], [], 0.0, 0.0, 0
    for b in range(x.shape[0]):
        R, t = weighted_rigid_transform(x[b], y[b], None if w is None else w[b], reflection_fix)
        ygt = R_true[b] @ x[b] + t_true[b].reshape(3, 1)
        s1 += np.abs(ygt - y[b]).sum()
        s2 += np.abs(ygt - (R @ x[b] + t.reshape(3, 1))).sum()
        cnt += x[b].size
        Rs.append(R)
        ts.append(t)
    return alpha * s1 / cnt + (1 - alpha) * s2 / cnt, np.stack(Rs), np.stack(ts)
