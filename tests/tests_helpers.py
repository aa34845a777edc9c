"""Small helpers shared by the tests (no product code)."""
import os

import numpy as np
import torch

from conftest import GOLDEN


def randomize_bn(model, seed=5):
    """Non-trivial eval-mode BatchNorm statistics (same recipe as tests/golden/make_golden.py)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                n = m.num_features
                m.weight.copy_(torch.rand(n, generator=g) + 0.5)
                m.bias.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_mean.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_var.copy_(torch.rand(n, generator=g) + 0.5)


def topk_parity(got_idx, got_score, want_idx, want_score, K, band_factor=4.0):
    """Per-rank top-k parity against the oracle (SURVEY.md 8(c) fixture 4's near-tie rule,
    applied rank by rank instead of to the whole list).

    The oracle's scores are ranked; the boundary between ranks i and i+1 (i < K, rank K being
    the first score left out) is *ambiguous* when their score gap is below ``band_factor`` x
    the measured GPU-vs-oracle score difference over the oracle's top 2K rows -- there the
    two fp32 pipelines may legitimately order the rows differently.  Ranks joined by ambiguous
    boundaries form blocks:
      * a rank with clear gaps on both sides must hold exactly the oracle's index;
      * a block inside the top K must hold the same set of indices as the oracle's block;
      * a block that reaches the K-th boundary must hold rows whose oracle score lies within
        the block's score range (widened by the band).
    Asserts those rules for every row; returns (exact, n_ambiguous) where ``exact`` says the
    whole (B, K) index sequence equals the oracle's (then the GPU's own top-k feeds the
    back half with no caveat)."""
    got_idx, want_idx = got_idx.cpu().long(), want_idx.cpu().long()
    got_score, want_score = got_score.cpu().double(), want_score.cpu().double()
    n_amb = 0
    for b in range(want_idx.shape[0]):
        ws, gs = want_score[b], got_score[b]
        order = torch.sort(ws, descending=True, stable=True).indices
        top2k = order[: 2 * K]
        noise = float((gs[top2k] - ws[top2k]).abs().max())
        band = band_factor * noise
        v = ws[want_idx[b]]                                   # oracle scores in oracle rank order
        v_next = float(ws[order[K]]) if ws.numel() > K else -float("inf")
        vals = torch.cat([v, torch.tensor([v_next], dtype=torch.float64)])
        amb = (vals[:-1] - vals[1:]) < band                   # boundary i | i+1 ambiguous
        n_amb += int(amb.sum())
        i = 0
        while i < K:
            j = i
            while j < K and bool(amb[j]):
                j += 1                                        # block = ranks i..j (j <= K)
            if j == i:
                assert int(got_idx[b, i]) == int(want_idx[b, i]), (b, i)
            elif j < K:
                assert set(got_idx[b, i:j + 1].tolist()) == set(want_idx[b, i:j + 1].tolist()), (b, i, j)
            else:
                lo, hi = float(vals[K]) - band, float(vals[i]) + band
                sc = ws[got_idx[b, i:K]]
                assert bool(((sc >= lo) & (sc <= hi)).all()), (b, i)
            i = j + 1
    return bool(torch.equal(got_idx, want_idx)), n_amb


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def golden_state_dict(z):
    return {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w::")}


def ball_rows_mismatch_ok(xyz, ctr, got, want, radius, ulps=4):
    """Ball-query rows (B, S, ns) that differ may only differ by points whose d2 sits within
    ``ulps`` of radius^2 (the oracle's BLAS-rounded square_distance against the kernel's
    restatement of it); d2 is formed for the differing rows only, so full-size layers stay cheap.
    Returns the number of differing rows (asserts the rule)."""
    import oracle as O
    bad = (got != want).any(-1)
    if not bad.any():
        return 0
    r2 = float(torch.tensor(radius ** 2, dtype=xyz.dtype))
    tol = ulps * torch.finfo(xyz.dtype).eps * r2
    for b, s in bad.nonzero().tolist():
        d2 = O.square_distance(ctr[b:b + 1, s:s + 1], xyz[b:b + 1])[0, 0]
        for n in set(got[b, s].tolist()) ^ set(want[b, s].tolist()):
            assert n < xyz.shape[1] and abs(float(d2[n]) - r2) <= tol, (b, s, n, float(d2[n]), r2)
    return int(bad.sum())


def padded_ball_rows(layer, c):
    """GPU FE layer trace (dvcp feat_extraction_layer.run(layer_trace=...)) -> cloud c's ball-query
    rows in the reference's padded form (S, ns) int64, one row per FPS centre in FPS order."""
    idx = layer["idx"][c].cpu()
    cnt = layer["count"][c].cpu().long()
    lst = layer["lst"][c].cpu().long()
    if layer["per_point"]:
        cnt, lst = cnt[idx], lst[idx]
    col = torch.arange(lst.shape[1])
    return torch.where(col[None, :] < cnt[:, None], lst, lst[:, :1])
