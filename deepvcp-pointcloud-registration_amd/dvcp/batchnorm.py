"""Batch-statistics BatchNorm for the grouped set-abstraction MLP (training mode).

The reference trains the whole model in ``model.train()`` (train.py:105-125), so every
``F.relu(bn(conv(x)))`` of pointnet2_utils.py:195-200 normalises with the statistics of the current
batch over all B * S * nsample grouped entries (BatchNorm2d over (B, H, W); the padding slots of
the ball query are entries like any other) and updates the running statistics (momentum, unbiased
variance), once per FE1 call -- src and tgt are separate calls (deepVCP.py:29,72).

The REF-R tables with fp32 inputs (sa1 3[+3]-16-16-32, sa2, sa3) run on the matrix cores
(csrc/sa_bn_mfma.hip, ``_train_forward_mfma`` / ``_train_backward_mfma``): every pass recomputes
the MLP per 32-entry tile, nothing per entry is stored, and the weight gradients are MFMA products
over the entries.  The rest (fp64 inputs, channel-first feature tables) takes the lane-per-entry
passes below.

Forward (``train_forward``): one statistics pass per layer (dvcp_sa_bn_stats: fp64 sums of z and
z^2, the layers below normalised by their batch statistics), then the eval kernel
(dvcp_sa_group_mlp) with the batch statistics folded into its scale / shift.
Backward (``train_backward``): every entry's conv outputs z_l, written once by the forward's last
statistics pass (64-entry blocks, a few GB per call at C3 -- HBM is 288 GB -- held until the
backward; dvcp_sa_bn_zrows recomputes them when absent), then torch's batch-norm backward,
    dz_l = scale_l (dy_l - mean(dy_l) - xhat_l mean(dy_l xhat_l)),
whose mean terms make every entry's gradient non-zero: sums of the top layer over the routed
(arg-max) rows, one dense pass per lower layer for its sums, and a final dense pass for dW, db and
the per-entry rows of the weight gradients and the feature gradient (dvcp_sa_bn_backward modes
L..1, 0; csrc/sa_bn.hip); dW_l, db_l are then GEMMs over the entries (hipBLASLt via torch.bmm
over the rows' 65536-entry chunks, chunk sums in fp64).
"""
import torch

from . import ops


def _layer_offsets(chans):
    """Per layer (offset, C_in, C_out) in the dvcp_sa_bn pack: W | bias | scale | shift | mean |
    istd | A/M | B/M."""
    offs, o = [], 0
    for cin, cout in zip(chans[:-1], chans[1:]):
        offs.append((o, cin, cout))
        o += cout * cin + 7 * cout
    return offs, o


def _update_running(bn, mean, var, M):
    """BatchNorm2d's running-statistics update in training mode (unbiased variance)."""
    if not bn.track_running_stats:
        return
    with torch.no_grad():
        bn.num_batches_tracked.add_(1)
        f = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
        unbiased = var * (M / max(M - 1, 1))
        bn.running_mean.mul_(1.0 - f).add_(mean.to(bn.running_mean.dtype), alpha=f)
        bn.running_var.mul_(1.0 - f).add_(unbiased.to(bn.running_var.dtype), alpha=f)


# z rows kept from the forward for the backward only up to this size per layer call (bytes); above
# it the backward recomputes them (dvcp_sa_bn_zrows), trading one pass for the memory.
ZROWS_KEEP_MAX_BYTES = 16 << 30


def _bnm_pack(sa, dev):
    offs, total = _layer_offsets(sa.chans)
    parts = []
    for conv, (o, cin, cout) in zip(sa.mlp_convs, offs):
        one, zero = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
        parts += [conv.weight.reshape(-1).float(), conv.bias.float(), one, zero, zero, one, zero, zero]
    pack = torch.cat(parts).contiguous()
    assert pack.numel() == total == ops.sa_bn_pack_floats(sa.chans)
    return pack, offs


def _set_stats(pack, bn, o, cin, cout, sums, M):
    """Batch mean / variance of one layer from its sums; scale, shift, mean, istd into the pack and
    the running-statistics update."""
    mean = sums[0] / M
    var = (sums[1] / M - mean * mean).clamp_min(0.0)
    istd = torch.rsqrt(var + bn.eps)
    scale = bn.weight.double() * istd
    shift = bn.bias.double() - mean * scale
    v = o + cout * cin + cout
    pack[v:v + 4 * cout] = torch.cat([scale, shift, mean, istd]).float()
    _update_running(bn, mean, var, M)


def _train_forward_mfma(sa, xyz, ctr, feat, count, lst, ns):
    """The REF-R tables on the matrix cores (csrc/sa_bn_mfma.hip): (two-layer tables) the
    per-point half of layer 1 once, one statistics pass per layer, then the forward with its
    arg-max routing.  Nothing per entry is kept for the backward; it recomputes the MLP."""
    chans = sa.chans
    B, S = ctr.shape[0], ctr.shape[2]
    M = B * S * ns
    with torch.no_grad():
        pack, offs = _bnm_pack(sa, xyz.device)
        U = ops.sa_bnm_pre(feat, chans, pack) if len(chans) == 3 else None
        for layer, (bn, (o, cin, cout)) in enumerate(zip(sa.mlp_bns, offs), 1):
            sums = ops.sa_bnm_stats(xyz, ctr, feat, count, lst, ns, chans, pack, U, layer)
            _set_stats(pack, bn, o, cin, cout, sums, M)
        fwd = ops.sa_bnm_forward(xyz, ctr, feat, count, lst, ns, chans, pack, U)
    return fwd[0], dict(pack=pack, M=M, U=U, fwd=fwd, mfma=True)


def _train_backward_mfma(sa, lay, g_out, want_feat_grad):
    chans = sa.chans
    offs, _ = _layer_offsets(chans)
    st = lay["bn"]
    pack, M, U, fwd = st["pack"].clone(), st["M"], st["U"], st["fwd"]
    args = (lay["pts"], lay["ctr"], lay["feat"], lay["count"], lay["lst"], lay["ns"], chans)
    g = g_out.float().contiguous()
    out, _, zb = fwd
    L = len(offs)
    sums = [None] * L
    # the last layer's sums over the routed rows (gy = g at each (centre, channel)'s arg-max when
    # the max is positive): A = sum gy, B = sum gy xhat
    o, cin, cout = offs[-1]
    v = o + cout * cin
    mu, istd = pack[v + 3 * cout:v + 4 * cout], pack[v + 4 * cout:v + 5 * cout]
    gy = torch.where(out > 0, g, torch.zeros_like(g)).double()
    xh = ((zb - mu) * istd).double()
    sums[-1] = torch.stack([gy.sum((0, 1)), (gy * xh).sum((0, 1))])
    pack[v + 5 * cout:v + 7 * cout] = (sums[-1] / M).reshape(-1).float()
    for k in range(L - 1, 0, -1):   # each lower layer's sums need those of the layers above
        sums[k - 1] = ops.sa_bnm_backward(*args, pack, U, fwd, g, k)
        o, cin, cout = offs[k - 1]
        v = o + cout * cin
        pack[v + 5 * cout:v + 7 * cout] = (sums[k - 1] / M).reshape(-1).float()
    grads, gF = ops.sa_bnm_backward(*args, pack, U, fwd, g, 0, want_feat_grad=want_feat_grad)
    parts, i = [], 0
    for (o, cin, cout), s in zip(offs, sums):   # per layer dW, db, dgamma, dbeta
        parts += [grads[i:i + cout * cin + cout], s[1], s[0]]
        i += cout * cin + cout
    return torch.cat([p.float() for p in parts]), gF


# The matrix-core path for the tables it takes (tests switch it off to check the VALU passes).
USE_MFMA = True


def train_forward(sa, xyz, ctr, feat, count, lst, ns, keep_zrows=False):
    """pointnet2_utils.py:195-200 with ``sa`` in training mode, on (B, 3, N) points, (B, 3, S)
    centres and (B, D, N) features.  Returns (out (B, S, C_last) fp32, state for the backward).
    ``keep_zrows``: a backward will run (the autograd path), so the last statistics pass also
    writes every entry's z rows for it (within ZROWS_KEEP_MAX_BYTES); a train-mode forward with no
    backward (no_grad, frozen extractor) allocates none."""
    chans = sa.chans
    if USE_MFMA and ops.sa_bnm_usable(xyz, ctr, feat, chans):
        return _train_forward_mfma(sa, xyz, ctr, feat, count, lst, ns)
    dev = xyz.device
    B, S = ctr.shape[0], ctr.shape[2]
    M = B * S * ns
    with torch.no_grad():
        pack, offs = _bnm_pack(sa, dev)
        zrows = None
        keep = keep_zrows and ops.sa_bn_zrows_bytes(B, S, ns, chans) <= ZROWS_KEEP_MAX_BYTES
        for layer, (bn, (o, cin, cout)) in enumerate(zip(sa.mlp_bns, offs), 1):
            if keep and layer == len(offs):  # the last pass also writes every entry's z rows
                sums, zrows = ops.sa_bn_stats(xyz, ctr, feat, count, lst, ns, chans, pack, layer, want_zrows=True)
            else:
                sums = ops.sa_bn_stats(xyz, ctr, feat, count, lst, ns, chans, pack, layer)
            _set_stats(pack, bn, o, cin, cout, sums, M)
        fwd = torch.cat([pack[o:o + cout * cin + 3 * cout] for o, cin, cout in offs]).contiguous()
    out = ops.sa_group_mlp(xyz, ctr, feat, count, lst, ns, chans, fwd)
    return out, dict(pack=pack, M=M, zrows=zrows)


def train_backward(sa, lay, g_out, want_feat_grad):
    """Backward of ``train_forward``: (packed parameter gradient -- per layer dW, db, dgamma,
    dbeta -- and dL/d feat (B, N, D) fp32 or None)."""
    if lay["bn"].get("mfma"):
        return _train_backward_mfma(sa, lay, g_out, want_feat_grad)
    chans = sa.chans
    offs, _ = _layer_offsets(chans)
    st = lay["bn"]
    pack, M = st["pack"].clone(), st["M"]
    args = (lay["pts"], lay["ctr"], lay["feat"], lay["count"], lay["lst"], lay["ns"], chans)
    g = g_out.float().contiguous()
    # every entry's conv outputs with this batch's statistics: written by the forward's last
    # statistics pass (held from the forward to here), else recomputed now
    zrows = st.pop("zrows", None)
    if zrows is None:
        zrows = ops.sa_bn_zrows(*args, st["pack"])
    sums = [None] * len(offs)
    for k in range(len(offs), 0, -1):   # the top layer's sums first: each lower one needs those above
        s = ops.sa_bn_backward(*args, pack, zrows, g, k)
        o, cin, cout = offs[k - 1]
        v = o + cout * cin + 5 * cout
        pack[v:v + 2 * cout] = (s / M).reshape(-1).float()
        sums[k - 1] = s
    rows, gF = ops.sa_bn_backward(*args, pack, zrows, g, 0, want_feat_grad=want_feat_grad)
    del zrows
    parts = []
    for (o, cin, cout), s, (gz, ha) in zip(offs, sums, rows):
        dwb = _gemm_nt(gz, ha)                  # [dW | db] = dz [h; 1]^T over the M entries
        parts += [dwb[:, :cin].reshape(-1), dwb[:, cin], s[1], s[0]]   # dW, db, dgamma, dbeta
    return torch.cat([p.float() for p in parts]), gF


def _gemm_nt(a, b):
    """sum over chunks of a_k @ b_k^T for (nch, m, K) / (nch, n, K) chunked row tables: fp32 GEMMs
    (hipBLASLt via torch.bmm, B transposed by strides, no copy), the chunk products summed in fp64
    in a fixed order."""
    return torch.bmm(a, b.transpose(1, 2)).double().sum(0)
