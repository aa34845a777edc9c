"""Autograd for the registration head: training drop-in for train.py:105-125.

The reference trains with ``loss.backward()`` through deepVCP_loss (two torch.svd), the corresponding
point generation (cpg.py), the deep feature embedding (deep_feat_embedding.py, src and tgt) and the
feature extractor.  Here the head's backward runs in hand-written HIP kernels:

  * ``pose_loss``  -- deepVCP_loss.py:105-121 forward (dvcp_svd_optimization) and backward
                      (dvcp_svd_optimization_backward, both Kabsch solves differentiated);
  * ``cpg``        -- cpg.py:27-60 (dvcp_cpg / dvcp_cpg_backward): gradients for the conv
                      weights and for both DFE outputs;
  * ``dfe_rows``   -- deep_feat_embedding.py on the source rows (dvcp_dfe / dvcp_dfe_backward);
  * ``dfe_tgt``    -- the fused target rows (dvcp_dfe_tgt / dvcp_dfe_tgt_backward), also
                      differentiable in the target features (the get_cat_feat_tgt.py:85 gather);
  * ``src_keypoints`` -- the key-point stage, differentiable in the source features (the
                      pointnet2_utils.py:59 gather, dvcp_src_keypoints_backward).

  * ``feat_extraction`` -- the feature extractor (deep_feat_extraction.py:18-32 + REF-R R1): fc
                      (dvcp_fe_head_backward) and the three set-abstraction MLPs, chained through the
                      FPS-order gathers and the ball-query groupings.  BatchNorm in eval mode
                      (frozen-BN training, FE1.eval()): dvcp_sa_group_mlp_backward; in training mode
                      (batch statistics, model.train() as train.py does): dvcp_sa_bn_backward
                      (dvcp/batchnorm.py).

The key points, candidates and kNN indices carry no gradient in the reference either (index
ops, knn_cuda under no_grad); the weighting layer gets none (only its top-k indices are used).
Parameter gradients come back summed over
the batch in a fixed order (deterministic); the feature scatters use float atomics.
"""
import torch

from . import batchnorm, ops


def _pack(weights):
    return torch.cat([w.detach().reshape(-1) for w in weights]).float().contiguous()


def _split(gp, weights):
    """Packed gradient -> one tensor per (shape, dtype) in ``weights``."""
    out, o = [], 0
    for shape, dtype in weights:
        n = shape.numel()
        out.append(gp[o:o + n].view(shape).to(dtype))
        o += n
    return out


class _DfeRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, *weights):
        params = _pack(weights)
        ctx.save_for_backward(X, params)
        ctx.weights = [(w.shape, w.dtype) for w in weights]
        return ops.dfe(X, params)

    @staticmethod
    def backward(ctx, g):
        X, params = ctx.saved_tensors
        if ctx.needs_input_grad[0]:
            gp, gX = ops.dfe_backward(X, params, g, want_input_grad=True)
            return (gX.to(X.dtype), *_split(gp, ctx.weights))
        return (None, *_split(ops.dfe_backward(X, params, g), ctx.weights))


class _DfeTgt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ref_xyz, ref_feat, cand, dist, idx, *weights):
        params = _pack(weights)
        ctx.save_for_backward(ref_xyz, ref_feat, cand, dist, idx, params)
        ctx.weights = [(w.shape, w.dtype) for w in weights]
        return ops.dfe_tgt(ref_xyz, ref_feat, cand, dist, idx, params, ref_pdim=2)

    @staticmethod
    def backward(ctx, g):
        ref_xyz, ref_feat, cand, dist, idx, params = ctx.saved_tensors
        if ctx.needs_input_grad[1]:  # the get_cat_feat_tgt.py:85 gather's backward
            gp, gF = ops.dfe_tgt_backward(ref_xyz, ref_feat, cand, dist, idx, params, g, ref_pdim=2,
                                          want_feat_grad=True)
            return (None, gF.to(ref_feat.dtype), None, None, None, *_split(gp, ctx.weights))
        gp = ops.dfe_tgt_backward(ref_xyz, ref_feat, cand, dist, idx, params, g, ref_pdim=2)
        return (None, None, None, None, None, *_split(gp, ctx.weights))


class _Cpg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, tgt, cand, G, *weights):
        params = _pack(weights)
        ctx.save_for_backward(src, tgt, cand, params)
        ctx.G = G
        ctx.weights = [(w.shape, w.dtype) for w in weights]
        return ops.cpg(src, tgt, cand, G, params)

    @staticmethod
    def backward(ctx, g):
        src, tgt, cand, params = ctx.saved_tensors
        gsrc, gtgt, gp = ops.cpg_backward(src, tgt, cand, ctx.G, params, g)
        gsrc = gsrc.view(src.shape).to(src.dtype) if ctx.needs_input_grad[0] else None
        gtgt = gtgt.to(tgt.dtype) if ctx.needs_input_grad[1] else None
        return (gsrc, gtgt, None, None, *_split(gp, ctx.weights))


class _SrcKeypoints(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fe_xyz, fe_feat, topk_idx, kstart, R_init, radius, nsample):
        keypts, src_cat, moved = ops.src_keypoints(fe_xyz, fe_feat, topk_idx, kstart, R_init, radius=radius,
                                                   nsample=nsample)
        ctx.save_for_backward(fe_xyz, topk_idx, kstart)
        ctx.radius, ctx.nsample, ctx.feat_dtype = radius, nsample, fe_feat.dtype
        ctx.mark_non_differentiable(keypts, moved)
        return keypts, src_cat, moved

    @staticmethod
    def backward(ctx, g_kp, g_cat, g_moved):
        fe_xyz, topk_idx, kstart = ctx.saved_tensors
        gF = None
        if ctx.needs_input_grad[1] and g_cat is not None:
            gF = ops.src_keypoints_backward(fe_xyz, topk_idx, kstart, g_cat, radius=ctx.radius,
                                            nsample=ctx.nsample).to(ctx.feat_dtype)
        return None, gF, None, None, None, None, None


class _PoseLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y_pred, R_true, t_true, alpha):
        x, y, Rt, tt = ops.pose_inputs(x, y_pred, R_true, t_true)
        R, t, x1, _, partial = ops.svd_optimization(x, y, Rt, tt)
        denom = float(x1.numel())
        loss = alpha * (partial[:, 0].sum() / denom) + (1 - alpha) * torch.abs(partial[:, 1].sum() / denom)
        ctx.save_for_backward(x, y, Rt, tt, partial)
        ctx.alpha = alpha
        ctx.y_dtype = y_pred.dtype
        ctx.mark_non_differentiable(R, t)
        return loss, R, t

    @staticmethod
    def backward(ctx, g_loss, g_R, g_t):
        x, y, Rt, tt, partial = ctx.saved_tensors
        gy = ops.svd_optimization_backward(x, y, Rt, tt, partial, g_loss, ctx.alpha)
        return None, gy.to(ctx.y_dtype), None, None, None


def _fe_params(fe):
    """FE1's trainable tensors in a fixed order: per SA layer (conv.weight, conv.bias, bn.weight,
    bn.bias) per MLP layer, then fc.weight, fc.bias."""
    out = []
    for sa in (fe.sa1, fe.sa2, fe.sa3):
        for conv, bn in zip(sa.mlp_convs, sa.mlp_bns):
            out += [conv.weight, conv.bias, bn.weight, bn.bias]
    return out + [fe.fc.weight, fe.fc.bias]


def _bn_stats(sa):
    """Per MLP layer: running_mean | 1 / sqrt(running_var + eps) (fp32), the eval-mode BN's
    normalisation for the gamma gradient."""
    parts = []
    for bn in sa.mlp_bns:
        parts += [bn.running_mean.float(), torch.rsqrt(bn.running_var.double() + bn.eps).float()]
    return torch.cat(parts).contiguous()


def _scatter_rows(g, idx, n):
    """The backward of gathering per-point rows by FPS indices: (B, S, C) -> (B, n, C)."""
    out = torch.zeros(g.shape[0], n, g.shape[2], dtype=torch.float32, device=g.device)
    return out.scatter_add_(1, idx.unsqueeze(-1).expand(-1, -1, g.shape[2]), g.float())


class _FeatExtract(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fe, pts, starts, wl, side_stream, fps, *params):
        saved = {}
        xyz, feat, score = fe.run(pts, starts, wl=wl, side_stream=side_stream, saved=saved, fps=fps)
        ctx.fe, ctx.saved = fe, saved
        ctx.shapes = [(p.shape, p.dtype) for p in params]
        ctx.mark_non_differentiable(xyz)
        if score is not None:
            ctx.mark_non_differentiable(score)
        return xyz, feat, score

    @staticmethod
    def backward(ctx, g_xyz, g_feat, g_score):
        fe, saved = ctx.fe, ctx.saved
        grads = []
        if g_feat is None:
            return (None,) * 6 + tuple(None for _ in ctx.shapes)
        B, S, _ = g_feat.shape
        gp_fc, g = ops.fe_head_backward(saved["f3"], fe.fc_params(), g_feat.reshape(B * S, 32))
        g = g.view(B, S, 64)
        per_layer = []
        for sa, lay in reversed(list(zip((fe.sa1, fe.sa2, fe.sa3), saved["layers"]))):
            n_l = lay["pts"].shape[2]
            g_out = _scatter_rows(g, lay["idx"], n_l) if lay["per_point"] else g
            first = sa is fe.sa1
            if lay["bn"] is not None:   # training-mode BN: batch statistics (dvcp/batchnorm.py)
                gp, g_in = batchnorm.train_backward(sa, lay, g_out, want_feat_grad=not first)
            else:
                gp, g_in = ops.sa_group_mlp_backward(lay["pts"], lay["ctr"], lay["feat"], lay["count"], lay["lst"],
                                                     lay["ns"], sa.chans, sa.packed_params(), _bn_stats(sa), g_out,
                                                     want_feat_grad=not first)
            per_layer.append((sa, gp))
            g = g_in  # (B, n_l, D): the previous layer's outputs, in its centre order
        for sa, gp in reversed(per_layer):
            o = 0
            for conv, bn in zip(sa.mlp_convs, sa.mlp_bns):
                co, ci = conv.weight.shape[0], conv.weight.shape[1]
                grads += [gp[o:o + co * ci].view(conv.weight.shape), gp[o + co * ci:o + co * ci + co],
                          gp[o + co * ci + co:o + co * ci + 2 * co], gp[o + co * ci + 2 * co:o + co * ci + 3 * co]]
                o += co * ci + 3 * co
        grads += [gp_fc[:32 * 64].view(32, 64), gp_fc[32 * 64:]]
        ctx.saved = None
        out = [gr.to(dt) if ctx.needs_input_grad[6 + k] else None for k, (gr, (_, dt)) in enumerate(zip(grads, ctx.shapes))]
        return (None, None, None, None, None, None, *out)


def feat_extraction(fe, pts, starts, wl=None, side_stream=None, fps=None):
    """FE1.run differentiable in FE1's parameters (BN in FE1's mode): -> (xyz, feat, score).
    ``fps``: the FPS chain launched ahead (FE1.launch_fps)."""
    return _FeatExtract.apply(fe, pts, starts, wl, side_stream, fps, *_fe_params(fe))


def dfe_rows(X, dfe_module):
    """deep_feat_embedding.py forward on materialised rows (..., 32, 35), differentiable in fc1-3."""
    return _DfeRows.apply(X, *_linears(dfe_module))


def dfe_tgt(ref_xyz, ref_feat, cand, dist, idx, dfe_module):
    """The fused target rows (get_cat_feat_tgt.py + deep_feat_embedding.py), differentiable in fc1-3."""
    return _DfeTgt.apply(ref_xyz, ref_feat, cand, dist, idx, *_linears(dfe_module))


def cpg(src, tgt, cand, G, cpg_module):
    """cpg.py:27-60, differentiable in src, tgt and the conv weights."""
    convs = [cpg_module.conv1, cpg_module.conv2, cpg_module.conv3]
    return _Cpg.apply(src, tgt, cand, G, *[t for c in convs for t in (c.weight, c.bias)])


def src_keypoints(fe_xyz, fe_feat, topk_idx, kstart, R_init, radius=1.0, nsample=32):
    """The key-point stage (deepVCP.py:39-68 + get_cat_feat_src.py), differentiable in fe_feat
    through the index_points gather (pointnet2_utils.py:59) and the distance weighting."""
    return _SrcKeypoints.apply(fe_xyz, fe_feat, topk_idx, kstart, R_init, radius, nsample)


def pose_loss(x, y_pred, R_true, t_true, alpha):
    """deepVCP_loss.py:105-121 on (B, 3, n) operands -> (loss, R, t); differentiable in y_pred."""
    return _PoseLoss.apply(x, y_pred, R_true, t_true, alpha)


def _linears(m):
    return [m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias, m.fc3.weight, m.fc3.bias]
