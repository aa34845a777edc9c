"""Feature extraction layer on the HIP path -- drop-in for deep_feat_extraction.py (REF-R R1).

Three set-abstraction layers (npoint 10000; r 0.1/0.2/0.4; nsample 256/128/64) chained on the
previous layer's features, then ``fc`` 64 -> 32 (deep_feat_extraction.py:10-32 as repaired:
the reference feeds sa2/sa3 the raw normals and never applies ``fc``, which crashes, C1/C2).
"""
import torch
import torch.nn as nn

from . import batchnorm, ops
from ._params import cached_pack, linear_pack, linear_tensors
from .pointnet2_utils import PointNetSetAbstraction


def fe_config(use_normal=True, npoint=10000):
    """deep_feat_extraction.py:10-13 (+R1 channels); npoint defaults to the literal 10000."""
    c_in = 6 if use_normal else 3
    return [
        dict(npoint=npoint, radius=0.1, nsample=256, in_channel=c_in, mlp=[16, 16, 32]),
        dict(npoint=npoint, radius=0.2, nsample=128, in_channel=32 + 3, mlp=[32, 64]),
        dict(npoint=npoint, radius=0.4, nsample=64, in_channel=64 + 3, mlp=[64, 64]),
    ]


class feat_extraction_layer(nn.Module):
    """deep_feat_extraction.py:5-32.  forward(pts (B, C_in, N)) -> (xyz (B, S, 3), feat (B, S, 32))."""

    def __init__(self, use_normal=True, npoint=10000):
        super().__init__()
        self.use_normal = use_normal
        cfg = fe_config(use_normal, npoint)
        self.sa1 = PointNetSetAbstraction(**cfg[0])
        self.sa2 = PointNetSetAbstraction(**cfg[1])
        self.sa3 = PointNetSetAbstraction(**cfg[2])
        self.fc = nn.Linear(64, 32)
        # workgroups per cloud of the FPS select rounds (None: ops.fps_parts, one unless
        # DVCP_FPS_PARTS says otherwise); see DeepVCP(fps_parts=...)
        self.fps_parts = None

    def fc_params(self, wl=None):
        lins = [self.fc] + ([wl.fc1[0], wl.fc2[0], wl.fc3[0]] if wl is not None else [])
        return cached_pack(self, "head" if wl is None else "head_wl", linear_tensors(*lins),
                           lambda: linear_pack(*lins))

    def launch_fps(self, pts, starts, stream):
        """The serial FPS chain of ``run`` (it depends on the coordinates alone) enqueued on
        ``stream``, for ``run(..., fps=...)``: a caller with two clouds starts the second cloud's
        chain while the first one's layers run (extract_features in training mode).  ->
        (indices, centres, events recorded on ``stream``)."""
        xyz = pts[:, :3, :] if self.use_normal else pts
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            return self._fps_chain(xyz, starts, stream)

    def _fps_chain(self, xyz, starts, stream):
        """The three FPS launches on ``stream`` (the current stream): -> (indices, centres, an
        event per layer recorded after its centres exist).  Layers 2 and 3 pick every point of
        their input (npoint = its point count, C3): one paired launch (ops.fps_pair) runs layer 3
        beside layer 2, and both layers' events are the pair's."""
        layers = (self.sa1, self.sa2, self.sa3)
        idxs, centres, events = [], [], []
        prev = xyz
        li = 0
        errs = None
        while li < 3:
            sa, st = layers[li], starts[li]
            if li == 1 and ops.fps_pair_ok(prev, sa.npoint, layers[2].npoint, pdim=2):
                i2, c2, i3, c3 = ops.fps_pair(prev, st.to(prev.device), starts[2].to(prev.device), pdim=2)
                ev = torch.cuda.Event()
                ev.record(stream)
                idxs += [i2, i3]
                centres += [c2, c3]
                events += [ev, ev]
                break
            if errs is None and ops.fps_uses_guard(prev, pdim=2, parts=self.fps_parts):
                # the guards' error words of the chain's split launches: one zeroed buffer
                errs = torch.zeros(3, dtype=torch.int32, device=prev.device)
            i, c = ops.fps(prev, sa.npoint, st.to(prev.device), pdim=2, parts=self.fps_parts,
                           err=errs[li:li + 1] if errs is not None and ops.fps_uses_guard(prev, 2, self.fps_parts)
                           else None)
            idxs.append(i)
            centres.append(c)
            ev = torch.cuda.Event()
            ev.record(stream)
            events.append(ev)
            prev = c
            li += 1
        return idxs, centres, events

    def run(self, pts, starts=None, wl=None, side_stream=None, saved=None, fps=None, layer_trace=None):
        """Fused forward.  starts: (3, B) FPS start indices (drawn like the reference if None).
        Returns xyz (B, 3, S) contiguous, feat (B, S, 32), score (B, S) when ``wl`` is given.
        ``saved`` (a dict): filled with what the backward needs (dvcp/autograd.py feat_extraction):
        per layer its points, centres, input features, ball-query lists and FPS indices, and the
        fc input rows.

        FPS of layer l+1 depends only on layer l's sampled centres, not on its features, so the
        FPS launches (the serial critical path; layers 2 and 3 as one paired launch where both
        pick every point, see ``_fps_chain``) run back to back on the current stream
        while each layer's ball query + grouped MLP runs on ``side_stream``.  A layer whose FPS
        picks every point (npoint >= its point count, layers 2 and 3 of the reference) is
        evaluated per point before its FPS finishes and gathered by the FPS order.

        In training mode (``self.training``) the set-abstraction BatchNorms use batch statistics
        over this call's grouped entries and update their running statistics (dvcp/batchnorm.py);
        every layer is then evaluated on its FPS centres (the statistics are over the centres).

        ``layer_trace`` (a list, parity tests): gets one dict per layer -- its FPS indices ``idx``,
        the ball query's distinct-hit ``count`` / ``lst`` and ``per_point`` (lists are then per
        point, to be read through ``idx``; else per FPS centre)."""
        train_bn = self.training
        B, _, N = pts.shape
        if self.use_normal:
            xyz, feat = pts[:, :3, :], pts[:, 3:, :]
        else:
            xyz, feat = pts, None
        if starts is None:
            starts = [torch.randint(0, n, (B,), dtype=torch.long)
                      for n in (N, self.sa1.npoint, self.sa2.npoint)]
        layers = (self.sa1, self.sa2, self.sa3)
        main = torch.cuda.current_stream()
        side = side_stream if side_stream is not None else main
        if side is not main:
            # the side stream reads the input points (for a per-point first layer before any FPS
            # event): it starts after the main stream's work so far (the 2B-cloud cat of
            # extract_features, a caller's uploads) -- not after the FPS chain enqueued next.  This
            # also joins it to a graph capture.
            ready = torch.cuda.Event()
            ready.record(main)
            side.wait_event(ready)
        if fps is not None:  # launched ahead on another stream (launch_fps)
            idxs, centres, events = fps
            for i, c in zip(idxs, centres):  # (the side stream waits for each layer's event)
                for t in (i, c):
                    t.record_stream(main)
                    t.record_stream(side)
        else:
            idxs, centres, events = self._fps_chain(xyz, starts, main)
        # Inference folds the gathers of per-point layers into their consumers: the next layer's
        # MLP reads its features through the FPS indices (dvcp_sa_group_mlp_rows_ws) and the head
        # reads sa3's rows the same way (dvcp_fe_head_rows).  Training (``saved``) keeps the
        # gathered tables, which its backward consumes.
        fold = saved is None and not train_bn
        with torch.cuda.stream(side):
            pts_l, f = xyz, feat
            f_rows = None  # (per-point table (B, Nf, C), FPS indices (B, n_l)): f is that gather
            for sa, i, c, ev in zip(layers, idxs, centres, events):
                n_l = pts_l.shape[2]
                ns = min(int(sa.nsample), n_l)
                per_point = sa.npoint >= n_l and not train_bn
                ctr_l = pts_l if per_point else c
                if not per_point:
                    side.wait_event(ev)
                # Every point of a layer with npoint >= n_l becomes a centre (FPS output = a
                # permutation, with repeats if npoint > n_l), and a centre's group and MLP depend
                # only on its coordinates and the layer's point set.  So evaluate every point as its
                # own centre now -- concurrently with this layer's FPS on the main stream -- and
                # take the rows in FPS order once the indices exist.  Bit-identical results.
                count, lst, _ = ops.ball_query(pts_l, ctr_l, sa.radius, ns, pdim=2, cdim_pts=2)
                bn_state = None
                if train_bn:
                    res, bn_state = batchnorm.train_forward(sa, pts_l, ctr_l, f, count, lst, ns,
                                                            keep_zrows=saved is not None)
                elif f_rows is not None:
                    res = ops.sa_group_mlp_rows(pts_l, ctr_l, f_rows[0], f_rows[1], count, lst, ns, sa.chans,
                                                sa.packed_params())
                else:
                    res = ops.sa_group_mlp(pts_l, ctr_l, f, count, lst, ns, sa.chans, sa.packed_params(),
                                           xyz_pdim=2, feat_ddim=1, feat_pdim=2)
                f_rows = None
                if per_point:
                    side.wait_event(ev)
                    i.record_stream(side)
                    if fold:
                        f_rows = (res, i)
                        out = None
                    else:
                        out = torch.gather(res, 1, i.unsqueeze(-1).expand(-1, -1, res.shape[2]))
                else:
                    out = res
                if layer_trace is not None:
                    layer_trace.append(dict(idx=i, count=count, lst=lst, per_point=per_point, n=n_l))
                if saved is not None:
                    saved.setdefault("layers", []).append(dict(pts=pts_l, ctr=ctr_l, feat=f, count=count, lst=lst,
                                                               ns=ns, idx=i, per_point=per_point, bn=bn_state))
                c.record_stream(side)
                pts_l, f = c, (out.permute(0, 2, 1) if out is not None else None)
            S = pts_l.shape[2]
            if f_rows is not None:
                f3 = None
                head, score = ops.fe_head_rows(f_rows[0], f_rows[1], self.fc_params(wl), with_score=wl is not None)
            else:
                f3 = f.permute(0, 2, 1).reshape(B * S, 64)  # sa output is (B, S, 64) in memory
                head, score = ops.fe_head(f3, self.fc_params(wl), with_score=wl is not None)
        if saved is not None:
            saved["f3"] = f3
        if side is not main:
            main.wait_stream(side)
            keep = [head, score]
            if saved is not None:
                keep += [saved["f3"]] + [t for lay in saved["layers"] for t in lay.values() if torch.is_tensor(t)]
                # the training-BN state (dvcp/batchnorm.py) nests its tensors one level down (the
                # pack is read on the main stream by the backward's z-row pass)
                keep += [t for lay in saved["layers"] if isinstance(lay.get("bn"), dict)
                         for t in lay["bn"].values() if torch.is_tensor(t)]
            for t in keep:
                if t is not None:
                    t.record_stream(main)  # allocated on the side stream, consumed on main
        return pts_l, head.view(B, S, 32), (score.view(B, S) if score is not None else None)

    def forward(self, pts):
        """deep_feat_extraction.py:18-32.  With gradients enabled and a trainable parameter the
        call is differentiable in FE1's parameters (dvcp.autograd.feat_extraction; BatchNorm in this
        module's mode, batch statistics when training), so ``model.FE1(pts)`` in a training loop
        back-propagates like the reference's; otherwise the inference path."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from . import autograd
            xyz, feat, _ = autograd.feat_extraction(self, pts, None)
        else:
            xyz, feat, _ = self.run(pts)
        return xyz.permute(0, 2, 1), feat
