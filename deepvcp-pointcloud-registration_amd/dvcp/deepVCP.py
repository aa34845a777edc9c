"""DeepVCP on the HIP path -- drop-in for deepVCP.py:16-110 (REF-R semantics).

Same constructor, submodule names (FE1, WL, DFE, cpg) and state_dict keys as the reference
(with the R1 shape changes of FE1.sa2/sa3), same forward signature and outputs:

    forward(src_pts (B, C_in, N), tgt_pts (B, C_in, N), R_init (B|1, 3, 3) fp64, t_init)
        -> (src_keypts (B, K, 3), tgt_vcp (B, K, 3) fp32)

Pipeline (every stage a gfx950 HIP kernel; the set abstractions' ball queries and tables and the
source rows' DFE run on a side stream beside the FPS chain / the target side of the head):
    FE(src) [fps, ball query, grouped MLP x3, fc + weighting] -> top-K
    -> key-point stage [gather, FPS among key points, ball query, Get_Cat_Feat_Src, R_init]
    -> DFE(src) -> FE(tgt) -> candidate grid -> kNN(k=32) -> fused gather + DFE(tgt) -> CPG.
The seven FPS start indices are drawn up front with torch.randint on the CPU generator in the
reference's order (src sa1, sa2, sa3, key points, tgt sa1, sa2, sa3), so a seeded run draws the
same starts as the reference.  t_init is unused, as in the reference (deepVCP.py:86).
"""
import warnings

import torch
import torch.nn as nn

from . import _lib, autograd, ops
from .cpg import cpg
from .deep_feat_embedding import feat_embedding_layer
from .deep_feat_extraction import feat_extraction_layer
from .pointnet2_utils import _inference_only
from .voxelize import grid_side
from .weighting_layer import weighting_layer


_F16_WARNED = False


def _warn_f16_autograd():
    """feat_dtype=float16 is an inference storage format (dvcp_dfe_tgt_f16); the autograd path
    gathers the fp32 table, so say so once instead of silently ignoring it."""
    global _F16_WARNED
    if not _F16_WARNED:
        _F16_WARNED = True
        warnings.warn("dvcp.DeepVCP(feat_dtype=torch.float16) applies to inference (torch.no_grad()) only; "
                      "this forward records autograd and uses the fp32 target feature table", RuntimeWarning,
                      stacklevel=3)


class DeepVCP(nn.Module):
    def __init__(self, use_normal, K=64, r=1.0, s=0.4, fe_npoint=10000, feat_dtype=torch.float32, dfe_literal=False,
                 fps_parts=None):
        """``feat_dtype``: storage of the target feature table the fused target stage gathers
        (torch.float16: BASELINE C5's "fp16 features", dvcp_dfe_tgt_f16; inference only -- the
        reference keeps fp32 features, so float16 is not reference precision).
        ``dfe_literal``: the fused target DFE chains fc1, fc2, fc3 as written (dvcp_dfe_tgt_literal,
        SURVEY App. A.3 Q14) instead of the collapsed 32x35 map (dvcp_dfe_tgt, the default: fc3.fc2.fc1
        formed in fp64 and rounded once; the same within 1e-7 on the tests).
        ``fps_parts``: workgroups per cloud of the feature extractor's FPS select rounds (1, 2, 4 or 8;
        None: ops.fps_parts -- one up to 16384 points, eight above, or DVCP_FPS_PARTS).  More workgroups shorten a lone batch's FPS chain (the split
        select, csrc/fps.hip FpsPartArgs: the same indices); with many batches in flight the CU time
        they take costs more pairs/s than the shorter chain gains, so one is the default below
        16384 points."""
        super().__init__()
        self.dfe_literal = bool(dfe_literal)
        if feat_dtype not in (torch.float32, torch.float16):
            raise ValueError(f"feat_dtype must be torch.float32 or torch.float16, got {feat_dtype}")
        self.feat_dtype = feat_dtype
        self.FE1 = feat_extraction_layer(use_normal=use_normal, npoint=fe_npoint)
        self.FE1.fps_parts = fps_parts
        self.WL = weighting_layer()
        self.DFE = feat_embedding_layer()
        self.cpg = cpg()
        self.K, self.r, self.s = K, r, s

    def _side_stream(self, dev):
        """The FE side stream paired with the calling stream (independent batches issued on
        different streams keep independent side streams, so they overlap)."""
        cache = self.__dict__.setdefault("_dvcp_streams", {})
        key = (dev, torch.cuda.current_stream(dev).cuda_stream)
        if key not in cache:
            cache[key] = torch.cuda.Stream(device=dev)
        return cache[key]

    def _fps_stream(self, dev):
        """A second stream per calling stream, for an FPS chain launched ahead (FE1.launch_fps)."""
        cache = self.__dict__.setdefault("_dvcp_fps_streams", {})
        key = (dev, torch.cuda.current_stream(dev).cuda_stream)
        if key not in cache:
            cache[key] = torch.cuda.Stream(device=dev)
        return cache[key]

    def _training_mode(self):
        """(train_head, train_fe) for this forward (train.py:105-125).  Autograd records through
        the head (DFE, CPG) when it is enabled and any head or extractor parameter requires
        gradients; through the feature extractor when its parameters require gradients.  FE1's
        BatchNorm follows FE1's mode like torch's: batch statistics (and running-statistics
        updates) in training mode, running statistics after FE1.eval() (frozen-BN fine-tuning).

        This follows autograd, not ``eval()``: ``model.eval()`` followed by a forward WITHOUT
        ``torch.no_grad()`` (parameters trainable, the torch default) records the autograd path,
        as the reference's modules would -- every saved table stays alive until the graph is freed
        and the inference path's folded gathers are not used.  Inference belongs under
        ``torch.no_grad()`` (train.py's test loop, vis_utils.py:85)."""
        head = [p for m in (self.DFE, self.cpg) for p in m.parameters()]
        fe_grad = any(p.requires_grad for p in self.FE1.parameters())
        grad = torch.is_grad_enabled()
        train_fe = grad and fe_grad
        train_head = grad and (any(p.requires_grad for p in head) or train_fe)
        if not train_head and self.training:
            raise NotImplementedError("dvcp.DeepVCP: training mode with autograd disabled or no trainable parameter")
        if not train_head:
            _inference_only(self)
        return train_head, train_fe

    def draw_starts(self, B, n_src, n_tgt):
        """The reference's seven torch.randint(0, n, (B,)) draws, in call order."""
        S1, S2, S3 = self.FE1.sa1.npoint, self.FE1.sa2.npoint, self.FE1.sa3.npoint
        sizes = (n_src, S1, S2, self.K, n_tgt, S1, S2)
        del S3
        return torch.stack([torch.randint(0, n, (B,), dtype=torch.long) for n in sizes])

    def extract_features(self, src_pts, tgt_pts, starts=None, train_fe=False, trace=None):
        """The feature-extractor half of forward (deepVCP.py:29,72 -- FE1 on both clouds, the
        weighting layer's scores): a dict the head half (``forward_head``) consumes.  It depends on
        no trainable head parameter, so with the extractor frozen a training loop can run it for
        upcoming batches on other streams while the current batch's head trains
        (tools/train_step_bench.py --prefetch)."""
        _lib.require_gpu(src_pts, tgt_pts)   # no CPU fallback
        B = src_pts.shape[0]
        dev = src_pts.device
        if starts is None:
            starts = self.draw_starts(B, src_pts.shape[2], tgt_pts.shape[2])
        one_pass = src_pts.shape == tgt_pts.shape and src_pts.dtype == tgt_pts.dtype and not self.FE1.training
        fe_starts = None
        if one_pass and starts.device.type == "cpu":
            # the 2B-cloud pass's start rows (src then tgt per layer) formed on the host and
            # uploaded with the seven draws in one copy (no per-layer concatenation on the GPU)
            fe = torch.stack([torch.cat([starts[i], starts[4 + i]]) for i in range(3)])
            both_rows = torch.cat([starts.reshape(-1), fe.reshape(-1)]).to(dev, non_blocking=True)
            starts = both_rows[:7 * B].view(7, B)
            fe_starts = list(both_rows[7 * B:].view(3, 2 * B))
        else:
            starts = starts.to(dev, non_blocking=True)
        side = self._side_stream(dev)
        if train_fe:  # differentiable in FE1's parameters (autograd.feat_extraction)
            def run(pts, st, wl=None, fps=None):
                return autograd.feat_extraction(self.FE1, pts, st, wl=wl, side_stream=side, fps=fps)
        else:
            lt = trace.setdefault("fe_layers", []) if trace is not None else None

            def run(pts, st, wl=None, side_stream=None):
                return self.FE1.run(pts, st, wl=wl, side_stream=side_stream, layer_trace=lt)
        if one_pass:
            # src and tgt share FE1's weights and eval-mode FE is per cloud: one 2B-cloud pass
            # (in training mode each call normalises with its own batch statistics: two passes)
            # (the serial FPS chain then runs once for both clouds, on 2B workgroups)
            both = torch.cat([src_pts, tgt_pts], 0)
            if fe_starts is None:
                fe_starts = [torch.cat([starts[i], starts[4 + i]]) for i in range(3)]
            xyz2, feat2, score2 = (run(both, fe_starts, wl=self.WL) if train_fe
                                   else run(both, fe_starts, wl=self.WL, side_stream=side))
            src_xyz, tgt_xyz = xyz2[:B], xyz2[B:]
            src_feat, tgt_feat = feat2[:B], feat2[B:]
            score = score2[:B]
        else:
            if train_fe:
                # two passes (batch statistics per call); the target's serial FPS chain, which
                # needs only its coordinates, runs on its own stream under the source's layers
                tgt_fps = self.FE1.launch_fps(tgt_pts, starts[4:7], self._fps_stream(dev))
                src_xyz, src_feat, score = run(src_pts, starts[0:3], wl=self.WL)
                tgt_xyz, tgt_feat, _ = run(tgt_pts, starts[4:7], fps=tgt_fps)
            else:
                src_xyz, src_feat, score = run(src_pts, starts[0:3], wl=self.WL, side_stream=side)
                tgt_xyz, tgt_feat, _ = run(tgt_pts, starts[4:7], side_stream=side)
        return dict(src_xyz=src_xyz, src_feat=src_feat, score=score, tgt_xyz=tgt_xyz, tgt_feat=tgt_feat,
                    starts=starts)

    def forward_head(self, feats, R_init, t_init=None, trace=None, keypoint_idx=None):
        """The head half of forward (deepVCP.py:39-110 after FE1): key points, DFE, candidates,
        kNN, CPG.  Differentiable in DFE/CPG when training the head (see ``_training_mode``)."""
        return self._head(feats, R_init, self._training_mode()[0], trace, keypoint_idx)

    def forward(self, src_pts, tgt_pts, R_init, t_init, starts=None, trace=None, keypoint_idx=None,
                return_weights=False):
        """``starts`` (7, B): FPS start indices (drawn like the reference when None).
        ``trace``: dict filled with the stage outputs.  ``keypoint_idx`` (B, K): stage override
        for parity testing -- use these FE-space key-point indices instead of the top-k.
        ``return_weights``: also return the key points' weighting-layer scores (B, K), the
        weights of the paper's weighted pose solve (dvcp.paper)."""
        train_head, train_fe = self._training_mode()
        tr = {} if (return_weights and trace is None) else trace
        with _lib.deferred_flags():  # the guards' host copies once, after the step's launches
            feats = self.extract_features(src_pts, tgt_pts, starts, train_fe=train_fe, trace=trace)
            keypts, vcp = self._head(feats, R_init, train_head, tr, keypoint_idx)
        if not return_weights:
            return keypts, vcp
        return keypts, vcp, torch.gather(feats["score"].detach(), 1, tr["topk"])

    def _head(self, f, R_init, train_head, trace, keypoint_idx):
        src_xyz, src_feat, score, tgt_xyz, tgt_feat, starts = (f["src_xyz"], f["src_feat"], f["score"], f["tgt_xyz"],
                                                               f["tgt_feat"], f["starts"])
        B = src_xyz.shape[0]
        K, r, s = self.K, self.r, self.s
        dev = src_xyz.device
        _lib.check_device_flags()   # guards of earlier launches (non-blocking)
        top = ops.topk(score, K) if keypoint_idx is None else keypoint_idx.to(dev, torch.int64).contiguous()
        if train_head and src_feat.requires_grad:
            keypts, src_cat, moved = autograd.src_keypoints(src_xyz, src_feat, top, starts[3], R_init)
        else:
            keypts, src_cat, moved = ops.src_keypoints(src_xyz, src_feat, top, starts[3], R_init, radius=1.0,
                                                       nsample=32)
        if train_head:
            src_dfe, side, dfe_pack = autograd.dfe_rows(src_cat, self.DFE), None, None
        else:
            # the source rows' DFE (a small launch) runs on the side stream beside the candidate
            # grid, kNN and target DFE, which do not read it; the CPG waits for it.  The packed
            # DFE parameters are formed (or fetched from the cache) on the current stream BEFORE
            # the side stream forks, so both DFE launches read one buffer that the current
            # stream owns and whose (re)build both streams are ordered after.
            cur, side = torch.cuda.current_stream(dev), self._side_stream(dev)
            dfe_pack = self.DFE.packed_params()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                src_dfe = ops.dfe(src_cat, dfe_pack)
            src_cat.record_stream(side)
            dfe_pack.record_stream(side)
            src_dfe.record_stream(cur)

        G = int((2 * r) / s + 1)                    # cpg.py:29
        if grid_side(r, s) != G:
            raise AssertionError("cpg.py:30: candidate count != grid_size^3")
        cand, verr = ops.voxelize(moved, r, s, G, pdim=1)
        # the reference's per-point aranges would not stack if a length differed from G (checked
        # without a stall: raised by a later dvcp call once this launch has completed)
        _lib.defer_flag_check("voxelize: a key point's per-axis grid length differs from the others", verr)
        C = G * G * G
        qry = cand.view(B, K * C, 3)
        dist, idx, _ = ops.knn(tgt_xyz, qry, 32, ref_pdim=2, qry_pdim=1, want_idx64=False)
        if train_head:
            if self.feat_dtype != torch.float32:
                _warn_f16_autograd()
            tgt_dfe = autograd.dfe_tgt(tgt_xyz, tgt_feat, qry, dist, idx, self.DFE).view(B, K, C, 32)
            vcp = autograd.cpg(src_dfe, tgt_dfe.permute(0, 1, 3, 2), cand, G, self.cpg)
        else:
            feat_t = tgt_feat if self.feat_dtype == torch.float32 else tgt_feat.to(self.feat_dtype)
            tgt_dfe = ops.dfe_tgt(tgt_xyz, feat_t, qry, dist, idx, dfe_pack, ref_pdim=2,
                                  literal=self.dfe_literal and self.feat_dtype == torch.float32)
            tgt_dfe = tgt_dfe.view(B, K, C, 32)
            torch.cuda.current_stream(dev).wait_stream(side)
            vcp = ops.cpg(src_dfe, tgt_dfe.permute(0, 1, 3, 2), cand, G, self.cpg.packed_params())
        if trace is not None:
            trace.update(src_xyz=src_xyz, src_feat=src_feat, score=score, topk=top, keypts=keypts,
                         src_cat=src_cat, moved=moved, src_dfe=src_dfe, tgt_xyz=tgt_xyz, tgt_feat=tgt_feat,
                         cand=cand, knn_dist=dist, knn_idx=idx, tgt_dfe=tgt_dfe)
        return keypts, vcp
