"""Tensor-level wrappers of the HIP entry points (one function per C-ABI call).

Every function takes GPU tensors, allocates its outputs with torch's caching allocator and
launches on torch's current stream.  Point tensors are passed as strided views: ``pdim`` is
the dimension that indexes points (1 for (B, N, 3), 2 for the reference's (B, 3, N)).
"""
import os

import torch

from . import _lib
from ._lib import call, dtype_code, ptr, stream


def _pts(t, pdim):
    cdim = 3 - pdim
    if t.dim() != 3 or t.shape[cdim] < 3:
        raise ValueError(f"dvcp: expected a (B, N, 3)/(B, 3, N) point tensor, got {tuple(t.shape)}")
    sb, sc, sn = _lib.point_strides(t, pdim, cdim)
    return t.shape[pdim], sb, sc, sn


# largest cloud the register-resident FPS kernel takes (csrc/fps.hip); beyond it a workspace
FPS_REG_LIMIT = {torch.float32: 16384, torch.float64: 8192}


# fp32 clouds the split select takes (several workgroups per cloud, one exchange per round;
# csrc/fps.hip FpsPartArgs), given a workspace
FPS_PART_RANGE = (2048, 65536)


def fps_parts(N, dtype=torch.float32):
    """Workgroups per cloud of the select kernel for an N-point cloud when the caller does not say
    (csrc/fps.hip fps_parts): above the one-workgroup kernel's 16384 points, 8 (C5's 65536-point
    layer 1); up to it one, unless DVCP_FPS_PARTS (2, 4 or 8) asks for the split select."""
    if dtype != torch.float32 or not FPS_PART_RANGE[0] <= N <= FPS_PART_RANGE[1]:
        return 1
    forced = int(os.environ.get("DVCP_FPS_PARTS", "0") or 0)
    if forced in (1, 2, 4, 8):
        return forced
    return 8 if N > FPS_REG_LIMIT[dtype] else 1


def fps(xyz, npoint, start, pdim=1, parts=None, err=None):
    """pointnet2_utils.py:63-84.  Returns (idx (B, npoint) int64, centres (B, 3, npoint)).
    ``parts`` (tests, A/B): workgroups per cloud of the select kernel (1, 2, 4 or 8; fp32 clouds of
    2048..65536 points), else ``fps_parts``; the indices are the same for every choice.  (Above
    16384 points, parts=1 takes the per-step split kernel, dvcp_fps_ws's.)  ``err``: the guard's
    error word (a zeroed int32 tensor of one element) when the launch takes several workgroups
    per cloud (``fps_uses_guard``); allocated here when None."""
    _lib.require_gpu(xyz, start)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, pdim)
    start = start.to(device=xyz.device, dtype=torch.int64).contiguous()
    idx = torch.empty(B, npoint, dtype=torch.int64, device=xyz.device)
    ctr = torch.empty(B, 3, npoint, dtype=xyz.dtype, device=xyz.device)
    limit = FPS_REG_LIMIT[xyz.dtype]
    _lib.check_device_flags()   # earlier launches' guards (non-blocking)
    split = N > limit
    S = parts if parts is not None else fps_parts(N, xyz.dtype)
    part = S > 1 and xyz.dtype == torch.float32 and FPS_PART_RANGE[0] <= N <= FPS_PART_RANGE[1]
    multi = split or part
    nbytes = int(_lib.load().dvcp_fps_workspace_bytes(B, N))
    ws = torch.empty((nbytes + 7) // 8, dtype=torch.int64, device=xyz.device)
    # (``err``: a caller's zeroed int32 word, e.g. one of a chain's; else a fresh one)
    err = (err if err is not None else torch.zeros(1, dtype=torch.int32, device=xyz.device)) if multi else None
    es = xyz.element_size()
    wgs = B * (S if part else -(-N // 16384) if split else 1)
    work = (9.0 * B * npoint * N, B * (3 * N * es + npoint * (8 + 3 * es)), None, wgs, npoint)
    call("dvcp_fps_parts", dtype_code(xyz), ptr(xyz), sb, sc, sn, B, N, npoint, ptr(start), ptr(idx), ptr(ctr),
         ptr(ws), ws.numel() * 8, ptr(err), int(parts if parts is not None else S), stream(), work=work)
    if multi:
        _lib.defer_flag_check(f"dvcp_fps: FPS workgroups gave up waiting for their peers (N={N})", err)
    return idx, ctr


def fps_uses_guard(xyz, pdim=1, parts=None):
    """Whether ``fps`` on this cloud takes several workgroups per cloud (and an error word)."""
    N = xyz.shape[pdim]
    S = parts if parts is not None else fps_parts(N, xyz.dtype)
    part = S > 1 and xyz.dtype == torch.float32 and FPS_PART_RANGE[0] <= N <= FPS_PART_RANGE[1]
    return N > FPS_REG_LIMIT[xyz.dtype] or part


FPS_PAIR_RANGE = (2048, 16384)


def fps_pair_ok(xyz, npoint2, npoint3, pdim=1):
    """Whether the FE chain takes ``fps_pair`` (opt-in: ``DVCP_FPS_PAIR=1``): fp32, both layers
    pick every point (npoint equal to the cloud's point count, FE layers 2 and 3) and the select
    kernel's cloud size.  Off by default: a launch ends with its slowest cloud, and with 16 clouds
    (C3) the largest of their random start3 draws sits near the end of layer 2's chain, where the
    pair takes as long as the serial launches (tools/fps_bench.py, profiles/round5/r5aw_pair_ab.log)
    while layer 3's per-point tables lose their overlap with layer 3's FPS.  It pays with one or
    two clouds per launch."""
    N = xyz.shape[pdim]
    return (os.environ.get("DVCP_FPS_PAIR", "0") == "1" and xyz.dtype == torch.float32
            and npoint2 == N and npoint3 == N and FPS_PAIR_RANGE[0] <= N <= FPS_PAIR_RANGE[1])


def fps_pair(xyz, start2, start3, pdim=1):
    """Two chained full-permutation FPS layers in one launch (dvcp_fps_pair): equal, bit for bit,
    to ``i2, c2 = fps(xyz, N, start2); i3, c3 = fps(c2, N, start3, pdim=2)``.  Returns
    (i2, c2, i3, c3)."""
    _lib.require_gpu(xyz, start2, start3)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, pdim)
    dev = xyz.device
    s2 = start2.to(device=dev, dtype=torch.int64).contiguous()
    s3 = start3.to(device=dev, dtype=torch.int64).contiguous()
    i2 = torch.empty(B, N, dtype=torch.int64, device=dev)
    i3 = torch.empty(B, N, dtype=torch.int64, device=dev)
    c2 = torch.empty(B, 3, N, dtype=xyz.dtype, device=dev)
    c3 = torch.empty(B, 3, N, dtype=xyz.dtype, device=dev)
    ws = torch.empty(int(_lib.load().dvcp_fps_pair_workspace_bytes(B, N)) // 4, dtype=torch.int32, device=dev)
    es = xyz.element_size()
    call("dvcp_fps_pair", dtype_code(xyz), ptr(xyz), sb, sc, sn, B, N, ptr(s2), ptr(s3), ptr(i2), ptr(c2), ptr(i3),
         ptr(c3), ptr(ws), stream(),
         work=(2 * 9.0 * B * N * N, 2 * B * (3 * N * es + N * (8 + 3 * es)), None, 2 * B, N))
    return i2, c2, i3, c3


def ball_query(xyz, ctr, radius, nsample, pdim=1, cdim_pts=1, compact=True, padded=False):
    """pointnet2_utils.py:87-107.  ``ctr`` uses point dim ``cdim_pts``.  Returns
    (count (B,S) int32, list (B,S,ns) int32) and/or padded (B,S,ns) int64."""
    _lib.require_gpu(xyz, ctr)
    if xyz.dtype != ctr.dtype:
        raise TypeError("dvcp.ball_query: xyz and centres must share a dtype")
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, pdim)
    S, cb, cc, cn = _pts(ctr, cdim_pts)
    dev = xyz.device
    count = torch.empty(B, S, dtype=torch.int32, device=dev) if compact else None
    lst = torch.empty(B, S, nsample, dtype=torch.int32, device=dev) if compact else None
    pad = torch.empty(B, S, nsample, dtype=torch.int64, device=dev) if padded else None
    es = xyz.element_size()
    out_b = (4 + 4 * nsample if compact else 0) + (8 * nsample if padded else 0)
    ws = None
    if xyz.dtype == torch.float32:
        nb = int(_lib.load().dvcp_ball_query_workspace_bytes(B, N, S))
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    call("dvcp_ball_query_ws", dtype_code(xyz), ptr(xyz), sb, sc, sn, N, ptr(ctr), cb, cc, cn, S, B, float(radius),
         int(nsample), ptr(count), ptr(lst), ptr(pad), ptr(ws), stream(),
         work=(9.0 * B * S * N, B * (3 * es * (N + S) + S * out_b)))
    return count, lst, pad


def square_distance(src, dst):
    """pointnet2_utils.py:19-40 on (B, S, 3) / (B, N, 3)."""
    _lib.require_gpu(src, dst)
    B = src.shape[0]
    S, sb, sc, sn = _pts(src, 1)
    N, db, dc, dn = _pts(dst, 1)
    out = torch.empty(B, S, N, dtype=src.dtype, device=src.device)
    call("dvcp_square_distance", dtype_code(src), ptr(src), sb, sc, sn, S, ptr(dst), db, dc, dn, N, B, ptr(out),
         stream())
    return out


def sa_group_mlp(xyz, ctr, feat, count, lst, nsample, chans, params, xyz_pdim=2, feat_ddim=1, feat_pdim=2,
                 ctr_pdim=2):
    """Grouping + [Conv1x1, BN, ReLU]* + max (pointnet2_utils.py:122-132, :195-200).
    ``feat`` is None or a (B, D, N)-indexable strided view; output (B, S, C_last) fp32.  Points
    in (B, N, 4) rows (``points_pack4``, xyz_pdim=1) are gathered one 16-byte load per row."""
    _lib.require_gpu(xyz, ctr, count, lst, params)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, xyz_pdim)
    S, cb, cc, cn = _pts(ctr, ctr_pdim)
    if feat is not None:
        st = feat.stride()
        D = feat.shape[feat_ddim]
        fb, fd, fn = st[0], st[feat_ddim], st[feat_pdim]
        fdt = dtype_code(feat)
    else:
        D, fb, fd, fn, fdt = 0, 0, 0, 0, _lib.F32
    ch = torch.tensor(list(chans), dtype=torch.int32)  # host array, read by the launcher only
    out = torch.empty(B, S, chans[-1], dtype=torch.float32, device=xyz.device)
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))
    # two-layer MFMA tables take a workspace: the per-point half of layer 1 and the centre order
    ws_bytes = _lib.load().dvcp_sa_group_mlp_workspace_bytes(B, N, S, len(chans) - 1, ch.data_ptr())
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=xyz.device) if ws_bytes else None
    call("dvcp_sa_group_mlp_ws", dtype_code(xyz), ptr(xyz), sb, sc, sn, N, ptr(ctr), cb, cc, cn, S, B, fdt,
         ptr(feat), fb, fd, fn, D, ptr(count), ptr(lst), int(nsample), len(chans) - 1, ptr(ch), ptr(params), ptr(out),
         ptr(ws), stream(),
         work=(2.0 * macs * B * S * nsample, B * S * (4 * nsample + 4 * chans[-1]) + B * N * 4 * (3 + D),
               _sa_exec_flops(chans, B, N, S, nsample, count)))
    return out


def sa_group_mlp_rows(xyz, ctr, feat, rows, count, lst, nsample, chans, params, xyz_pdim=2, ctr_pdim=2):
    """``sa_group_mlp`` for the two-layer tables with point n of cloud b taking feature row
    ``rows[b, n]`` of ``feat`` (B, Nf, D) fp32 point-major: the previous layer's per-point rows
    gathered by its FPS order (pointnet2_utils.py:59) without materialising the gathered table."""
    _lib.require_gpu(xyz, ctr, feat, rows, count, lst, params)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, xyz_pdim)
    S, cb, cc, cn = _pts(ctr, ctr_pdim)
    Nf, D = feat.shape[1], feat.shape[2]
    if feat.dtype != torch.float32 or feat.stride(2) != 1 or rows.dtype != torch.int64 or tuple(rows.shape) != (B, N):
        raise ValueError("sa_group_mlp_rows: feat must be (B, Nf, D) fp32 with contiguous rows, rows (B, N) int64")
    rows = rows.contiguous()
    ch = torch.tensor(list(chans), dtype=torch.int32)
    out = torch.empty(B, S, chans[-1], dtype=torch.float32, device=xyz.device)
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))
    ws_bytes = _lib.load().dvcp_sa_group_mlp_workspace_bytes(B, N, S, len(chans) - 1, ch.data_ptr())
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=xyz.device)
    call("dvcp_sa_group_mlp_rows_ws", dtype_code(xyz), ptr(xyz), sb, sc, sn, N, ptr(ctr), cb, cc, cn, S, B,
         ptr(feat), feat.stride(0), feat.stride(1), Nf, D, ptr(rows), ptr(count), ptr(lst), int(nsample),
         len(chans) - 1, ptr(ch), ptr(params), ptr(out), ptr(ws), stream(),
         work=(2.0 * macs * B * S * nsample, B * S * (4 * nsample + 4 * chans[-1]) + B * N * (4 * (3 + D) + 8),
               _sa_exec_flops(chans, B, N, S, nsample, count)))
    return out


MFMA_F32_32X32X2_FLOPS = 2 * 32 * 32 * 2     # one v_mfma_f32_32x32x2_f32
MFMA_BF16_32X32X16_FLOPS = 2 * 32 * 32 * 16  # one v_mfma_f32_32x32x16_bf16


def _sa_exec_flops(chans, B, N, S, nsample, count):
    """The flops the kernels execute on this launch, from the ball query's real hit counts
    (evaluated lazily -- after the timed region -- by bench.py: one device reduction of ``count``).
    Rows run in 16-row half tiles, two per 32-row MFMA tile (csrc/sa_mlp_mfma.hip: a centre takes
    ceil(clamp(count, 1, ns) / 16) half tiles; padded rows execute like real ones).

    * two-layer MFMA tables (sa2 35-32-64, sa3 67-64-64): layer 1 is split into the per-point pass
      sa_pre_kernel (VALU, 2 D C1 per input point) and, per tile, 2 MT v_mfma_f32_32x32x2_f32 (xyz
      k-steps) and layer 2 as MT 2 CT 16-deep k-steps of six v_mfma_f32_32x32x16_bf16 (the
      fp32-accurate three-way bf16 split);
    * sa1 (3 / 6-16-16-32): per tile ceil(C0 / 2) v_mfma_f32_32x32x2_f32 (layer 1, 32 output
      channels of which 16 are padding) and one 16-deep split k-step each for layers 2 (32 x 16
      padded) and 3;
    * other tables (csrc/sa_mlp.hip, VALU): one row per distinct hit, clamp(count, 0, ns)
      rows x 2 sum(C_l C_l+1).
    Returns a callable -> (executed fp32-equivalent flops, of which on the matrix cores, of which
    on the bf16 pipe as fp32-equivalent flops, the bf16 pipe's own flops (6 x those))."""
    def tiles():
        return float(((count.clamp(1, nsample).long() + 15) // 16).sum()) / 2.0
    if len(chans) == 3 and chans[0] - 3 in (32, 64):
        D, C1, C2 = chans[0] - 3, chans[1], chans[2]
        mt, ct = C1 // 32, C2 // 32
        xyz_tile = 2 * mt * MFMA_F32_32X32X2_FLOPS
        l2_tile = 2 * mt * ct * MFMA_BF16_32X32X16_FLOPS  # = 2 x 32 rows x C1 x C2

        def f():
            t = tiles()
            mfma = t * (xyz_tile + l2_tile)
            return 2.0 * B * N * D * C1 + mfma, mfma, t * l2_tile, 6.0 * t * l2_tile
        return f
    if len(chans) == 4 and chans[0] in (3, 6) and list(chans[1:]) == [16, 16, 32]:
        l1_tile = (chans[0] + 1) // 2 * MFMA_F32_32X32X2_FLOPS
        bf_tile = 2 * MFMA_BF16_32X32X16_FLOPS

        def h():
            t = tiles()
            return t * (l1_tile + bf_tile), t * (l1_tile + bf_tile), t * bf_tile, 6.0 * t * bf_tile
        return h
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))

    def g():
        return 2.0 * macs * float(count.clamp(0, nsample).long().sum()), 0.0
    return g


def fe_head(x, params, with_score):
    """deep_feat_extraction.py:15 fc (+ weighting_layer.py:26-30).  x (P, 64) fp32."""
    _lib.require_gpu(x, params)
    P = x.shape[0]
    feat = torch.empty(P, 32, dtype=torch.float32, device=x.device)
    score = torch.empty(P, dtype=torch.float32, device=x.device) if with_score else None
    call("dvcp_fe_head", ptr(x), P, ptr(params), ptr(feat), ptr(score), stream())
    return feat, score


def fe_head_rows(x, rows, params, with_score):
    """``fe_head`` on x (B, Nx, 64) fp32 rows gathered per cloud by ``rows`` (B, S) int64 (sa3's
    per-point rows in its FPS order, pointnet2_utils.py:59), without materialising the gather."""
    _lib.require_gpu(x, rows, params)
    B, Nx, C = x.shape
    if C != 64 or x.dtype != torch.float32 or not x.is_contiguous() or rows.dtype != torch.int64 or rows.shape[0] != B:
        raise ValueError("fe_head_rows: x must be contiguous (B, Nx, 64) fp32 and rows (B, S) int64")
    rows = rows.contiguous()
    S = rows.shape[1]
    P = B * S
    feat = torch.empty(P, 32, dtype=torch.float32, device=x.device)
    score = torch.empty(P, dtype=torch.float32, device=x.device) if with_score else None
    call("dvcp_fe_head_rows", ptr(x), ptr(rows), S, Nx, P, ptr(params), ptr(feat), ptr(score), stream())
    return feat, score


def weighting(feat, params):
    _lib.require_gpu(feat, params)
    P = feat.shape[0]
    score = torch.empty(P, dtype=torch.float32, device=feat.device)
    call("dvcp_weighting", ptr(feat), P, ptr(params), ptr(score), stream())
    return score


def topk(score, K):
    """weighting_layer.py:31 on (B, S) scores -> (B, K) int64 (descending, ties -> lower index)."""
    _lib.require_gpu(score)
    B, S = score.shape
    idx = torch.empty(B, K, dtype=torch.int64, device=score.device)
    call("dvcp_topk", ptr(score), B, S, K, ptr(idx), stream())
    return idx


def src_keypoints(fe_xyz, fe_feat, topk_idx, kstart, R_init, radius=1.0, nsample=32):
    """deepVCP.py:44-68 + get_cat_feat_src.py + deepVCP.py:86-91 (REF-R R2/R3)."""
    _lib.require_gpu(fe_xyz, fe_feat, topk_idx, kstart, R_init)
    B, _, S = fe_xyz.shape
    K = topk_idx.shape[1]
    if R_init.dtype != torch.float64:
        # deepVCP.py:90 multiplies R_init with a .double() tensor; any other dtype raises there.
        raise RuntimeError(f"expected R_init of dtype torch.float64, got {R_init.dtype}")
    R = R_init.reshape(-1, 3, 3).contiguous()
    if R.shape[0] not in (1, B):
        raise RuntimeError(f"R_init batch {R.shape[0]} does not broadcast to B={B}")
    r_b = 9 if R.shape[0] == B and B > 1 else 0
    dev = fe_xyz.device
    # keep every temporary alive across the launch (a freed block could be handed to the next
    # allocation in the same argument list)
    xyz_c, feat_c = fe_xyz.contiguous(), fe_feat.contiguous()
    top_c, ks_c = topk_idx.contiguous(), kstart.to(device=dev, dtype=torch.int64).contiguous()
    keypts = torch.empty(B, K, 3, dtype=fe_xyz.dtype, device=dev)
    src_cat = torch.empty(B, K, nsample, 35, dtype=torch.float32, device=dev)
    moved = torch.empty(B, K, 3, dtype=torch.float64, device=dev)
    call("dvcp_src_keypoints", dtype_code(fe_xyz), ptr(xyz_c), ptr(feat_c), S, ptr(top_c), B, K, ptr(ks_c),
         float(radius), int(nsample), ptr(R), r_b, ptr(keypts), ptr(src_cat), ptr(moved), stream())
    return keypts, src_cat, moved


def voxelize(pts, r, s, G, pdim=1):
    """voxelize.py:19-83: (B, Kp, 3) -> (B, Kp, G^3, 3) fp32 candidates, plus an error flag."""
    _lib.require_gpu(pts)
    B = pts.shape[0]
    Kp, pb, pc, pn = _pts(pts, pdim)
    cand = torch.empty(B, Kp, G * G * G, 3, dtype=torch.float32, device=pts.device)
    err = torch.zeros(1, dtype=torch.int32, device=pts.device)
    call("dvcp_voxelize", dtype_code(pts), ptr(pts), pb, pc, pn, B, Kp, float(r), float(s), int(G), ptr(cand),
         ptr(err), stream())
    return cand, err


# kNN method choice.  All are exact and return identical results.
#   tiled: Morton-sorted reference tiles scanned nearest-first per wave (dvcp_knn_tiled; k > 16:
#          lane-private candidate buffers merged by bitonic networks); M <= KNN_TILED_MAX_M.
#   tiled_insert: the same scan inserting every candidate into the sorted list at once (the
#          round-2 kernel, dvcp_knn_tiled_insert), kept for parity tests and A/B timing.
#   brute: index-order scan of every reference point (dvcp_knn); best for small M.
#   grid:  per-query cell-shell search (dvcp_knn_grid); loses on the forward's workload, where
#          most voxel candidates lie outside the target cloud (profiles/round1: 35.8 ms vs 12.4 ms
#          brute per C3 step).  Kept as an option.
KNN_TILED_MIN_M = 512
KNN_TILED_MAX_M = 16384


def knn_method(M):
    return "tiled" if KNN_TILED_MIN_M <= M <= KNN_TILED_MAX_M else "brute"


def knn(ref, qry, k, ref_pdim=1, qry_pdim=1, want_idx64=True, method=None):
    """Exact kNN (knn_cuda.KNN replacement).  Returns dist (B,Q,k) fp32, idx int32, idx64."""
    _lib.require_gpu(ref, qry)
    if ref.dtype != qry.dtype:
        qry = qry.to(ref.dtype)  # both sides are cast to fp32 inside, like knn_cuda's .float()
    B = ref.shape[0]
    M, rb, rc, rn = _pts(ref, ref_pdim)
    Q, qb, qc, qn = _pts(qry, qry_pdim)
    dev = ref.device
    dist = torch.empty(B, Q, k, dtype=torch.float32, device=dev)
    idx = torch.empty(B, Q, k, dtype=torch.int32, device=dev)
    idx64 = torch.empty(B, Q, k, dtype=torch.int64, device=dev) if want_idx64 else None
    work = (9.0 * B * Q * M, B * (12 * (M + Q) + Q * k * (8 + (8 if want_idx64 else 0))))
    method = method or knn_method(M)
    if method in ("tiled", "tiled_insert"):
        ws = torch.empty(int(_lib.load().dvcp_knn_tiled_workspace_bytes(B, M, Q)), dtype=torch.uint8, device=dev)
        call("dvcp_knn_tiled" if method == "tiled" else "dvcp_knn_tiled_insert", dtype_code(ref), ptr(ref), rb, rc, rn, M, ptr(qry), qb, qc, qn, Q, B, int(k), ptr(ws),
             ptr(dist), ptr(idx), ptr(idx64), stream(), work=work)
    elif method == "grid":
        ws = torch.empty(int(_lib.load().dvcp_knn_grid_workspace_bytes(B, M)), dtype=torch.uint8, device=dev)
        call("dvcp_knn_grid", dtype_code(ref), ptr(ref), rb, rc, rn, M, ptr(qry), qb, qc, qn, Q, B, int(k), ptr(ws),
             ptr(dist), ptr(idx), ptr(idx64), stream(), work=work)
    else:
        call("dvcp_knn", dtype_code(ref), ptr(ref), rb, rc, rn, M, ptr(qry), qb, qc, qn, Q, B, int(k), ptr(dist),
             ptr(idx), ptr(idx64), stream(), work=work)
    return dist, idx, idx64


def dfe(X, params):
    """deep_feat_embedding.py on materialised rows: X (..., 32, 35) -> (..., 32) fp32."""
    _lib.require_gpu(X, params)
    lead = X.shape[:-2]
    if tuple(X.shape[-2:]) != (32, 35):
        raise RuntimeError(f"feat_embedding_layer expects (..., 32, 35), got {tuple(X.shape)}")
    Xc = X.contiguous()
    R = Xc.numel() // (32 * 35)
    out = torch.empty(R, 32, dtype=torch.float32, device=X.device)
    call("dvcp_dfe", dtype_code(Xc), ptr(Xc), R, ptr(params), ptr(out), stream(),
         work=(2.0 * 3168 * 32 * R, Xc.numel() * Xc.element_size() + 128 * R))
    return out.view(*lead, 32)


def dfe_tgt(ref_xyz, ref_feat, cand, dist, idx, params, ref_pdim=2, literal=False):
    """get_cat_feat_tgt.py:54-96 fused with deep_feat_embedding.py:47-60.  cand (B, Q, 3).
    ``literal``: fc1-fc3 chained as written instead of collapsed into one map (Q14)."""
    _lib.require_gpu(ref_xyz, ref_feat, cand, dist, idx, params)
    B = ref_xyz.shape[0]
    M, rb, rc, rn = _pts(ref_xyz, ref_pdim)
    Q = cand.shape[1]
    feat_c, cand_c, dist_c, idx_c = ref_feat.contiguous(), cand.contiguous(), dist.contiguous(), idx.contiguous()
    out = torch.empty(B, Q, 32, dtype=torch.float32, device=ref_xyz.device)
    half = feat_c.dtype == torch.float16   # the C5 fp16-feature storage (dvcp_dfe_tgt_f16)
    if half and literal:
        raise ValueError("dfe_tgt: the literal (Q14) path takes fp32 features only")
    if not half and feat_c.dtype != torch.float32:
        raise TypeError(f"dfe_tgt: features must be float32 or float16, got {feat_c.dtype}")
    name = "dvcp_dfe_tgt_f16" if half else ("dvcp_dfe_tgt_literal" if literal else "dvcp_dfe_tgt")
    row = 64 if half else 128
    if ref_xyz.dtype == torch.float32 and not literal and not (rc == 1 and rn == 4):
        ref_xyz, rb, rc, rn = points_pack4(ref_xyz, ref_pdim), 4 * M, 1, 4
    call(name, dtype_code(ref_xyz), ptr(ref_xyz), rb, rc, rn, M, ptr(feat_c), ptr(cand_c), ptr(dist_c),
         ptr(idx_c), B, Q, ptr(params), ptr(out), stream(),
         work=(2.0 * 3168 * 32 * B * Q, B * (M * (12 + row) + Q * (12 + 32 * 8 + 128)),
               _dfe_tgt_exec(literal, float(B * Q))))
    return out


def points_pack4(xyz, pdim=2):
    """(B, M, 4) fp32 rows (x, y, z, 0) of fp32 points (B, 3, M) (pdim=2) or (B, M, 3) (pdim=1):
    the layout the target DFE gathers with one 16-byte load per neighbour (dvcp_points_pack4)."""
    _lib.require_gpu(xyz)
    if xyz.dtype != torch.float32:
        raise TypeError(f"points_pack4: fp32 points only, got {xyz.dtype}")
    B = xyz.shape[0]
    M, rb, rc, rn = _pts(xyz, pdim)
    out = torch.empty(B, M, 4, dtype=torch.float32, device=xyz.device)
    call("dvcp_points_pack4", ptr(xyz), rb, rc, rn, M, B, ptr(out), stream(), work=(0.0, 28.0 * B * M, 0.0))
    return out


def _dfe_tgt_exec(literal, cands):
    """Executed MFMA work of the target DFE (csrc/dfe_mfma.hip), as bench.py's 4-tuple (fp32-equivalent
    flops, of which on the matrix cores, of which on the bf16 pipe, the bf16 pipe's own flops).
    Literal (Q14) path: 51 v_mfma_f32_32x32x2_f32 per candidate (fc1's 35 inputs in 19 k-steps, 16 +
    16 for fc2, fc3).  Collapsed path: the xyz columns in 2 fp32 k-steps and the 32 feature columns
    in 2 split-3 bf16 k-steps (six v_mfma_f32_32x32x16_bf16 each)."""
    if literal:
        f = 51 * MFMA_F32_32X32X2_FLOPS * cands
        return f, f
    bf = 2 * MFMA_BF16_32X32X16_FLOPS * cands
    f = 2 * MFMA_F32_32X32X2_FLOPS * cands + bf
    return f, f, bf, 6.0 * bf


MFMA_BF16_16X16X32_FLOPS = 2 * 16 * 16 * 32  # one v_mfma_f32_16x16x32_bf16


def cpg(src, tgt, cand, G, params, want_weight=False):
    """cpg.py:27-60.  src (B, K, 32) or (B, K, 1, 32); tgt: the reference's (B, K, 32, C)
    (any strides); cand (B, K, C, 3).  Returns vcp (B, K, 3) [, weights (B, K, C)]."""
    _lib.require_gpu(src, tgt, cand, params)
    B, K, C, _ = cand.shape
    if tgt.dim() != 4 or tuple(tgt.shape) != (B, K, 32, C):
        raise RuntimeError(f"cpg: tgt_dfe_feat must be (B, K, 32, C), got {tuple(tgt.shape)}")
    if tgt.stride(0) != K * tgt.stride(1):
        tgt = tgt.contiguous()
    srcc = src.reshape(B * K, 32).contiguous().float()
    candc = cand.contiguous()
    vcp = torch.empty(B, K, 3, dtype=torch.float32, device=cand.device)
    w = torch.empty(B, K, C, dtype=torch.float32, device=cand.device) if want_weight else None
    call("dvcp_cpg", ptr(srcc), ptr(tgt), tgt.stride(1), tgt.stride(2), tgt.stride(3), ptr(candc), B * K, int(G),
         ptr(params), ptr(vcp), ptr(w), stream(),
         work=(2.0 * 27 * (32 * 16 + 16 * 4 + 4) * B * K * C, B * K * (128 + C * (128 + 12) + 12),
               _cpg_exec(B * K, C)))
    return (vcp, w) if want_weight else vcp


def _cpg_exec(P, C):
    """Executed work of the CPG forward (csrc/cpg.hip) as bench.py's 4-tuple: conv1 on
    v_mfma_f32_16x16x32_bf16 with the split-3 (per 16-voxel tile and 8-channel quarter, 7 k-steps of
    4 taps: one zero tap of padding), conv2 and conv3 on VALU (reference-graph flops)."""
    conv1 = float(P) * (-(-C // 16)) * 4 * 7 * MFMA_BF16_16X16X32_FLOPS
    rest = 2.0 * 27 * (16 * 4 + 4) * P * C
    return conv1 + rest, conv1, conv1, 6.0 * conv1


def rigid_transform(x, y):
    """deepVCP_loss.py:13-44 on (B, 3, n) fp64."""
    _lib.require_gpu(x, y)
    x = x.double().contiguous()
    y = y.double().contiguous()
    B, _, n = x.shape
    R = torch.empty(B, 3, 3, dtype=torch.float64, device=x.device)
    t = torch.empty(B, 3, 1, dtype=torch.float64, device=x.device)
    call("dvcp_rigid_transform", ptr(x), ptr(y), B, n, ptr(R), ptr(t), stream())
    return R, t


def svd_optimization(x, y_pred, R_true, t_true):
    """deepVCP_loss.py:57-90 (+ the per-pair loss sums of :110-119)."""
    _lib.require_gpu(x, y_pred, R_true, t_true)
    x, y_pred, Rt, tt = pose_inputs(x, y_pred, R_true, t_true)
    B, _, n = x.shape
    n_in = int(n * 0.8)
    dev = x.device
    R2 = torch.empty(B, 3, 3, dtype=torch.float64, device=dev)
    t2 = torch.empty(B, 3, 1, dtype=torch.float64, device=dev)
    x1 = torch.empty(B, 3, n_in, dtype=torch.float64, device=dev)
    y2 = torch.empty(B, 3, n_in, dtype=torch.float64, device=dev)
    partial = torch.empty(B, 2, dtype=torch.float64, device=dev)
    call("dvcp_svd_optimization", ptr(x), ptr(y_pred), ptr(Rt), ptr(tt), B, n, ptr(R2), ptr(t2), ptr(x1), ptr(y2),
         ptr(partial), stream())
    return R2, t2, x1, y2, partial


def deepvcp_loss(x, y_pred, R_true, t_true, alpha):
    """deepVCP_loss.py:105-121 on (B, 3, n) operands: (loss () fp64, R2, t2, partial (B, 2))."""
    _lib.require_gpu(x, y_pred, R_true, t_true)
    x, y_pred, Rt, tt = pose_inputs(x, y_pred, R_true, t_true)
    B, _, n = x.shape
    dev = x.device
    R2 = torch.empty(B, 3, 3, dtype=torch.float64, device=dev)
    t2 = torch.empty(B, 3, 1, dtype=torch.float64, device=dev)
    partial = torch.empty(B, 2, dtype=torch.float64, device=dev)
    loss = torch.empty((), dtype=torch.float64, device=dev)
    call("dvcp_deepvcp_loss", ptr(x), ptr(y_pred), ptr(Rt), ptr(tt), B, n, float(alpha), ptr(R2), ptr(t2),
         ptr(partial), ptr(loss), stream())
    return loss, R2, t2, partial


def registration_error(R_pred, t_pred, R_gt, t_gt):
    """train.py:112-120 (C8 fixed): per-pair rotation error (Euler xyz, degrees) and translation
    error, both nn.PairwiseDistance(p=2) with eps 1e-6.  R_pred (B,3,3), t_pred (B,3[,1]);
    R_gt (B|1,3,3), t_gt (B|1,3[,1]).  Returns (rot_err (B,), trans_err (B,)) fp64."""
    _lib.require_gpu(R_pred, t_pred, R_gt, t_gt)
    B = R_pred.shape[0]
    Rp = R_pred.double().reshape(B, 9).contiguous()
    tp = t_pred.double().reshape(B, 3).contiguous()
    Rg = R_gt.double().reshape(-1, 9).contiguous()
    tg = t_gt.double().reshape(-1, 3).contiguous()
    if Rg.shape[0] not in (1, B) or tg.shape[0] not in (1, B):
        raise RuntimeError("registration_error: ground truth must have 1 or B poses")
    rot = torch.empty(B, dtype=torch.float64, device=Rp.device)
    trans = torch.empty(B, dtype=torch.float64, device=Rp.device)
    call("dvcp_registration_error", ptr(Rp), ptr(tp), ptr(Rg), 0 if Rg.shape[0] == 1 else 9, ptr(tg),
         0 if tg.shape[0] == 1 else 3, B, ptr(rot), ptr(trans), stream())
    return rot, trans


def rigid_apply(pts, R, t=None, pdim=2):
    """R @ pts (+ t) in fp64 (KITTIDataset.py:80-81, ModelNet40Dataset.py:74-85).  pts (B, C, N)
    with C = 3 or 6 (xyz [+ normals, rotated only]); R (B, 3, 3); t (B|1, 3[, 1]) or None."""
    _lib.require_gpu(pts, R)
    B, C = pts.shape[0], pts.shape[1]
    N, sb, sc, sn = pts.shape[pdim], pts.stride(0), pts.stride(1), pts.stride(pdim)
    Rc = R.double().reshape(B, 9).contiguous()
    tc = None if t is None else t.double().reshape(-1, 3).contiguous()
    out = torch.empty(B, C, N, dtype=torch.float64, device=pts.device)
    call("dvcp_rigid_apply", dtype_code(pts), ptr(pts), sb, sc, sn, B, N, C, ptr(Rc), ptr(tc),
         0 if tc is None or tc.shape[0] == 1 else 3, ptr(out), stream())
    return out


# ---- backward entry points (training; see dvcp/autograd.py) -----------------------------------

DFE_NPARAMS = 3264   # fc1-3 weights and biases, packed
CPG_NPARAMS = 15681  # conv1-3 weights and biases, packed


def dfe_backward(X, params, grad_out, want_input_grad=False):
    """Parameter gradient of ``dfe`` (deep_feat_embedding.py:23-61) for rows X (..., 32, 35),
    and (``want_input_grad``) the rows' own gradient, shaped like X, fp32."""
    _lib.require_gpu(X, params, grad_out)
    Xc = X.contiguous()
    R = Xc.numel() // (32 * 35)
    g = grad_out.reshape(R, 32).float().contiguous()
    ws = torch.empty(max(1, int(_lib.load().dvcp_dfe_backward_workspace_bytes(R)) // 4), dtype=torch.float32,
                     device=X.device)
    gp = torch.empty(DFE_NPARAMS, dtype=torch.float32, device=X.device)
    gX = torch.empty(X.shape, dtype=torch.float32, device=X.device) if want_input_grad else None
    call("dvcp_dfe_backward", dtype_code(Xc), ptr(Xc), R, ptr(params), ptr(g), ptr(ws), ptr(gp), ptr(gX), stream())
    return (gp, gX) if want_input_grad else gp


def dfe_tgt_backward(ref_xyz, ref_feat, cand, dist, idx, params, grad_out, ref_pdim=2, want_feat_grad=False):
    """Parameter gradient of ``dfe_tgt`` (get_cat_feat_tgt.py:54-96 + deep_feat_embedding.py:47-60),
    and (``want_feat_grad``) the gradient of ``ref_feat`` (B, M, 32) through the :85 gather, summed
    per target row in a fixed order (bit-identical run to run)."""
    _lib.require_gpu(ref_xyz, ref_feat, cand, dist, idx, params, grad_out)
    B = ref_xyz.shape[0]
    M, rb, rc, rn = _pts(ref_xyz, ref_pdim)
    Q = cand.shape[1]
    feat_c, cand_c, dist_c, idx_c = ref_feat.contiguous(), cand.contiguous(), dist.contiguous(), idx.contiguous()
    g = grad_out.reshape(B, Q, 32).float().contiguous()
    nbytes = int(_lib.load().dvcp_dfe_tgt_backward_workspace_bytes(B, Q, M, int(bool(want_feat_grad))))
    if nbytes < 0:
        raise RuntimeError("dvcp_dfe_tgt_backward_workspace_bytes: size query failed")
    ws = torch.empty(max(1, (nbytes + 3) // 4), dtype=torch.float32, device=ref_xyz.device)
    gp = torch.empty(DFE_NPARAMS, dtype=torch.float32, device=ref_xyz.device)
    gF = torch.empty(B, M, 32, dtype=torch.float32, device=ref_xyz.device) if want_feat_grad else None
    call("dvcp_dfe_tgt_backward", dtype_code(ref_xyz), ptr(ref_xyz), rb, rc, rn, M, ptr(feat_c), ptr(cand_c),
         ptr(dist_c), ptr(idx_c), B, Q, ptr(params), ptr(g), ptr(ws), ptr(gp), ptr(gF), stream(),
         work=(2.0 * 3168 * 32 * B * Q, B * (M * (12 + 128) + Q * (12 + 32 * 8 + 128))))
    return (gp, gF) if want_feat_grad else gp


def src_keypoints_backward(fe_xyz, topk_idx, kstart, grad_cat, radius=1.0, nsample=32):
    """Gradient of FE features (B, S, 32) through the key-point stage's feature rows
    (pointnet2_utils.py:59 gather + get_cat_feat_src.py:50 weighting); ``grad_cat`` is the
    src_cat gradient (B, K, nsample, 35)."""
    _lib.require_gpu(fe_xyz, topk_idx, grad_cat)
    B, _, S_ = fe_xyz.shape
    K = topk_idx.shape[1]
    dev = fe_xyz.device
    xyz_c, top_c = fe_xyz.contiguous(), topk_idx.contiguous()
    ks_c = kstart.to(device=dev, dtype=torch.int64).contiguous()
    g = grad_cat.float().contiguous()
    gF = torch.zeros(B, S_, 32, dtype=torch.float32, device=dev)
    call("dvcp_src_keypoints_backward", dtype_code(fe_xyz), ptr(xyz_c), S_, ptr(top_c), B, K, ptr(ks_c),
         float(radius), int(nsample), ptr(g), ptr(gF), stream())
    return gF


def cpg_backward(src, tgt, cand, G, params, grad_vcp):
    """Gradients of ``cpg`` (cpg.py:27-60): (d src (B,K,32), d tgt (B,K,32,C), d params)."""
    _lib.require_gpu(src, tgt, cand, params, grad_vcp)
    B, K, C, _ = cand.shape
    if tgt.dim() != 4 or tuple(tgt.shape) != (B, K, 32, C):
        raise RuntimeError(f"cpg_backward: tgt_dfe_feat must be (B, K, 32, C), got {tuple(tgt.shape)}")
    if tgt.stride(0) != K * tgt.stride(1):
        tgt = tgt.contiguous()
    P = B * K
    srcc = src.reshape(P, 32).contiguous().float()
    candc = cand.contiguous()
    gv = grad_vcp.reshape(P, 3).float().contiguous()
    dev = cand.device
    gsrc = torch.empty(B, K, 32, dtype=torch.float32, device=dev)
    gtgt = torch.empty(B, K, 32, C, dtype=torch.float32, device=dev)
    ws = torch.empty(max(1, int(_lib.load().dvcp_cpg_backward_workspace_bytes(P)) // 4), dtype=torch.float32,
                     device=dev)
    gp = torch.empty(CPG_NPARAMS, dtype=torch.float32, device=dev)
    call("dvcp_cpg_backward", ptr(srcc), ptr(tgt), tgt.stride(1), tgt.stride(2), tgt.stride(3), ptr(candc), P, int(G),
         ptr(params), ptr(gv), ptr(gsrc), ptr(gtgt), ptr(ws), ptr(gp), stream(),
         work=(3 * 2.0 * 27 * (32 * 16 + 16 * 4 + 4) * P * C, P * (128 + C * (128 + 12 + 128) + 12)))
    return gsrc, gtgt, gp


def sa_group_mlp_backward(xyz, ctr, feat, count, lst, nsample, chans, params, bnstat, grad_out, want_feat_grad,
                          xyz_pdim=2, feat_ddim=1, feat_pdim=2):
    """Backward of ``sa_group_mlp`` with eval-mode BN (pointnet2_utils.py:176-202 + the :59 gather).
    Returns (packed parameter gradient: per layer dW, db, dgamma, dbeta; dL/d feat (B, N, D) fp32
    or None)."""
    _lib.require_gpu(xyz, ctr, count, lst, params, bnstat, grad_out)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, xyz_pdim)
    S, cb, cc, cn = _pts(ctr, 2)
    if feat is not None:
        st = feat.stride()
        D = feat.shape[feat_ddim]
        fb, fd, fn = st[0], st[feat_ddim], st[feat_pdim]
        fdt = dtype_code(feat)
    else:
        D, fb, fd, fn, fdt = 0, 0, 0, 0, _lib.F32
    ch = torch.tensor(list(chans), dtype=torch.int32)
    nl = len(chans) - 1
    npar = sum(a * b + 3 * b for a, b in zip(chans[:-1], chans[1:]))
    dev = xyz.device
    ws = torch.empty(max(1, int(_lib.load().dvcp_sa_group_mlp_backward_workspace_bytes(B, S, nl, ch.data_ptr())) // 4),
                     dtype=torch.float32, device=dev)
    gp = torch.empty(npar, dtype=torch.float32, device=dev)
    gF = torch.zeros(B, N, D, dtype=torch.float32, device=dev) if (want_feat_grad and D > 0) else None
    g = grad_out.float().contiguous()
    call("dvcp_sa_group_mlp_backward", dtype_code(xyz), ptr(xyz), sb, sc, sn, N, ptr(ctr), cb, cc, cn, S, B, fdt,
         ptr(feat), fb, fd, fn, D, ptr(count), ptr(lst), int(nsample), nl, ptr(ch), ptr(params), ptr(bnstat), ptr(g),
         ptr(gF), ptr(ws), ptr(gp), stream())
    return gp, gF


def _bn_common(xyz, ctr, feat, count, lst, nsample, chans, pack, xyz_pdim, feat_ddim, feat_pdim, workspace=True):
    """The grouping arguments shared by dvcp_sa_bn_stats / dvcp_sa_bn_backward."""
    _lib.require_gpu(xyz, ctr, count, lst, pack)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, xyz_pdim)
    S, cb, cc, cn = _pts(ctr, 2)
    if feat is not None:
        st = feat.stride()
        D = feat.shape[feat_ddim]
        fb, fd, fn = st[0], st[feat_ddim], st[feat_pdim]
        fdt = dtype_code(feat)
    else:
        D, fb, fd, fn, fdt = 0, 0, 0, 0, _lib.F32
    ch = torch.tensor(list(chans), dtype=torch.int32)
    nl = len(chans) - 1
    ws = None
    if workspace:
        ws_bytes = int(_lib.load().dvcp_sa_bn_workspace_bytes(B, S, nl, ch.data_ptr()))
        ws = torch.empty(max(1, ws_bytes // 4), dtype=torch.float32, device=xyz.device)
    args = (dtype_code(xyz), ptr(xyz), sb, sc, sn, N, ptr(ctr), cb, cc, cn, S, B, fdt, ptr(feat), fb, fd, fn, D,
            ptr(count), ptr(lst), int(nsample), nl, ptr(ch), ptr(pack))
    return args, ws, (B, N, S, D), ch


def sa_bn_pack_floats(chans):
    ch = torch.tensor(list(chans), dtype=torch.int32)
    return int(_lib.load().dvcp_sa_bn_pack_floats(len(chans) - 1, ch.data_ptr()))


def sa_bn_stats(xyz, ctr, feat, count, lst, nsample, chans, pack, layer, xyz_pdim=2, feat_ddim=1, feat_pdim=2,
                want_zrows=False):
    """Training-mode BatchNorm statistics of the grouped MLP (pointnet2_utils.py:198 in train()):
    (2, C_layer) fp64 = per-channel sum z and sum z^2 of layer ``layer``'s conv output over all
    B * S * nsample grouped entries, the layers below it normalised by ``pack``.  ``want_zrows``
    (last layer only): also -> every entry's z rows, as ``sa_bn_zrows`` returns them."""
    args, ws, (B, N, S, D), ch = _bn_common(xyz, ctr, feat, count, lst, nsample, chans, pack, xyz_pdim, feat_ddim,
                                            feat_pdim)
    sums = torch.empty(2, chans[layer], dtype=torch.float64, device=xyz.device)
    zrows = None
    if want_zrows:
        n = int(_lib.load().dvcp_sa_bn_zrows_floats(B, S, int(nsample), len(chans) - 1, ch.data_ptr()))
        zrows = torch.empty(max(n, 1), dtype=torch.float32, device=xyz.device)
    macs = sum(a * b for a, b in zip(chans[:layer], chans[1:layer + 1]))
    call("dvcp_sa_bn_stats", *args, int(layer), ptr(ws), ptr(sums), ptr(zrows), stream(),
         work=(2.0 * macs * B * S * nsample, B * S * 4 * nsample + B * N * 4 * (3 + D)))
    return (sums, zrows) if want_zrows else sums


def sa_bn_zrows_bytes(B, S, nsample, chans):
    """Size of ``sa_bn_zrows``'s output for this grouping (bytes)."""
    ch = torch.tensor(list(chans), dtype=torch.int32)
    return 4 * int(_lib.load().dvcp_sa_bn_zrows_floats(B, S, int(nsample), len(chans) - 1, ch.data_ptr()))


def sa_bn_zrows(xyz, ctr, feat, count, lst, nsample, chans, pack, xyz_pdim=2, feat_ddim=1, feat_pdim=2):
    """Every grouped entry's conv outputs z_l of every layer with the batch statistics in ``pack``:
    flat fp32, per layer (M / 64, C_l, 64) blocks (what dvcp_sa_bn_backward reads)."""
    args, _, (B, N, S, D), ch = _bn_common(xyz, ctr, feat, count, lst, nsample, chans, pack, xyz_pdim, feat_ddim,
                                           feat_pdim, workspace=False)
    n = int(_lib.load().dvcp_sa_bn_zrows_floats(B, S, int(nsample), len(chans) - 1, ch.data_ptr()))
    z = torch.empty(max(n, 1), dtype=torch.float32, device=xyz.device)
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))
    call("dvcp_sa_bn_zrows", *args, ptr(z), stream(), work=(2.0 * macs * B * S * nsample, 4.0 * n))
    return z


def sa_bn_backward(xyz, ctr, feat, count, lst, nsample, chans, pack, zrows, grad_out, mode, want_feat_grad=False,
                   xyz_pdim=2, feat_ddim=1, feat_pdim=2):
    """Training-mode (batch-statistics) backward of the grouped MLP.  mode k >= 1: (2, C_k) fp64
    sums (A_k = dbeta_k, B_k = dgamma_k); mode 0: (per layer (dL/dz_l, [h_{l-1}; 1]) as
    (chunks, C, 65536) fp32 views, dL/d feat (B, N, D) fp32 or None)."""
    args, ws, (B, N, S, D), ch = _bn_common(xyz, ctr, feat, count, lst, nsample, chans, pack, xyz_pdim, feat_ddim,
                                            feat_pdim)
    dev = xyz.device
    g = grad_out.float().contiguous()
    if mode > 0:
        sums = torch.empty(2, chans[mode], dtype=torch.float64, device=dev)
        call("dvcp_sa_bn_backward", *args, ptr(zrows), int(mode), ptr(g), None, ptr(ws), ptr(sums), None, stream())
        return sums
    M = B * S * int(nsample)
    nrows = int(_lib.load().dvcp_sa_bn_rows_floats(B, S, int(nsample), len(chans) - 1, ch.data_ptr()))
    rows = torch.empty(max(nrows, 1), dtype=torch.float32, device=dev)
    gF = None
    if want_feat_grad and D > 0:
        if D in (32, 64):   # per-entry rows summed per point in entry order (deterministic)
            fb = int(_lib.load().dvcp_sa_bn_feat_workspace_bytes(B, S, int(nsample), N, D))
            if fb < 0:
                raise RuntimeError("dvcp_sa_bn_feat_workspace_bytes: size query failed")
            ws = torch.empty(max(1, (fb + 3) // 4), dtype=torch.float32, device=dev)
            gF = torch.empty(B, N, D, dtype=torch.float32, device=dev)
        else:
            gF = torch.zeros(B, N, D, dtype=torch.float32, device=dev)
    call("dvcp_sa_bn_backward", *args, ptr(zrows), 0, ptr(g), ptr(gF), ptr(ws), None, ptr(rows), stream())
    Kc = 65536              # tables are 65536-entry chunks, channel-major inside (csrc/sa_bn.hip bn_at_rows)
    Mk = -(-M // Kc) * Kc
    views, o = [], 0
    for cin, cout in zip(chans[:-1], chans[1:]):
        gz = rows[o:o + cout * Mk].view(Mk // Kc, cout, Kc)
        o += cout * Mk
        ha = rows[o:o + (cin + 1) * Mk].view(Mk // Kc, cin + 1, Kc)
        o += (cin + 1) * Mk
        if Mk > M:  # the padding entries of the last chunk take no part in the GEMMs
            gz[-1, :, M % Kc:] = 0.0
            ha[-1, :, M % Kc:] = 0.0
        views.append((gz, ha))
    return views, gF


def sa_bnm_usable(xyz, ctr, feat, chans):
    """Whether the matrix-core training path (dvcp_sa_bnm_*) takes this grouping: the REF-R tables
    (sa1 3[+3]-16-16-32, sa2, sa3) with fp32 points and features; the two-layer tables need
    point-major feature rows (16-byte aligned)."""
    ch = torch.tensor(list(chans), dtype=torch.int32)
    if not _lib.load().dvcp_sa_bnm_supported(len(chans) - 1, ch.data_ptr()):
        return False
    if xyz.dtype != torch.float32 or ctr.dtype != torch.float32:
        return False
    if feat is None:
        return len(chans) == 4 and int(chans[0]) == 3
    if feat.dtype != torch.float32 or feat.dim() != 3:
        return False
    if len(chans) == 3 and (feat.stride(1) != 1 or feat.stride(0) % 4 or feat.stride(2) % 4 or feat.data_ptr() % 16):
        return False
    return True


def _bnm_args(xyz, ctr, feat, count, lst, nsample, chans):
    _lib.require_gpu(xyz, ctr, count, lst)
    B = xyz.shape[0]
    N, sb, sc, sn = _pts(xyz, 2)
    S, cb, cc, cn = _pts(ctr, 2)
    if feat is not None:
        D = feat.shape[1]
        fb, fd, fn = feat.stride(0), feat.stride(1), feat.stride(2)
    else:
        D, fb, fd, fn = 0, 0, 0, 0
    ch = torch.tensor(list(chans), dtype=torch.int32)
    return (B, N, S, D), ch, (ptr(xyz), sb, sc, sn, N, ptr(ctr), cb, cc, cn, S, B, ptr(feat), fb, fd, fn, D,
                              ptr(count), ptr(lst), int(nsample), len(chans) - 1, ptr(ch))


def _bnm_ws(B, S, N, nsample, ch, backward, dev):
    nb = int(_lib.load().dvcp_sa_bnm_workspace_bytes(B, S, N, int(nsample), ch.numel() - 1, ch.data_ptr(),
                                                     int(backward)))
    if nb < 0:
        raise RuntimeError("dvcp_sa_bnm_workspace_bytes: size query failed")
    return torch.empty(max(1, (nb + 3) // 4), dtype=torch.float32, device=dev)


def sa_bnm_pre(feat, chans, pack):
    """U (B, N, C1) = W1[:, 3:] f_n + b1 for (B, D, N) point-major fp32 features: the per-point half
    of layer 1 that every dvcp_sa_bnm pass of a two-layer table starts from."""
    _lib.require_gpu(feat, pack)
    B, D, N = feat.shape
    C1 = int(chans[1])
    ch = torch.tensor(list(chans), dtype=torch.int32)
    U = torch.empty(B, N, C1, dtype=torch.float32, device=feat.device)
    call("dvcp_sa_bnm_pre", ptr(feat), feat.stride(0), feat.stride(2), N, B, len(chans) - 1, ch.data_ptr(), ptr(pack),
         ptr(U), stream(), work=(2.0 * B * N * D * C1, 4.0 * B * N * (D + C1)))
    return U


def sa_bnm_stats(xyz, ctr, feat, count, lst, nsample, chans, pack, U, layer):
    """Training-mode BatchNorm statistics on the matrix cores: (2, C_layer) fp64 = sum z, sum z^2 of
    layer ``layer``'s conv output over all B * S * nsample grouped entries."""
    (B, N, S, D), ch, args = _bnm_args(xyz, ctr, feat, count, lst, nsample, chans)
    ws = _bnm_ws(B, S, N, nsample, ch, False, xyz.device)
    sums = torch.empty(2, int(chans[layer]), dtype=torch.float64, device=xyz.device)
    macs = sum(a * b for a, b in zip(chans[:layer], chans[1:layer + 1]))
    call("dvcp_sa_bnm_pass", int(layer), *args, ptr(pack), ptr(U), None, None, None, None, ptr(ws), ptr(sums), None,
         None, stream(), work=(2.0 * macs * B * S * nsample, B * S * 4 * nsample + B * N * 4 * (3 + D)))
    return sums


def sa_bnm_forward(xyz, ctr, feat, count, lst, nsample, chans, pack, U):
    """The training-mode forward output (B, S, C_last) fp32 with batch statistics, plus each
    (centre, channel)'s first arg-max slot (int32) and that slot's z (what routes the backward)."""
    (B, N, S, D), ch, args = _bnm_args(xyz, ctr, feat, count, lst, nsample, chans)
    dev = xyz.device
    C = int(chans[-1])
    out = torch.empty(B, S, C, dtype=torch.float32, device=dev)
    arg = torch.empty(B, S, C, dtype=torch.int32, device=dev)
    zb = torch.empty(B, S, C, dtype=torch.float32, device=dev)
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))
    call("dvcp_sa_bnm_pass", 10, *args, ptr(pack), ptr(U), None, ptr(arg), ptr(out), ptr(zb), None, None, None, None,
         stream(), work=(2.0 * macs * B * S * nsample, B * S * (4 * nsample + 12 * C) + B * N * 4 * (3 + D)))
    return out, arg, zb


def sa_bnm_backward(xyz, ctr, feat, count, lst, nsample, chans, pack, U, fwd, grad_out, mode, want_feat_grad=False):
    """Training-mode backward on the matrix cores.  mode k >= 1: (2, C_k) fp64 = A_k, B_k (the pack
    holds A / M, B / M of the layers above); mode 0: (per layer dW | db fp32, dL/d feat (B, N, D)
    fp32 or None -- two-layer tables only)."""
    (B, N, S, D), ch, args = _bnm_args(xyz, ctr, feat, count, lst, nsample, chans)
    dev = xyz.device
    out, arg, _ = fwd
    g = grad_out.float().contiguous()
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))
    E = B * S * int(nsample)
    if mode > 0:
        ws = _bnm_ws(B, S, N, nsample, ch, False, dev)
        sums = torch.empty(2, int(chans[mode]), dtype=torch.float64, device=dev)
        call("dvcp_sa_bnm_pass", 20 + int(mode), *args, ptr(pack), ptr(U), ptr(g), ptr(arg), ptr(out), None, ptr(ws),
             ptr(sums), None, None, stream(), work=(4.0 * macs * E, E * 4 + B * N * 4 * (3 + D)))
        return sums
    ws = _bnm_ws(B, S, N, nsample, ch, True, dev)
    ngrad = sum(a * b + b for a, b in zip(chans[:-1], chans[1:]))
    grads = torch.empty(ngrad, dtype=torch.float32, device=dev)
    gF = torch.empty(B, N, D, dtype=torch.float32, device=dev) if (want_feat_grad and D > 0) else None
    call("dvcp_sa_bnm_pass", 30, *args, ptr(pack), ptr(U), ptr(g), ptr(arg), ptr(out), None, ptr(ws), None,
         ptr(grads), ptr(gF), stream(), work=(6.0 * macs * E, E * (8 + 4 * int(chans[1]))))
    return grads, gF


def fe_head_backward(x, params, grad):
    """Backward of the feature extractor's fc (deep_feat_extraction.py:15) on rows x (P, 64):
    (packed dW | db, dL/dx (P, 64))."""
    _lib.require_gpu(x, params, grad)
    P = x.shape[0]
    xc = x.float().contiguous()
    g = grad.reshape(P, 32).float().contiguous()
    ws = torch.empty(max(1, int(_lib.load().dvcp_fe_head_backward_workspace_bytes(P)) // 4), dtype=torch.float32,
                     device=x.device)
    gp = torch.empty(32 * 64 + 32, dtype=torch.float32, device=x.device)
    gx = torch.empty(P, 64, dtype=torch.float32, device=x.device)
    call("dvcp_fe_head_backward", ptr(xc), P, ptr(params), ptr(g), ptr(gx), ptr(ws), ptr(gp), stream())
    return gp, gx


def pose_inputs(x, y_pred, R_true, t_true):
    """deepVCP_loss.py's operands as the pose kernels take them: x, y_pred (B, 3, n) fp64
    contiguous; R_true (B, 3, 3), t_true (B, 3, 1) broadcast and contiguous."""
    x = x.double().contiguous()
    y_pred = y_pred.double().contiguous()
    B = x.shape[0]
    Rt = R_true.double().expand(B, 3, 3).contiguous()
    tt = t_true.double()
    if tt.dim() == 2:
        tt = tt.unsqueeze(0)
    if tt.shape[-1] != 1:
        raise RuntimeError("t_true must broadcast as (B, 3, 1)")
    return x, y_pred, Rt, tt.expand(B, 3, 1).contiguous()


def svd_optimization_backward(x, y_pred, R_true, t_true, partial, grad_loss, alpha):
    """dL/dy_pred (B, 3, n) fp64 of deepVCP_loss (deepVCP_loss.py:57-121); operands as
    ``pose_inputs`` returns them, ``partial`` from ``svd_optimization``."""
    _lib.require_gpu(x, y_pred, R_true, t_true, partial, grad_loss)
    B, _, n = x.shape
    g = torch.empty(B, 3, n, dtype=torch.float64, device=x.device)
    gl = grad_loss.double().reshape(1).contiguous()
    call("dvcp_svd_optimization_backward", ptr(x), ptr(y_pred), ptr(R_true), ptr(t_true), B, n,
         ptr(partial.contiguous()), ptr(gl), float(alpha), ptr(g), stream())
    return g


# ---- paper-faithful mode (dvcp/paper.py) -----------------------------------

def feature_propagation(xyz1, xyz2, p2_rows, p1, chans, relu, params):
    """pointnet2_utils.py:265-315 (PointNetFeaturePropagation) + an optional last linear layer:
    xyz1 (B, 3, N1), xyz2 (B, 3, N2) (any strides), p2_rows (B, N2, D2) fp32 with contiguous rows,
    p1 None or a (B, D1, N1) fp32 strided view -> (B, N1, chans[-1]) fp32."""
    _lib.require_gpu(xyz1, xyz2, p2_rows, params)
    B = xyz1.shape[0]
    N1, x1b, x1c, x1n = _pts(xyz1, 2)
    N2, x2b, x2c, x2n = _pts(xyz2, 2)
    if p2_rows.dtype != torch.float32 or p2_rows.stride(2) != 1:
        raise ValueError("feature_propagation: p2 rows must be fp32 with contiguous channels")
    D2 = p2_rows.shape[2]
    if p1 is not None:
        if p1.dtype != torch.float32:
            p1 = p1.float()
        D1, (p1b, p1d, p1n) = p1.shape[1], p1.stride()
    else:
        D1, p1b, p1d, p1n = 0, 0, 0, 0
    ch = torch.tensor(list(chans), dtype=torch.int32)
    rl = torch.tensor([int(bool(r)) for r in relu], dtype=torch.int32)
    out = torch.empty(B, N1, chans[-1], dtype=torch.float32, device=xyz1.device)
    macs = sum(a * b for a, b in zip(chans[:-1], chans[1:]))
    call("dvcp_feature_propagation", ptr(xyz1), x1b, x1c, x1n, N1, ptr(xyz2), x2b, x2c, x2n, N2, B, ptr(p1), p1b,
         p1d, p1n, D1, ptr(p2_rows), p2_rows.stride(0), p2_rows.stride(1), D2, len(chans) - 1, ptr(ch), ptr(rl),
         ptr(params), ptr(out), stream(),
         work=(B * N1 * (9.0 * N2 + 2.0 * macs), 4.0 * B * (3 * (N1 + N2) + N2 * D2 + N1 * (D1 + chans[-1]))))
    return out


def group_rows(ctr, xyz, feat, count, lst, nsample, radius, ctr_pdim=1, xyz_pdim=2):
    """Paper Sec. 3.3 DFE input: (B, Q, nsample, 3 + D) rows [(p - c) / radius, feat(p)] over the
    ball-query lists (first-hit padding; zero rows where a centre has no point in range)."""
    _lib.require_gpu(ctr, xyz, count, lst)
    B = ctr.shape[0]
    Q, cb, cc, cn = _pts(ctr, ctr_pdim)
    _, sb, sc, sn = _pts(xyz, xyz_pdim)
    D = 0 if feat is None else feat.shape[2]
    if feat is not None and (feat.dtype != torch.float32 or feat.stride(2) != 1):
        raise ValueError("group_rows: features must be (B, N, D) fp32 with contiguous rows")
    rows = torch.empty(B, Q, nsample, 3 + D, dtype=torch.float32, device=ctr.device)
    call("dvcp_group_rows", ptr(ctr), cb, cc, cn, Q, ptr(xyz), sb, sc, sn, ptr(feat),
         0 if feat is None else feat.stride(0), 0 if feat is None else feat.stride(1), D, ptr(count), ptr(lst),
         lst.shape[2], int(nsample), float(radius), B, ptr(rows), stream())
    return rows


def cpg1d(src, tgt, cand, params, want_weight=False):
    """Paper Sec. 3.6's 1-D CPG: src (B, K, 32), tgt (B, K, Gz, 32), cand (B, K, Gz, 3) -> vcp (B, K, 3)
    [, weights (B, K, Gz)]."""
    _lib.require_gpu(src, tgt, cand, params)
    B, K, Gz, _ = cand.shape
    s, t, c = src.reshape(B * K, 32).float().contiguous(), tgt.float().contiguous(), cand.float().contiguous()
    vcp = torch.empty(B, K, 3, dtype=torch.float32, device=cand.device)
    w = torch.empty(B, K, Gz, dtype=torch.float32, device=cand.device) if want_weight else None
    call("dvcp_cpg1d", ptr(s), ptr(t), ptr(c), B * K, Gz, ptr(params), ptr(vcp), ptr(w), stream(),
         work=(2.0 * 3 * (32 * 16 + 16 * 4 + 4) * B * K * Gz, 4.0 * B * K * (32 + Gz * 35 + 3)))
    return (vcp, w) if want_weight else vcp


def paper_pose(x, y, w, reflection_fix=True, inlier_ratio=1.0, R_true=None, t_true=None):
    """Weighted Kabsch with reflection fix and the paper's outlier rejection on (B, 3, n) fp64
    operands (w (B, n) or None) -> R (B, 3, 3), t (B, 3, 1)[, partial (B, 2) with R_true, t_true]."""
    _lib.require_gpu(x, y, w)
    x, y = x.double().contiguous(), y.double().contiguous()
    B, _, n = x.shape
    wc = None if w is None else w.double().reshape(B, n).contiguous()
    R = torch.empty(B, 3, 3, dtype=torch.float64, device=x.device)
    t = torch.empty(B, 3, 1, dtype=torch.float64, device=x.device)
    partial = torch.empty(B, 2, dtype=torch.float64, device=x.device) if R_true is not None else None
    call("dvcp_paper_pose", ptr(x), ptr(y), ptr(wc), B, n, int(bool(reflection_fix)), float(inlier_ratio),
         ptr(R_true), ptr(t_true), ptr(R), ptr(t), ptr(partial), stream())
    return (R, t) if partial is None else (R, t, partial)


def paper_pose_backward(x, y, w, R_true, t_true, alpha, grad_loss, reflection_fix=True, inlier_ratio=1.0,
                        want_w=True):
    """d loss / d y (B, 3, n) and d loss / d w (B, n) of the paper loss (dvcp_paper_pose_backward)."""
    _lib.require_gpu(x, y, R_true, t_true, grad_loss)
    B, _, n = x.shape
    gy = torch.empty(B, 3, n, dtype=torch.float64, device=x.device)
    gw = torch.empty(B, n, dtype=torch.float64, device=x.device) if (want_w and w is not None) else None
    gl = grad_loss.double().reshape(1).contiguous()   # alive across the launch
    call("dvcp_paper_pose_backward", ptr(x), ptr(y), ptr(w), B, n, int(bool(reflection_fix)), float(inlier_ratio),
         ptr(R_true), ptr(t_true), float(alpha), ptr(gl), ptr(gy), ptr(gw), stream())
    return gy, gw
