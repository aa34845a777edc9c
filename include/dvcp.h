/* dvcp.h -- C ABI of libdvcp_hip.so, the MI355X (gfx950) DeepVCP registration hot path.
 *
 * The reference (vccheng2001/DeepVCP-Pointcloud-Registration) has no FFI: its boundary is
 * the Python nn.Module / free-function surface.  Each entry point below
 * replaces one reference interface, cited as file:line.  The Python host package
 * (deepvcp-pointcloud-registration_amd/dvcp) binds them with ctypes and mirrors the
 * reference module surface on top.
 *
 * Conventions
 *   - Plain pointers and sizes, no torch types.  All buffers are device pointers allocated
 *     by the caller; the library never allocates, frees or retains them.
 *   - Strided point inputs: coordinate c (0..2) of point n of batch b lives at
 *     p[b*sb + c*sc + n*sn] (element strides).  This covers both the reference's
 *     channel-first (B,C,N) tensors and (B,N,3) rows without a copy.
 *   - dtype: DVCP_F32 or DVCP_F64 for coordinate tensors (feature tensors are fp32, as the
 *     reference's .float() casts make them).
 *   - Every call is asynchronous on `stream` (a hipStream_t; NULL = default stream), never
 *     synchronises the host and is safe to capture into a hipGraph.
 *   - Return 0 on success, a negative DVCP_E* code otherwise; dvcp_last_error() gives a
 *     thread-local message.
 */
#ifndef DVCP_H
#define DVCP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVCP_F32 0
#define DVCP_F64 1

#define DVCP_OK 0
#define DVCP_EINVAL (-1)    /* bad argument / unsupported shape */
#define DVCP_EHIP (-2)      /* HIP launch error */

/* Bumped on every incompatible signature change; dvcp/_lib.py refuses a library whose version differs. */
#define DVCP_ABI_VERSION 4

const char* dvcp_last_error(void);
int dvcp_abi_version(void);

/* Farthest point sampling.  Replaces pointnet2_utils.py:63-84 farthest_point_sample.
 * xyz: B x N points (strided, dtype); start: B int64 start indices (the reference draws them
 * with torch.randint on the CPU generator, :75 -- the caller does the same);
 * out_idx: B x npoint int64; out_xyz (optional, may be NULL): B x 3 x npoint of dtype
 * (the sampled centres, channel-first = the reference's new_xyz.permute(0,2,1)).
 * Running minimum kept in fp32 for both dtypes (:74,:82), strict '<' update (:81),
 * first-index argmax (:83). */
int dvcp_fps(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
             int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz, void* stream);

/* dvcp_fps with a B x N fp32 workspace, required when N exceeds the register-resident limit
 * (16384 fp32 / 8192 fp64 points per cloud).  Such clouds are split over ceil(N / 16384)
 * workgroups (8192 fp64) that exchange one argmax key per step through device-scope atomics.
 * With DVCP_FPS_PARTS=2|4|8 in the environment, fp32 clouds of 2048..16384 points whose
 * exchange slots fit in B x N x 4 bytes run their select rounds on that many workgroups per
 * cloud, exchanging one candidate list per round (the split select, csrc/fps.hip FpsPartArgs;
 * dvcp_fps_parts chooses per call, and takes it by default above 16384 points, where its
 * workspace exceeds B x N x 4).  Same indices either way.  err (optional int32, zeroed by the
 * caller): set to 1 if a workgroup gave up waiting for its peers (a guard; the indices then stay
 * in range but are not FPS). */
int dvcp_fps_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz, float* ws,
                int32_t* err, void* stream);

/* Bytes of workspace dvcp_fps_parts needs for B clouds of N points (>= B x N x 4). */
int64_t dvcp_fps_workspace_bytes(int B, int N);

/* dvcp_fps_ws with a sized workspace (ws_bytes >= dvcp_fps_workspace_bytes(B, N), 8-byte aligned)
 * and the split select's workgroups per cloud: parts = 0 (the library's choice: 8 above 16384
 * fp32 points, else 1 unless DVCP_FPS_PARTS says), 1 (the one-workgroup select kernel; above 16384
 * points the per-step split kernel), 2, 4 or 8 (the split select: fp32, 2048 <= N <= 65536; 8
 * above 32768 points).  Same contract and results as dvcp_fps; err as for dvcp_fps_ws.  The
 * product path (dvcp/ops.py fps) calls this. */
int dvcp_fps_parts(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                   int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz, void* ws,
                   int64_t ws_bytes, int32_t* err, int parts, void* stream);

/* Two chained full-permutation FPS layers in one launch (the FE's layers 2 and 3 at C3:
 * pointnet2_utils.py:63-84 called by deep_feat_extraction.py:28 and :29 with npoint equal to the
 * layer's point count).  Bit-identical to dvcp_fps(xyz, N, start2) -> (idx2, xyz2) followed by
 * dvcp_fps(xyz2, N, start3) -> (idx3, xyz3); the second layer runs beside the first from the
 * point the first picks at step start3 (clouds whose second-layer argmax meets a tie are
 * recomputed in the serial order).  fp32, 2048 <= N <= 16384; xyz2 / xyz3 B x 3 x N contiguous;
 * ws: dvcp_fps_pair_workspace_bytes(B, N) bytes, 4-byte aligned, reserved for this call. */
int64_t dvcp_fps_pair_workspace_bytes(int B, int N);
int dvcp_fps_pair(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                  const int64_t* start2, const int64_t* start3, int64_t* idx2, void* xyz2,
                  int64_t* idx3, void* xyz3, void* ws, void* stream);

/* Measurement probe (no reference counterpart): `blocks` workgroups each run `steps` steps of
 * the FPS chain's per-step synchronisation with no point work (wave DPP argmax, LDS slot, one
 * barrier, slot reduction); out: blocks floats.  bench.py times it as the latency floor. */
int dvcp_fps_step_floor(int steps, int blocks, float* out, void* stream);

/* Test hook of the split FPS guard (no reference counterpart): the split path of dvcp_fps_ws
 * for N in (16384, 262144] fp32 / (8192, 131072] fp64, with at most spin_cap polls per wait and
 * `withhold` workgroups left out of the grid, so that the last cloud cannot complete and must
 * raise *err. */
int dvcp_fps_split_probe(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B,
                         int N, int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz,
                         float* ws, int32_t* err, uint32_t spin_cap, int withhold, void* stream);

/* Ball query.  Replaces pointnet2_utils.py:87-107 query_ball_point (and the
 * square_distance expansion it uses, :19-40): the first `nsample` ascending point indices
 * whose d2 = ((-2*dot) + |c|^2) + |p|^2 is not > radius^2 (dot = MKL's fma chain).
 * xyz: B x N points, ctr: B x S centres (both strided, dtype).
 * Outputs (each optional): count B x S int32 (number of distinct hits, <= nsample),
 * list B x S x nsample int32 (the hits, ascending; entries >= count undefined),
 * padded B x S x nsample int64 (reference format: padded with the first hit, or N if
 * there is none). */
int dvcp_ball_query(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                    const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                    double radius, int nsample, int32_t* count, int32_t* list,
                    int64_t* padded, void* stream);
/* The same with a device workspace of dvcp_ball_query_workspace_bytes(B, N, S) bytes (fp32
 * only; ignored for fp64).  Identical results.  For N <= 16384 points are Morton-sorted into
 * 64-point tiles and each wave of 64 Morton-consecutive centres scans, in ascending index order,
 * only the points a rounding-safe box bound cannot exclude; otherwise each wave streams all points
 * in index order as scalar loads with its own early exit. */
int64_t dvcp_ball_query_workspace_bytes(int B, int N, int S);
int dvcp_ball_query_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                       const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                       double radius, int nsample, int32_t* count, int32_t* list,
                       int64_t* padded, void* workspace, void* stream);

/* Dense expansion-form squared distance, pointnet2_utils.py:19-40 (API completeness).
 * out: B x S x N of dtype. */
int dvcp_square_distance(int dtype, const void* src, int64_t sb, int64_t sc, int64_t sn, int S,
                         const void* dst, int64_t db, int64_t dc, int64_t dn, int N, int B,
                         void* out, void* stream);

/* Grouped set-abstraction MLP.  Replaces pointnet2_utils.py:122-132 (grouping) +
 * :195-200 ([Conv2d 1x1 + BN2d(eval) + ReLU] x L, max over nsample).  Rows are the
 * distinct ball-query hits (count/list of dvcp_ball_query): the reference's padded
 * duplicates repeat the first hit, so the max is identical.
 * Row input = [ (p - c) cast to fp32 (3), feature (D) ]; features are read as
 * feat[b*fb + d*fd + n*fn] of dtype feat_dtype (fp32 or fp64, cast to fp32), or NULL when D=0.
 * Layers: nlayer in {2,3}; chans = {C0=3+D, C1, ..., C_nlayer}; for layer l:
 * W_l (C_{l+1} x C_l), bias_l, bn_scale_l, bn_shift_l (all fp32) packed back-to-back in
 * `params` in that order, layer by layer.  y = relu((W x + bias) * scale + shift).
 * out: B x S x C_last fp32 (row-major per centre).  A centre with count 0 (no hit; the reference
 * would gather the padding index N) gets a zero row, and its list row is not read. */
int dvcp_sa_group_mlp(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                      const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                      int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                      const int32_t* count, const int32_t* list, int nsample,
                      int nlayer, const int* chans, const float* params, float* out,
                      void* stream);

/* dvcp_sa_group_mlp with a device workspace of dvcp_sa_group_mlp_workspace_bytes(B, N, S,
 * nlayer, chans) bytes (16-B aligned; 0 bytes = none needed, NULL allowed).  N = points of
 * xyz/feat, S = centres.  For the two-layer fp32 tables (sa2 35-32-64, sa3 67-64-64) layer 1 is
 * split into its per-point part U = W1[:, 3:] f + b1, evaluated once per input point into the
 * workspace, and the per-(centre, point) part W1[:, :3] (p - c); same results up to fp32
 * summation order.  Centres are visited in Hilbert-curve order (also kept in the workspace) so
 * the gathered rows of concurrently running waves stay in L2; the order does not change results. */
int64_t dvcp_sa_group_mlp_workspace_bytes(int B, int N, int S, int nlayer, const int* chans);
int dvcp_sa_group_mlp_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                         const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                         int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                         const int32_t* count, const int32_t* list, int nsample,
                         int nlayer, const int* chans, const float* params, float* out,
                         void* workspace, void* stream);

/* dvcp_sa_group_mlp_ws for the two-layer tables with the features given through a row map:
 * point n of cloud b takes row feat_rows[b * N + n] (int64, clamped to [0, Nf)) of the fp32
 * point-major table feat (cloud stride fb, row stride fn, 16-B aligned rows, Nf rows per cloud).
 * This folds the gather of the previous layer's per-point rows by its FPS order
 * (pointnet2_utils.py:59 index_points on the layer's new_points) into the MLP's per-point
 * pre-pass, so the gathered table is never written.  Needs the workspace. */
int dvcp_sa_group_mlp_rows_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                              const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                              const float* feat, int64_t fb, int64_t fn, int Nf, int D,
                              const int64_t* feat_rows, const int32_t* count, const int32_t* list,
                              int nsample, int nlayer, const int* chans, const float* params, float* out,
                              void* workspace, void* stream);

/* Per-point affine + weighting MLP.  Replaces deep_feat_extraction.py:15 (fc, applied per
 * REF-R R1) and weighting_layer.py:26-30 (Linear 32-16-8-1, ReLU, ReLU, Softplus).
 * x: P x 64 fp32 -> feat: P x 32 fp32 (= fc(x)); score (optional, may be NULL): P fp32.
 * params: fc.W(32x64), fc.b(32) [, wl1.W(16x32), wl1.b, wl2.W(8x16), wl2.b, wl3.W(1x8), wl3.b]. */
int dvcp_fe_head(const float* x, int P, const float* params, float* feat, float* score,
                 void* stream);

/* dvcp_fe_head on rows gathered per cloud: output row i reads x row (i / S) * Nx + rows[i]
 * (int64, clamped to [0, Nx)); P = clouds x S.  Folds the gather of sa3's per-point rows by its
 * FPS order (pointnet2_utils.py:59) into the head's load. */
int dvcp_fe_head_rows(const float* x, const int64_t* rows, int S, int Nx, int P, const float* params,
                      float* feat, float* score, void* stream);

/* Weighting layer alone.  Replaces weighting_layer.py:26-30 on given features:
 * feat: P x 32 fp32 -> score: P fp32.  params: wl1.W(16x32), wl1.b, wl2.W(8x16), wl2.b,
 * wl3.W(1x8), wl3.b. */
int dvcp_weighting(const float* feat, int P, const float* params, float* score, void* stream);

/* Top-K per row (descending value, ties to the lower index).  Replaces
 * weighting_layer.py:31 torch.topk(X, K, dim=1).  score: B x S fp32 -> idx: B x K int64. */
int dvcp_topk(const float* score, int B, int S, int K, int64_t* idx, void* stream);

/* Source key-point stage, one workgroup per pair.  Replaces deepVCP.py:44-68 +
 * get_cat_feat_src.py:16-55 with REF-R R2/R7 and deepVCP.py:86-91 (R3):
 *   keypts = fe_xyz[topk]; FPS among the K key points (start = kstart[b]);
 *   ball query r=radius, nsample among them; src_cat = [grouped - keypt, F[picked]*w] (Q4,Q5);
 *   moved = R_init[b] @ keypts (fp64).
 * fe_xyz: B x 3 x S (dtype, channel-first), fe_feat: B x S x 32 fp32, topk: B x K int64,
 * R_init: B x 3 x 3 fp64 (row stride r_b: 0 broadcasts one matrix).
 * Outputs: keypts B x K x 3 (dtype), src_cat B x K x nsample x 35 fp32 (the DFE input after
 * its .float()), moved B x K x 3 fp64. */
int dvcp_src_keypoints(int dtype, const void* fe_xyz, const float* fe_feat, int S,
                       const int64_t* topk, int B, int K, const int64_t* kstart,
                       double radius, int nsample, const double* R_init, int64_t r_b,
                       void* keypts, float* src_cat, double* moved, void* stream);

/* Candidate grid.  Replaces voxelize.py:19-83: cand[b,k,(ix*G+iy)*G+iz,a] =
 * fp32(fma(s, i_a, (c_a - r) - s/2)) evaluated in fp64 (torch.arange, Q9).
 * pts: B x Kp points (strided, dtype) -> cand: B x Kp x G^3 x 3 fp32.
 * err (optional int32): set to 1 if a point's per-axis arange length differs from G. */
int dvcp_voxelize(int dtype, const void* pts, int64_t pb, int64_t pc, int64_t pn, int B, int Kp,
                  double r, double s, int G, float* cand, int32_t* err, void* stream);

/* Exact k-nearest neighbours (R6 contract: fp32 d2 = (dx*dx+dy*dy)+dz*dz, ascending, ties to
 * the lower index, dist = sqrt(d2)).  Replaces knn_cuda.KNN (get_cat_feat_tgt.py:45,52;
 * deepVCP_loss.py:70,72).  ref: B x M points, qry: B x Q points (both strided, dtype; cast to
 * fp32 like knn_cuda).  Outputs (B x Q x k): dist fp32, idx int32 and/or idx64 int64 (any may
 * be NULL).  k <= 32. */
int dvcp_knn(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M,
             const void* qry, int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k,
             float* dist, int32_t* idx, int64_t* idx64, void* stream);

/* Exact kNN through a uniform cell grid (same contract and outputs as dvcp_knn).  The reference
 * set is counting-sorted into cells once per cloud, then each query scans Chebyshev shells of
 * cells around its home cell until no unscanned cell can hold a point at or below its k-th
 * distance.  workspace: dvcp_knn_grid_workspace_bytes(B, M) bytes of device memory. */
int dvcp_knn_grid(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M,
                  const void* qry, int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k,
                  void* workspace, float* dist, int32_t* idx, int64_t* idx64, void* stream);
int64_t dvcp_knn_grid_workspace_bytes(int B, int M);

/* Exact kNN over spatially sorted reference tiles: same contract and results as dvcp_knn
 * (replaces knn_cuda.KNN at get_cat_feat_tgt.py:45,52).  References are Morton-sorted into
 * 16-point tiles with boxes and queries into Morton order; each wave of 64 queries scans tiles in
 * ascending lower-bound order and stops once no unscanned tile can hold a point at or below any
 * lane's k-th distance.  For k > 16 each lane buffers its candidates in LDS and the wave merges
 * them into the sorted lists with bitonic networks.  M <= 16384, k <= 32.
 * workspace: dvcp_knn_tiled_workspace_bytes(B, M, Q) bytes of device memory. */
int dvcp_knn_tiled(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M,
                   const void* qry, int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k,
                   void* workspace, float* dist, int32_t* idx, int64_t* idx64, void* stream);
/* dvcp_knn_tiled with every candidate inserted into the sorted list at once, for every k (the
 * round-2 kernel): a second exact implementation for the parity tests and A/B timing. */
int dvcp_knn_tiled_insert(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M,
                          const void* qry, int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k,
                          void* workspace, float* dist, int32_t* idx, int64_t* idx64, void* stream);
int64_t dvcp_knn_tiled_workspace_bytes(int B, int M, int Q);

/* Deep feature embedding on a materialised input.  Replaces deep_feat_embedding.py:23-61
 * (X.float(); Linear 35-32-32-32, no activations; MaxPool1d(32) over the neighbour axis).
 * X: R x 32 x 35 rows of x_dtype (fp32/fp64) contiguous -> out: R x 32 fp32.
 * params: fc1.W(32x35), fc1.b, fc2.W(32x32), fc2.b, fc3.W(32x32), fc3.b. */
int dvcp_dfe(int x_dtype, const void* X, int64_t R, const float* params, float* out,
             void* stream);

/* Target-side fused gather + DFE.  Replaces get_cat_feat_tgt.py:54-96 (R4, R5, Q10) +
 * deep_feat_embedding.py:47-60 without materialising the (B,K,C,32,35) fp64 tensor.
 * For query q with neighbours j (idx/dist from dvcp_knn, k = 32):
 *   X[j] = [ (ref[idx_j] - cand_q) -> fp32 (3),
 *            fp32( F[idx_j, f] * (double(dist_f) / sum_j double(dist_j)) ) (32) ]
 * ref_xyz: B x M (strided, dtype), ref_feat: B x M x 32 fp32, cand: B x Q x 3 fp32.
 * out: B x Q x 32 fp32. */
int dvcp_dfe_tgt(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                 const float* ref_feat, const float* cand, const float* dist, const int32_t* idx,
                 int B, int Q, const float* params, float* out, void* stream);

/* (x, y, z, 0) float4 rows of B clouds of M fp32 points (xyz strided like ref_xyz above) into out
 * (B x M x 4 fp32, 16-byte aligned).  dvcp_dfe_tgt / dvcp_dfe_tgt_f16 given fp32 points in this
 * layout (rb = 4 M, rc = 1, rn = 4) gather a neighbour's coordinates as one 16-byte load instead
 * of three scattered 4-byte loads; the results are the same bits either way.  (Added in ABI 3
 * without a version change: no existing entry point changed.) */
int dvcp_points_pack4(const float* xyz, int64_t sb, int64_t sc, int64_t sn, int M, int B, float* out,
                      void* stream);

/* dvcp_dfe_tgt with the target feature table stored as fp16 (ref_feat: B x M x 32 IEEE halves) --
 * BASELINE C5's "fp16 features" storage, half the gathered feature bytes.  Each gathered row is
 * widened to fp32 and the rest is dvcp_dfe_tgt's fp32 arithmetic: the output equals dvcp_dfe_tgt
 * on the fp32 table holding the same (fp16-rounded) values.  Not reference precision (the
 * reference keeps fp32/fp64 features); an opt-in storage mode (DeepVCP(feat_dtype=float16)). */
int dvcp_dfe_tgt_f16(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                     const uint16_t* ref_feat, const float* cand, const float* dist, const int32_t* idx,
                     int B, int Q, const float* params, float* out, void* stream);

/* dvcp_dfe_tgt evaluating fc1, fc2, fc3 one after the other exactly as deep_feat_embedding.py:
 * 48-50 chains them.  dvcp_dfe_tgt instead collapses the three linear
 * layers into one 32 x 35 map (formed in fp64, rounded once to fp32); both agree within fp32
 * rounding (tests/test_gpu_kernels.py). */
int dvcp_dfe_tgt_literal(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                         const float* ref_feat, const float* cand, const float* dist,
                         const int32_t* idx, int B, int Q, const float* params, float* out,
                         void* stream);

/* Backward of dvcp_sa_group_mlp with eval-mode BatchNorm (running statistics; the frozen-BN
 * training mode), replacing autograd through pointnet2_utils.py:176-202 (+ the index_points gather
 * of the grouped features, :59).  Same geometry arguments and folded `params` as the forward;
 * bnstat: per layer running_mean (C_l) | 1/sqrt(running_var + eps) (C_l).
 * grad_out: B x S x C_last fp32 (dL/d output).  grad_feat (optional): B x N x D fp32, ACCUMULATED
 * (the caller zeroes it): dL/d feat through the grouping.  grad_params: per layer dW (C_{l+1} x C_l),
 * db, dgamma, dbeta (fp32, packed in that order).  torch.max routes each channel's gradient to the
 * first row holding the maximum.  Tables: sa1 (3[+3]-16-16-32), sa2 (35-32-64), sa3 (67-64-64).
 * workspace: dvcp_sa_group_mlp_backward_workspace_bytes(B, S, nlayer, chans) bytes. */
int64_t dvcp_sa_group_mlp_backward_workspace_bytes(int B, int S, int nlayer, const int* chans);
int dvcp_sa_group_mlp_backward(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                               const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                               int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn,
                               int D, const int32_t* count, const int32_t* list, int nsample,
                               int nlayer, const int* chans, const float* params,
                               const float* bnstat, const float* grad_out, float* grad_feat,
                               void* workspace, float* grad_params, void* stream);

/* The grouped set-abstraction MLP with BatchNorm in TRAINING mode (batch statistics) --
 * pointnet2_utils.py:195-200 with the module in train() (train.py:105-125 trains the whole model).
 * Same grouping arguments as dvcp_sa_group_mlp_backward.  pack: per layer l (C_l -> C_{l+1})
 * W (C_{l+1} x C_l) | conv bias | scale | shift | batch mean | 1/sqrt(batch var + eps) | A/M | B/M
 * (fp32; dvcp_sa_bn_pack_floats(nlayer, chans) floats), scale = gamma * istd, shift = beta -
 * mean * scale, M = B * S * nsample grouped entries (padding slots included), A_l / B_l the
 * batch-norm backward sums of layer l (zero until known).
 * dvcp_sa_bn_stats: sums (2 x C_layer fp64) = per-channel sum z and sum z^2 of the conv output of
 *   `layer` (1-based) over all M entries, the layers below it normalised by their pack entries.
 *   zrows (optional, layer = nlayer only): also write dvcp_sa_bn_zrows's output (every lower
 *   layer's statistics are final by then), so the backward needs no z-row pass of its own.
 * dvcp_sa_bn_zrows: zrows (dvcp_sa_bn_zrows_floats floats) = every entry's conv output z_l of
 *   every layer, channel-major (C_l x M per layer, entry e = centre * nsample + slot), with the
 *   pack's final batch statistics; the backward reads them instead of recomputing the MLP.
 * dvcp_sa_bn_backward(mode): mode = k >= 1 -> sums (2 x C_k fp64) = A_k = sum dL/dy_k (dbeta) and
 *   B_k = sum dL/dy_k * xhat_k (dgamma), needing A, B of the layers above k (mode = nlayer needs
 *   none); mode = 0 -> rows (dvcp_sa_bn_rows_floats floats): per layer l, dL/dz_l of every entry
 *   (C_l x M, channel-major) then the layer's input rows and a ones row (C_{l-1} + 1 x M), so
 *   [dW_l | db_l] = dz_l [h_{l-1}; 1]^T is a plain GEMM over the entries (the host runs it); and,
 *   if grad_feat is given, dL/d feat (B x N x D fp32) through the grouping: for D = 32 / 64
 *   overwritten with per-point sums of per-entry rows taken in entry order (deterministic; mode-0
 *   workspace: dvcp_sa_bn_feat_workspace_bytes(B, S, nsample, N, D) bytes), for other D
 *   accumulated with float atomics (zero it first).
 *   grad_out: B x S x C_last fp32.  workspace (modes >= 1): dvcp_sa_bn_workspace_bytes bytes.
 * Replaces the training-mode forward/backward of pointnet2_utils.py:176-202 (BatchNorm2d batch
 * statistics, running-stat update done by the host). */
int64_t dvcp_sa_bn_pack_floats(int nlayer, const int* chans);
int64_t dvcp_sa_bn_workspace_bytes(int B, int S, int nlayer, const int* chans);
int64_t dvcp_sa_bn_rows_floats(int B, int S, int nsample, int nlayer, const int* chans);
int64_t dvcp_sa_bn_feat_workspace_bytes(int B, int S, int nsample, int N, int D);
int64_t dvcp_sa_bn_zrows_floats(int B, int S, int nsample, int nlayer, const int* chans);
int dvcp_sa_bn_zrows(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                     const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                     int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                     const int32_t* count, const int32_t* list, int nsample, int nlayer,
                     const int* chans, const float* pack, float* zrows, void* stream);
int dvcp_sa_bn_stats(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                     const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                     int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                     const int32_t* count, const int32_t* list, int nsample, int nlayer,
                     const int* chans, const float* pack, int layer, void* workspace,
                     double* sums, float* zrows, void* stream);
int dvcp_sa_bn_backward(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                        const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                        int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn,
                        int D, const int32_t* count, const int32_t* list, int nsample, int nlayer,
                        const int* chans, const float* pack, const float* zrows, int mode,
                        const float* grad_out, float* grad_feat, void* workspace, double* sums,
                        float* rows, void* stream);

/* The same training-mode forward / backward on the matrix cores (csrc/sa_bn_mfma.hip) for the
 * REF-R tables sa1 (3[+3]-16-16-32), sa2 (35-32-64) and sa3 (67-64-64): nothing per entry is
 * stored, every pass recomputes the MLP per 32-entry tile.  fp32 points / centres / features
 * (feat[b fb + d fd + n fn]; the two-layer tables need point-major rows, fd = 1, 16-byte
 * aligned); pack and the grouping as dvcp_sa_bn_stats.  Replaces pointnet2_utils.py:176-202 in
 * train() (train.py:105-125).
 * dvcp_sa_bnm_supported(nlayer, chans): 1 for those tables.
 * dvcp_sa_bnm_pre (two-layer tables): U (B x N x C1 fp32) = W1[:, 3:] f_n + b1, the per-point half
 *   of layer 1 every pass of the call starts from (NULL for sa1).
 * dvcp_sa_bnm_pass(pass):
 *   1..nlayer: sums (2 x C_pass fp64) = sum z, sum z^2 of layer `pass` over the M entries;
 *   10: the forward -- out (B S x C_last) = max over slots of relu(y_last), arg = its first
 *       arg-max slot, zbest = that slot's z_last;
 *   20 + k (k < nlayer): sums (2 x C_k fp64) = A_k, B_k (needs A, B of the layers above in the
 *       pack; the last layer's: A = sum of grad_out where out > 0, B = the same weighted by
 *       xhat(zbest), summed by the host);
 *   30: grads = per layer dW | db (fp32, dvcp_sa_bn_pack order without the BN vectors) and, for
 *       the two-layer tables if grad_feat is given, dL/d feat (B x N x D fp32); fixed-order sums.
 *   grad_out: B S x C_last fp32; arg / out / zbest: pass 10's outputs (read by passes 20+, 30).
 *   workspace: dvcp_sa_bnm_workspace_bytes(B, S, N, nsample, nlayer, chans, backward = pass 30).
 *   A centre without hits (count 0; FPS centres always hit themselves, so the reference never
 *   has one) is treated here as the ball query's padded form describes it: count clamped to 1,
 *   so its nsample slots are nsample copies of list entry 0 (point 0), counted in the batch
 *   statistics, and its output row is the MLP of that entry.  (The eval tables,
 *   dvcp_sa_group_mlp*, give such a centre a zero row instead.)
 */
int dvcp_sa_bnm_supported(int nlayer, const int* chans);
int64_t dvcp_sa_bnm_workspace_bytes(int B, int S, int N, int nsample, int nlayer, const int* chans,
                                    int backward);
int dvcp_sa_bnm_pre(const float* feat, int64_t fb, int64_t fn, int N, int B, int nlayer,
                    const int* chans, const float* pack, float* U, void* stream);
int dvcp_sa_bnm_pass(int pass, const float* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                     const float* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                     const float* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                     const int32_t* count, const int32_t* list, int nsample, int nlayer,
                     const int* chans, const float* pack, const float* U, const float* grad_out,
                     int32_t* arg, float* out, float* zbest, void* workspace, double* sums,
                     float* grads, float* grad_feat, void* stream);

/* Backward of the feature extractor's fc (deep_feat_extraction.py:15, Linear 64 -> 32):
 * x: P x 64 fp32 (its input rows), params: fc.W (32 x 64) | fc.b (32), grad: P x 32;
 * grad_x (optional): P x 64; grad_params: dW (32 x 64) | db (32), summed in fixed order.
 * workspace: dvcp_fe_head_backward_workspace_bytes(P) bytes. */
int64_t dvcp_fe_head_backward_workspace_bytes(int P);
int dvcp_fe_head_backward(const float* x, int P, const float* params, const float* grad,
                          float* grad_x, void* workspace, float* grad_params, void* stream);

/* Paper-faithful pose solve (DeepVCP paper Sec. 3.4-3.5; NOT reference
 * parity -- the reference's get_rigid_transform, deepVCP_loss.py:13-44, is unweighted with no
 * reflection fix): weighted Kabsch with per-point weights w (B x n fp64, NULL = uniform),
 * centroids sum(w x) / sum(w), and with reflection_fix the det-sign correction
 * R = V diag(1,1,sign det(V U^T)) U^T.  inlier_ratio in (0, 1]: below 1, the paper's outlier
 * rejection -- the int(inlier_ratio n) pairs with the smallest |R x + t - y| under the first
 * solve (ties: the lower index) are solved again (n <= 1024).  x, y: B x 3 x n fp64 ->
 * R (B x 3 x 3), t (B x 3 x 1).  partial (optional, B x 2 fp64, needs R_true (B x 3 x 3) and
 * t_true (B x 3 x 1)): per pair sum |R_true x + t_true - y| and sum |R_true x + t_true - (R x + t)|
 * (the paper's two L1 terms, on every key point). */
int dvcp_paper_pose(const double* x, const double* y, const double* w, int B, int n, int reflection_fix,
                    double inlier_ratio, const double* R_true, const double* t_true, double* R, double* t,
                    double* partial, void* stream);
/* Backward of the paper loss alpha * S1 / (3 B n) + (1 - alpha) * S2 / (3 B n) (S1, S2 the sums
 * of dvcp_paper_pose's partial) in y and w: grad_loss (1 fp64, device) -> grad_y (B x 3 x n),
 * grad_w (B x n, optional).  The rejection's selection carries no gradient (piecewise constant);
 * the second solve does (weighted Procrustes derivative, reflection fix included). */
int dvcp_paper_pose_backward(const double* x, const double* y, const double* w, int B, int n,
                             int reflection_fix, double inlier_ratio, const double* R_true,
                             const double* t_true, double alpha, const double* grad_loss, double* grad_y,
                             double* grad_w, void* stream);

/* Paper-faithful mode, PointNet++ feature propagation (paper Sec. 3.1 + supplement; the
 * reference's own PointNetFeaturePropagation, pointnet2_utils.py:265-315, which it never calls):
 * for every xyz1 point (B x N1, strided) the 3 nearest xyz2 points (B x N2, strided) under the
 * expansion-form squared distance (:296; ties to the lower index), weights 1/(d + 1e-8)
 * normalised (:300-302), the interpolated p2 rows (B x N2 x D2 point-major, strides p2b, p2n)
 * appended to the p1 rows (B x D1 x N1 strided, optional) (:305-307); then nlayer layers
 * chans[0] = D1 + D2 -> ... -> chans[nlayer] (<= 64), each y = (W x + b) * scale + shift
 * (packed W | b | scale | shift per layer: eval BN folded) with ReLU where relu[l] != 0 (:312-314;
 * a last layer with relu 0, scale 1, shift 0 is a plain fully connected layer).
 * out: B x N1 x chans[nlayer] fp32. */
int dvcp_feature_propagation(const float* xyz1, int64_t x1b, int64_t x1c, int64_t x1n, int N1,
                             const float* xyz2, int64_t x2b, int64_t x2c, int64_t x2n, int N2, int B,
                             const float* p1, int64_t p1b, int64_t p1d, int64_t p1n, int D1,
                             const float* p2, int64_t p2b, int64_t p2n, int D2, int nlayer,
                             const int* chans, const int* relu, const float* params, float* out,
                             void* stream);
/* Paper-faithful mode, the DFE input of paper Sec. 3.3: rows [(p - c) / radius, feat(p)] for
 * every centre (B x Q, strided) over its ball-query list (count B x Q, list B x Q x ns_list from
 * dvcp_ball_query), padded with the first hit (pointnet2_utils.py:104-106) up to ns_out; a centre
 * with no point within radius gets zero rows.  xyz: B x N strided, feat: B x N x D point-major.
 * rows: B x Q x ns_out x (3 + D) fp32. */
int dvcp_group_rows(const float* ctr, int64_t cb, int64_t cc, int64_t cn, int Q, const float* xyz,
                    int64_t sb, int64_t sc, int64_t sn, const float* feat, int64_t fb, int64_t fn, int D,
                    const int32_t* count, const int32_t* list, int ns_list, int ns_out, double radius, int B,
                    float* rows, void* stream);
/* Paper-faithful mode, the duplicated network's CPG (paper Sec. 3.6): per key point the cost
 * (src - tgt)^2 over its Gz (<= 64) candidates on a z line, Conv1d 32-16-4-1 (k 3, p 1, no
 * activations), softmax over the line, vcp = sum(w cand) / sum(w).  src: P x 32, tgt: P x Gz x 32,
 * cand: P x Gz x 3 fp32; params: conv1.W | b | conv2.W | b | conv3.W | b (dvcp_cpg1d_nparams()
 * floats, torch Conv1d layout); vcp: P x 3, weight (optional): P x Gz. */
int dvcp_cpg1d(const float* src, const float* tgt, const float* cand, int P, int Gz, const float* params,
               float* vcp, float* weight, void* stream);
int dvcp_cpg1d_nparams(void);

/* Corresponding point generation.  Replaces cpg.py:27-60: cost volume
 * (src - scrambled tgt)^2 (Q11), Conv3d 32-16-4-1 (k3, p1, no activations), softmax over C,
 * vcp = sum(w*cand)/sum(w).
 * src: P x 32 fp32 (P = B*K key points); tgt: the reference's (B,K,32,C) tensor given by
 * element strides (t_p per key point, t_f per feature, t_c per candidate);
 * cand: P x C x 3 fp32; params: conv1.W(16x32x27), conv1.b, conv2.W(4x16x27), conv2.b,
 * conv3.W(1x4x27), conv3.b.  out: P x 3 fp32; weight (optional): P x C softmax weights. */
int dvcp_cpg(const float* src, const float* tgt, int64_t t_p, int64_t t_f, int64_t t_c,
             const float* cand, int P, int G, const float* params, float* vcp, float* weight,
             void* stream);

/* Kabsch.  Replaces deepVCP_loss.py:13-44 get_rigid_transform: x, y: B x 3 x n fp64
 * (contiguous) -> R: B x 3 x 3, t: B x 3 x 1 (fp64). R = V U^T, no reflection fix (Q13). */
int dvcp_rigid_transform(const double* x, const double* y, int B, int n, double* R, double* t,
                         void* stream);

/* Two-pass pose solve.  Replaces deepVCP_loss.py:57-90 svd_optimization (+ the loss terms of
 * :105-121).  x, y_pred: B x 3 x n fp64; R_true: B x 3 x 3; t_true: B x 3 x 1 (fp64).
 * Outputs: R2 B x 3 x 3, t2 B x 3 x 1, x1 / y_pred2 (optional) B x 3 x n_in with
 * n_in = int(n * 0.8); partial (optional) B x 2: per pair sum|y_pred2 - y_true1| and
 * sum(y_pred2 - y_true1) for the loss. */
int dvcp_svd_optimization(const double* x, const double* y_pred, const double* R_true,
                          const double* t_true, int B, int n, double* R2, double* t2,
                          double* x1, double* y2, double* partial, void* stream);

/* Registration error of the reference's training/eval harness (train.py:112-120 and :156-164, with
 * crash C8 fixed: translation error over the three components).  Per pair b:
 *   rot_err[b]   = || euler_xyz_deg(R_pred[b]) - euler_xyz_deg(R_gt[b]) + 1e-6 ||_2
 *   trans_err[b] = || t_pred[b] - t_gt[b] + 1e-6 ||_2
 * euler_xyz_deg = scipy Rotation.from_matrix(.).as_euler('xyz', degrees=True); nn.PairwiseDistance
 * adds its eps (1e-6) to the difference.  R_pred: B x 3 x 3, t_pred: B x 3 fp64 (contiguous);
 * R_gt / t_gt rows at element strides rg_b / tg_b (0 broadcasts one pose).  rot_err is NaN where a
 * matrix has det <= 0 (scipy raises there). */
int dvcp_registration_error(const double* R_pred, const double* t_pred, const double* R_gt, int64_t rg_b,
                            const double* t_gt, int64_t tg_b, int B, double* rot_err, double* trans_err,
                            void* stream);

/* Training-pair synthesis: out = R x (+ t) per cloud, in fp64.  Replaces the numpy transform of
 * KITTIDataset.py:80-81 (target = R @ src + t) and ModelNet40Dataset.py:74-85 (points rotated
 * and translated, normals rotated).  in: B x C x N (strided, dtype; C = 3 xyz or 6 xyz+normals),
 * R: B x 3 x 3 fp64, t: B x 3 fp64 at row stride t_b (NULL: no translation; 0 broadcasts),
 * out: B x C x N fp64 contiguous (channels 0-2 translated, 3-5 rotated only). */
int dvcp_rigid_apply(int dtype, const void* in, int64_t ib, int64_t ic, int64_t in_n, int B, int N, int C,
                     const double* R, const double* t, int64_t t_b, double* out, void* stream);

/* ---- Backward (training: train.py:105-125 loss.backward()).  Gradients of the parameters come
 * back packed in the forward's params layout, summed over the batch in a fixed order. ---- */

/* deepVCP_loss backward.  Replaces autograd through deepVCP_loss.py:57-121 (torch.svd backward of
 * :29 twice, the gathers of :81-82): dL/dy_pred (B x 3 x n fp64) for
 * loss = alpha*mean|y_true1 - y2| + (1-alpha)*|mean(y2 - y_true1)|.  partial: the forward's
 * (B x 2) per-pair sums; grad_loss: device scalar dL/dloss. */
/* deepVCP_loss.py:105-121 in full: dvcp_svd_optimization (x1, y2 not returned) plus the scalar
 * loss alpha * mean|y2 - y_true1| + (1 - alpha) * |mean(y2 - y_true1)| (loss: 1 fp64, partial:
 * B x 2 fp64 scratch that also feeds dvcp_svd_optimization_backward). */
int dvcp_deepvcp_loss(const double* x, const double* y_pred, const double* R_true, const double* t_true,
                      int B, int n, double alpha, double* R2, double* t2, double* partial, double* loss,
                      void* stream);

int dvcp_svd_optimization_backward(const double* x, const double* y_pred, const double* R_true,
                                   const double* t_true, int B, int n, const double* partial,
                                   const double* grad_loss, double alpha, double* grad_y_pred,
                                   void* stream);

/* Feature-embedding backward.  Replaces autograd through deep_feat_embedding.py:23-61 (fc1-3,
 * MaxPool1d) for the materialised rows X (R x 32 x 35, fp32|fp64): grad_out R x 32 fp32 ->
 * grad_params (3264 fp32: W1, b1, W2, b2, W3, b3) and, optionally, grad_X (R x 32 x 35 fp32).
 * ws: dvcp_dfe_backward_workspace_bytes(R). */
int64_t dvcp_dfe_backward_workspace_bytes(int64_t R);
int dvcp_dfe_backward(int x_dtype, const void* X, int64_t R, const float* params, const float* grad_out,
                      float* ws, float* grad_params, float* grad_X, void* stream);

/* Target-side backward.  Replaces autograd through get_cat_feat_tgt.py:54-96 +
 * deep_feat_embedding.py:47-60; same arguments as dvcp_dfe_tgt plus grad_out (B x Q x 32 fp32),
 * ws (dvcp_dfe_tgt_backward_workspace_bytes(B, Q, M, grad_ref_feat != NULL); -1: the size query
 * failed) and grad_params (3264 fp32).  grad_ref_feat (optional, B x M x 32 fp32, overwritten)
 * receives the gradient of the gathered target features (the get_cat_feat_tgt.py:85 gather,
 * weighted as :95), summed per target row in a fixed order (a stable radix sort of the routed
 * entries by target row): bit-identical run to run.  Needs B*Q*32 < 2^31 and B*M < 2^31. */
int64_t dvcp_dfe_tgt_backward_workspace_bytes(int B, int Q, int M, int want_feat_grad);
int dvcp_dfe_tgt_backward(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                          const float* ref_feat, const float* cand, const float* dist, const int32_t* idx,
                          int B, int Q, const float* params, const float* grad_out, float* ws,
                          float* grad_params, float* grad_ref_feat, void* stream);

/* Key-point stage backward.  Replaces autograd through the source feature gather
 * (pointnet2_utils.py:59 index_points, deepVCP.py:62) and its weighting (get_cat_feat_src.py:50):
 * dvcp_src_keypoints' inputs plus grad_cat (B x K x nsample x 35, the src_cat gradient) ->
 * grad_feat (B x S x 32 fp32, accumulated: zero it first). */
int dvcp_src_keypoints_backward(int dtype, const void* fe_xyz, int S, const int64_t* topk, int B, int K,
                                const int64_t* kstart, double radius, int nsample, const float* grad_cat,
                                float* grad_feat, void* stream);

/* CPG backward.  Replaces autograd through cpg.py:27-60: dvcp_cpg's arguments plus grad_vcp
 * (P x 3) -> grad_src (P x 32), grad_tgt (P x 32 x C contiguous, the (B,K,32,C) tensor's
 * logical order), grad_params (15681 fp32).  ws: dvcp_cpg_backward_workspace_bytes(P). */
int64_t dvcp_cpg_backward_workspace_bytes(int P);
int dvcp_cpg_backward(const float* src, const float* tgt, int64_t t_p, int64_t t_f, int64_t t_c,
                      const float* cand, int P, int G, const float* params, const float* grad_vcp,
                      float* grad_src, float* grad_tgt, float* ws, float* grad_params, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DVCP_H */
