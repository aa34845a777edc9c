// knn.hip -- candidate grid (voxelize.py:19-83) and exact kNN (the un-vendored knn_cuda.KNN
// called at get_cat_feat_tgt.py:45,52 and deepVCP_loss.py:70,72; REF-R R6).
//
// kNN contract: fp32 d2 = (dx*dx + dy*dy) + dz*dz (dx = ref - query, no
// fma), ascending, ties to the lower index, dist = correctly rounded sqrt(d2).
//
// Design: one lane per query, 256 queries per workgroup.  Reference points are staged in LDS
// tiles (fp32 {x,y,z,_}, a broadcast ds_read_b128 per point) and each lane keeps its sorted
// top-KT list (distance + index) in VGPRs.  Points are scanned in ascending index order, so a
// strict '<' insertion keeps the lower index first on equal distances.  Insertion is a
// static-index shift network (no dynamic register indexing, no scratch).
#include "common.h"

namespace dvcp {

constexpr int kKnnThreads = 256;
constexpr int kKnnTile = 2048;

template <int KT>
__device__ __forceinline__ void topk_insert(float (&kd)[KT], int (&ki)[KT], float d, int i) {
  // kd sorted ascending; insert (d, i) after every entry <= d, dropping the last one.
#pragma unroll
  for (int t = KT - 1; t > 0; --t) {
    const bool here = d < kd[t];
    const bool before = d < kd[t - 1];
    kd[t] = before ? kd[t - 1] : (here ? d : kd[t]);
    ki[t] = before ? ki[t - 1] : (here ? i : ki[t]);
  }
  if (d < kd[0]) {
    kd[0] = d;
    ki[0] = i;
  }
}

template <typename T, int KT>
__global__ __launch_bounds__(kKnnThreads) void knn_kernel(PointsView<T> ref, int M, PointsView<T> qry, int Q, int k,
                                                          float* __restrict__ dist, int32_t* __restrict__ idx,
                                                          int64_t* __restrict__ idx64) {
  __shared__ float4 tile[kKnnTile];
  const int b = blockIdx.y;
  const int q = blockIdx.x * kKnnThreads + threadIdx.x;
  const bool live = q < Q;
  float qx = 0.f, qy = 0.f, qz = 0.f;
  if (live) {  // knn_cuda casts both inputs with .float()
    qx = static_cast<float>(qry.at(b, 0, q));
    qy = static_cast<float>(qry.at(b, 1, q));
    qz = static_cast<float>(qry.at(b, 2, q));
  }
  float kd[KT];
  int ki[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    kd[t] = __builtin_huge_valf();
    ki[t] = -1;
  }
  for (int t0 = 0; t0 < M; t0 += kKnnTile) {
    const int nt = min(kKnnTile, M - t0);
    __syncthreads();
    for (int j = threadIdx.x; j < nt; j += kKnnThreads)
      tile[j] = make_float4(static_cast<float>(ref.at(b, 0, t0 + j)), static_cast<float>(ref.at(b, 1, t0 + j)),
                            static_cast<float>(ref.at(b, 2, t0 + j)), 0.f);
    __syncthreads();
    for (int j = 0; j < nt; ++j) {
      const float4 p = tile[j];
      const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
      const float d2 = (dx * dx + dy * dy) + dz * dz;
      if (d2 < kd[KT - 1]) topk_insert<KT>(kd, ki, d2, t0 + j);
    }
  }
  if (!live) return;
  const int64_t o = (static_cast<int64_t>(b) * Q + q) * k;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    if (t < k) {
      if (dist) dist[o + t] = sqrt_rn(kd[t]);
      if (idx) idx[o + t] = ki[t];
      if (idx64) idx64[o + t] = ki[t];
    }
  }
}

// torch.arange(start, end, s) values fp32(fma(s, i, start)) with start = (c - r) - s/2,
// end = c + r, all in fp64 (voxelize.py:62-64; torch's CPU arange kernel is compiled with fma
// contraction, visible at zero crossings); length ceil((end - start)/s) must equal G (cpg.py:29-30).
template <typename T>
__global__ void voxelize_kernel(PointsView<T> pts, int Kp, double r, double s, int G, float* __restrict__ cand,
                                int32_t* __restrict__ err) {
  const int C = G * G * G;
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (gid >= static_cast<int64_t>(Kp) * C) return;
  const int kp = static_cast<int>(gid / C), c = static_cast<int>(gid % C);
  const int ii[3] = {c / (G * G), (c / G) % G, c % G};
  float* o = cand + (static_cast<int64_t>(b) * Kp * C + gid) * 3;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double m = static_cast<double>(pts.at(b, a, kp));
    const double lo = m - r, hi = m + r;
    const double start = lo - s / 2;
    if (err && c == 0 && static_cast<int>(ceil((hi - start) / s)) != G) *err = 1;
    o[a] = static_cast<float>(__fma_rn(s, static_cast<double>(ii[a]), start));
  }
}

template <typename T>
static int launch_knn(const void* ref, int64_t rb, int64_t rc, int64_t rn, int M, const void* qry, int64_t qb,
                      int64_t qc, int64_t qn, int Q, int B, int k, float* dist, int32_t* idx, int64_t* idx64,
                      hipStream_t st) {
  PointsView<T> rv{static_cast<const T*>(ref), rb, rc, rn};
  PointsView<T> qv{static_cast<const T*>(qry), qb, qc, qn};
  dim3 grid(ceil_div(Q, kKnnThreads), B);
#define DVCP_KNN(KK)                                                                                          \
  if (k <= KK) {                                                                                              \
    hipLaunchKernelGGL((knn_kernel<T, KK>), grid, dim3(kKnnThreads), 0, st, rv, M, qv, Q, k, dist, idx, idx64); \
    return launch_status("dvcp_knn");                                                                         \
  }
  DVCP_KNN(1)
  DVCP_KNN(4)
  DVCP_KNN(8)
  DVCP_KNN(16)
  DVCP_KNN(32)
#undef DVCP_KNN
  set_error("dvcp_knn: k=%d > 32 unsupported", k);
  return DVCP_EINVAL;
}

}  // namespace dvcp

extern "C" int dvcp_knn(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M, const void* qry,
                        int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k, float* dist, int32_t* idx,
                        int64_t* idx64, void* stream) {
  DVCP_REQUIRE(ref && qry, "dvcp_knn: null pointer");
  DVCP_REQUIRE(k > 0 && M >= 0 && Q >= 0 && B >= 0, "dvcp_knn: bad sizes");
  DVCP_REQUIRE(B <= 65535, "dvcp_knn: B too large");
  if (B == 0 || Q == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_knn<float>(ref, rb, rc, rn, M, qry, qb, qc, qn, Q, B, k, dist, idx, idx64, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_knn<double>(ref, rb, rc, rn, M, qry, qb, qc, qn, Q, B, k, dist, idx, idx64, st);
  dvcp::set_error("dvcp_knn: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

extern "C" int dvcp_voxelize(int dtype, const void* pts, int64_t pb, int64_t pc, int64_t pn, int B, int Kp,
                             double r, double s, int G, float* cand, int32_t* err, void* stream) {
  DVCP_REQUIRE(pts && cand, "dvcp_voxelize: null pointer");
  DVCP_REQUIRE(G > 0 && s > 0 && B <= 65535, "dvcp_voxelize: bad arguments");
  if (B == 0 || Kp == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t total = static_cast<int64_t>(Kp) * G * G * G;
  dim3 grid(dvcp::ceil_div(total, 256), B);
  if (dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::voxelize_kernel<float>), grid, dim3(256), 0, st,
                       dvcp::PointsView<float>{static_cast<const float*>(pts), pb, pc, pn}, Kp, r, s, G, cand, err);
  else if (dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::voxelize_kernel<double>), grid, dim3(256), 0, st,
                       dvcp::PointsView<double>{static_cast<const double*>(pts), pb, pc, pn}, Kp, r, s, G, cand, err);
  else {
    dvcp::set_error("dvcp_voxelize: bad dtype %d", dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_voxelize");
}
