// dfe.hip -- deep feature embedding (deep_feat_embedding.py:23-61).
//
//   X.float(); fc1 (35->32), fc2 (32->32), fc3 (32->32), NO nonlinearity (Q14, kept
//   un-collapsed); MaxPool1d(32) over the neighbour axis.
//
// dvcp_dfe     : materialised input rows (the source side, B*K*32 rows).
// dvcp_dfe_tgt : target side fused with get_cat_feat_tgt.py:54-96 -- the (B,K,C,32,35) fp64
//                tensor (763 MB per pair at C=1331) is never materialised; each row is
//                gathered and weighted in registers straight from the kNN output.
//
// One thread = one neighbour row, 8 queries x 32 rows = 256 threads per workgroup.  Weights
// are wave-uniform scalar loads; the max over a query's 32 rows goes through LDS.
#include "common.h"

#include <cstdlib>

namespace dvcp {

// dfe_mfma.hip: the target side on fp32 MFMA (default; DVCP_DFE_VALU=1 selects the kernel below)
template <typename T>
int launch_dfe_tgt_mfma(PointsView<T> ref, const float* feat, int M, const float* cand, const float* dist,
                        const int32_t* idx, int B, int Q, const float* params, float* out, hipStream_t st);

static bool dfe_valu_forced() {
  static const bool v = [] {
    const char* e = getenv("DVCP_DFE_VALU");
    return e && *e && *e != '0';
  }();
  return v;
}

constexpr int kDfeRowsPerQ = 32;
constexpr int kDfeThreads = 256;
constexpr int kDfeQPerBlock = kDfeThreads / kDfeRowsPerQ;

__device__ __forceinline__ void dfe_mlp(const float (&x)[35], float (&y)[32], const float* __restrict__ params) {
  float h1[32], h2[32];
  linear_sgpr<35, 32>(x, h1, params);
  const float* p2 = params + 35 * 32 + 32;
  linear_sgpr<32, 32>(h1, h2, p2);
  linear_sgpr<32, 32>(h2, y, p2 + 32 * 32 + 32);
}

// rows -> per-query max over the 32 rows (rows of query ql are threads ql*32 .. ql*32+31)
__device__ __forceinline__ void dfe_pool_store(const float (&y)[32], float (*red)[33], int64_t q0, int64_t nq,
                                               float* __restrict__ out) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int c = 0; c < 32; ++c) red[tid][c] = y[c];
  __syncthreads();
  const int ql = tid / 32, c = tid % 32;
  if (q0 + ql < nq) {
    float m = red[ql * 32][c];
#pragma unroll 8
    for (int j = 1; j < 32; ++j) m = fmaxf(m, red[ql * 32 + j][c]);
    out[(q0 + ql) * 32 + c] = m;
  }
}

template <typename XT>
__global__ __launch_bounds__(kDfeThreads) void dfe_kernel(const XT* __restrict__ X, int64_t R,
                                                          const float* __restrict__ params, float* __restrict__ out) {
  __shared__ float red[kDfeThreads][33];
  const int64_t q0 = static_cast<int64_t>(blockIdx.x) * kDfeQPerBlock;
  const int64_t row = q0 * kDfeRowsPerQ + threadIdx.x;
  float x[35];
  if (row < R * kDfeRowsPerQ) {
    const XT* src = X + row * 35;
#pragma unroll
    for (int i = 0; i < 35; ++i) x[i] = static_cast<float>(src[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 35; ++i) x[i] = 0.f;
  }
  float y[32];
  dfe_mlp(x, y, params);
  dfe_pool_store(y, red, q0, R, out);
}

template <typename T>
__global__ __launch_bounds__(kDfeThreads) void dfe_tgt_kernel(PointsView<T> ref, const float* __restrict__ feat, int M,
                                                              const float* __restrict__ cand,
                                                              const float* __restrict__ dist,
                                                              const int32_t* __restrict__ idx, int Q,
                                                              const float* __restrict__ params,
                                                              float* __restrict__ out) {
  __shared__ float red[kDfeThreads][33];
  __shared__ double wq[kDfeQPerBlock][32];
  const int b = blockIdx.y;
  const int tid = threadIdx.x, ql = tid / 32, j = tid % 32;
  const int64_t q0 = static_cast<int64_t>(blockIdx.x) * kDfeQPerBlock;
  const int64_t q = q0 + ql;
  const bool live = q < Q;
  const int64_t kq = (static_cast<int64_t>(b) * Q + (live ? q : 0)) * 32;
  // get_cat_feat_tgt.py:57-58: dist_sum in fp64, w = dist / dist_sum (fp64)
  const float dj = live ? dist[kq + j] : 1.0f;
  double s = static_cast<double>(dj);
  // fixed-order fp64 sum over the query's 32 neighbours (lanes ql*32 .. ql*32+31)
  __shared__ double dsh[kDfeThreads];
  dsh[tid] = s;
  __syncthreads();
  double acc = 0.0;
  for (int t = 0; t < 32; ++t) acc += dsh[ql * 32 + t];
  wq[ql][j] = static_cast<double>(dj) / acc;
  __syncthreads();

  float x[35];
  int n = live ? idx[kq + j] : 0;
  n = n < 0 ? 0 : (n >= M ? M - 1 : n);
  const float* cq = cand + (static_cast<int64_t>(b) * Q + (live ? q : 0)) * 3;
  // candidates_grouped_local = tgt_pts_picked - candidate (tgt xyz dtype, then .float())
  x[0] = static_cast<float>(ref.at(b, 0, n) - static_cast<T>(cq[0]));
  x[1] = static_cast<float>(ref.at(b, 1, n) - static_cast<T>(cq[1]));
  x[2] = static_cast<float>(ref.at(b, 2, n) - static_cast<T>(cq[2]));
  // tgt_feat_norm[j, f] = F[idx_j, f] * w[f]   (Q10: weight indexed by the feature channel)
  const float4* fr = reinterpret_cast<const float4*>(feat + (static_cast<int64_t>(b) * M + n) * 32);
#pragma unroll
  for (int f4 = 0; f4 < 8; ++f4) {
    const float4 v = fr[f4];
    x[3 + 4 * f4 + 0] = static_cast<float>(static_cast<double>(v.x) * wq[ql][4 * f4 + 0]);
    x[3 + 4 * f4 + 1] = static_cast<float>(static_cast<double>(v.y) * wq[ql][4 * f4 + 1]);
    x[3 + 4 * f4 + 2] = static_cast<float>(static_cast<double>(v.z) * wq[ql][4 * f4 + 2]);
    x[3 + 4 * f4 + 3] = static_cast<float>(static_cast<double>(v.w) * wq[ql][4 * f4 + 3]);
  }
  float y[32];
  dfe_mlp(x, y, params);
  dfe_pool_store(y, red, static_cast<int64_t>(b) * Q + q0,
                 static_cast<int64_t>(b) * Q + min(static_cast<int64_t>(Q), q0 + kDfeQPerBlock), out);
}

}  // namespace dvcp

extern "C" int dvcp_dfe(int x_dtype, const void* X, int64_t R, const float* params, float* out, void* stream) {
  DVCP_REQUIRE(X && params && out, "dvcp_dfe: null pointer");
  if (R <= 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(dvcp::ceil_div(R, dvcp::kDfeQPerBlock));
  if (x_dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::dfe_kernel<float>), grid, dim3(dvcp::kDfeThreads), 0, st, static_cast<const float*>(X), R,
                       params, out);
  else if (x_dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::dfe_kernel<double>), grid, dim3(dvcp::kDfeThreads), 0, st, static_cast<const double*>(X),
                       R, params, out);
  else {
    dvcp::set_error("dvcp_dfe: bad dtype %d", x_dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_dfe");
}

extern "C" int dvcp_dfe_tgt(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                            const float* ref_feat, const float* cand, const float* dist, const int32_t* idx, int B, int Q,
                            const float* params, float* out, void* stream) {
  DVCP_REQUIRE(ref_xyz && ref_feat && cand && dist && idx && params && out, "dvcp_dfe_tgt: null pointer");
  DVCP_REQUIRE(M > 0 && B <= 65535, "dvcp_dfe_tgt: bad sizes");
  if (B == 0 || Q == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!dvcp::dfe_valu_forced()) {
    if (dtype == DVCP_F32)
      return dvcp::launch_dfe_tgt_mfma<float>(dvcp::PointsView<float>{static_cast<const float*>(ref_xyz), rb, rc, rn},
                                              ref_feat, M, cand, dist, idx, B, Q, params, out, st);
    if (dtype == DVCP_F64)
      return dvcp::launch_dfe_tgt_mfma<double>(
          dvcp::PointsView<double>{static_cast<const double*>(ref_xyz), rb, rc, rn}, ref_feat, M, cand, dist, idx, B,
          Q, params, out, st);
  }
  dim3 grid(dvcp::ceil_div(Q, dvcp::kDfeQPerBlock), B);
  if (dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::dfe_tgt_kernel<float>), grid, dim3(dvcp::kDfeThreads), 0, st,
                       dvcp::PointsView<float>{static_cast<const float*>(ref_xyz), rb, rc, rn}, ref_feat, M, cand, dist,
                       idx, Q, params, out);
  else if (dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::dfe_tgt_kernel<double>), grid, dim3(dvcp::kDfeThreads), 0, st,
                       dvcp::PointsView<double>{static_cast<const double*>(ref_xyz), rb, rc, rn}, ref_feat, M, cand,
                       dist, idx, Q, params, out);
  else {
    dvcp::set_error("dvcp_dfe_tgt: bad dtype %d", dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_dfe_tgt");
}
