// keypoints.hip -- source key-point stage, one workgroup per cloud pair.
//
// Replaces, in order (REF-R):
//   deepVCP.py:44-46  (R2) keypts = index_points(fe_xyz, topk)
//   deepVCP.py:54     sample_and_group(npoint=K, radius=1, nsample=32, keypts, None, returnidx)
//                     -> FPS among the K key points (pointnet2_utils.py:63-84) and a ball query
//                        among them (:87-107); grouped = keypts[idx] - centre
//   deepVCP.py:62     src_keyfeats = fe_feat[picked]   (Q4: key-point-local indices into FE rows)
//   get_cat_feat_src.py:37-53  dist = ||(keypt - grouped) + 1e-6||, w = dist / sum_j dist,
//                     cat([grouped - keypt, feat * w])  (Q5)  -> .float() at the DFE input
//   deepVCP.py:86-91  (R3) moved = R_init @ keypts (fp64)
// Everything lives in LDS (K <= 256 points, nsample <= 32); rounding follows the torch ops.
#include "common.h"

namespace dvcp {

constexpr int kKpThreads = 256;
constexpr int kKpMaxK = 256;
constexpr int kKpMaxNs = 32;

template <typename T>
__global__ __launch_bounds__(kKpThreads) void src_keypoints_kernel(
    const T* __restrict__ fe_xyz, const float* __restrict__ fe_feat, int S, const int64_t* __restrict__ topk, int K,
    const int64_t* __restrict__ kstart, T r2, int ns, const double* __restrict__ R_init, int64_t r_b,
    T* __restrict__ keypts, float* __restrict__ src_cat, double* __restrict__ moved,
    const float* __restrict__ grad_cat, float* __restrict__ grad_feat) {  // backward: grad_cat -> grad_feat
  __shared__ T kx[kKpMaxK], ky[kKpMaxK], kz[kKpMaxK], kss[kKpMaxK];
  __shared__ int fidx[kKpMaxK];
  __shared__ int pidx[kKpMaxK * kKpMaxNs];
  __shared__ T dist[kKpMaxK * kKpMaxNs];
  __shared__ T dsum[kKpMaxK];
  __shared__ uint64_t slots[2][kKpThreads / kWave];

  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* X = fe_xyz + static_cast<int64_t>(b) * 3 * S;

  // 1. gather key points (top-k order)
  if (tid < K) {
    int64_t n = topk[static_cast<int64_t>(b) * K + tid];
    n = n < 0 ? 0 : (n >= S ? S - 1 : n);
    const T x = X[n], y = X[S + n], z = X[2 * S + n];
    kx[tid] = x;
    ky[tid] = y;
    kz[tid] = z;
    kss[tid] = sumsq3(x, y, z);
  }
  if (tid < K && !grad_cat) {
    const T x = kx[tid], y = ky[tid], z = kz[tid];
    T* o = keypts + (static_cast<int64_t>(b) * K + tid) * 3;
    o[0] = x;
    o[1] = y;
    o[2] = z;
    // R3: moved = R_init @ keypts, fp64, MKL dgemm rounding (fma chain over the 3 terms)
    const double* R = R_init + b * r_b;
    double* m = moved + (static_cast<int64_t>(b) * K + tid) * 3;
    const double dx = static_cast<double>(x), dy = static_cast<double>(y), dz = static_cast<double>(z);
#pragma unroll
    for (int a = 0; a < 3; ++a) m[a] = dot3_blas<double>(R[3 * a], R[3 * a + 1], R[3 * a + 2], dx, dy, dz);
  }
  __syncthreads();

  // 2. FPS among the K key points (fp32 running min, strict '<', first-index argmax)
  float dmin = tid < K ? 1e10f : -1.0f;
  int cur = static_cast<int>(kstart[b]);
  cur = cur < 0 || cur >= K ? 0 : cur;
  for (int step = 0; step < K; ++step) {
    if (tid == 0) fidx[step] = cur;
    const T cx = kx[cur], cy = ky[cur], cz = kz[cur];
    if (tid < K) {
      const T dx = kx[tid] - cx, dy = ky[tid] - cy, dz = kz[tid] - cz;
      const T d = (dx * dx + dy * dy) + dz * dz;
      if (d < static_cast<T>(dmin)) dmin = static_cast<float>(d);
    }
    const uint64_t mine = dmin >= 0.0f ? argmax_key(dmin, static_cast<uint32_t>(tid)) : 0ull;
    const uint64_t w = wave_max_u64(mine);
    if (lane == 0) slots[step & 1][wave] = w;
    lds_barrier();
    uint64_t m = slots[step & 1][0];
#pragma unroll
    for (int q = 1; q < kKpThreads / kWave; ++q) m = slots[step & 1][q] > m ? slots[step & 1][q] : m;
    cur = static_cast<int>(key_index(m));
  }
  __syncthreads();

  // 3. ball query among the key points: centre slot i = key point fidx[i]
  if (tid < K) {
    const int c = fidx[tid];
    const T cx = kx[c], cy = ky[c], cz = kz[c], ssc = kss[c];
    int cnt = 0, first = K;
    for (int j = 0; j < K && cnt < ns; ++j) {
      const T d2 = expansion_d2(dot3_blas(cx, cy, cz, kx[j], ky[j], kz[j]), ssc, kss[j]);
      if (!(d2 > r2)) {
        if (cnt == 0) first = j;
        pidx[tid * ns + cnt++] = j;
      }
    }
    for (int j = cnt; j < ns; ++j) pidx[tid * ns + j] = first;
  }
  __syncthreads();

  // 4. Get_Cat_Feat_Src distances: a = key point i (top-k order), g = grouped local coords
  const T eps = static_cast<T>(1e-6);
  for (int e = tid; e < K * ns; e += kKpThreads) {
    const int i = e / ns;
    const int c = fidx[i], p = pidx[e];
    const T gx = kx[p] - kx[c], gy = ky[p] - ky[c], gz = kz[p] - kz[c];
    const T ex = (kx[i] - gx) + eps, ey = (ky[i] - gy) + eps, ez = (kz[i] - gz) + eps;
    dist[e] = sqrt_rn(fma_rn<T>(ez, ez, fma_rn<T>(ey, ey, ex * ex)));
  }
  __syncthreads();
  if (tid < K) {
    T acc = 0;
    for (int j = 0; j < ns; ++j) acc += dist[tid * ns + j];
    dsum[tid] = acc;
  }
  __syncthreads();

  if (grad_cat) {  // backward of step 5's feature product (pointnet2_utils.py:59 gather, get_cat_feat_src.py:50)
    float* dF = grad_feat + static_cast<int64_t>(b) * S * 32;
    for (int e = tid; e < K * ns; e += kKpThreads) {
      const int i = e / ns, p = pidx[e];
      const T w = dist[e] / dsum[i];
      const float* g = grad_cat + (static_cast<int64_t>(b) * K * ns + e) * 35 + 3;
      for (int q = 0; q < 32; ++q)
        if (g[q] != 0.f) atomicAdd(dF + static_cast<int64_t>(p) * 32 + q, static_cast<float>(static_cast<T>(g[q]) * w));
    }
    return;
  }
  // 5. rows of the DFE input: [grouped - keypt (3), feat * w (32)] -> fp32
  const float* F = fe_feat + static_cast<int64_t>(b) * S * 32;
  for (int e = tid; e < K * ns; e += kKpThreads) {
    const int i = e / ns;
    const int c = fidx[i], p = pidx[e];
    const T w = dist[e] / dsum[i];
    float* o = src_cat + (static_cast<int64_t>(b) * K * ns + e) * 35;
    o[0] = static_cast<float>((kx[p] - kx[c]) - kx[i]);
    o[1] = static_cast<float>((ky[p] - ky[c]) - ky[i]);
    o[2] = static_cast<float>((kz[p] - kz[c]) - kz[i]);
    const float* f = F + static_cast<int64_t>(p) * 32;  // Q4: FE row p, p a key-point-local index
#pragma unroll 8
    for (int q = 0; q < 32; ++q) o[3 + q] = static_cast<float>(static_cast<T>(f[q]) * w);
  }
}

template <typename T>
static int launch_kp(const void* fe_xyz, const float* fe_feat, int S, const int64_t* topk, int B, int K,
                     const int64_t* kstart, double radius, int ns, const double* R, int64_t r_b, void* keypts,
                     float* src_cat, double* moved, hipStream_t st) {
  const T r2 = static_cast<T>(radius * radius);
  hipLaunchKernelGGL((src_keypoints_kernel<T>), dim3(B), dim3(kKpThreads), 0, st, static_cast<const T*>(fe_xyz),
                     fe_feat, S, topk, K, kstart, r2, ns, R, r_b, static_cast<T*>(keypts), src_cat, moved, nullptr,
                     nullptr);
  return launch_status("dvcp_src_keypoints");
}

}  // namespace dvcp

extern "C" int dvcp_src_keypoints(int dtype, const void* fe_xyz, const float* fe_feat, int S, const int64_t* topk,
                                  int B, int K, const int64_t* kstart, double radius, int nsample,
                                  const double* R_init, int64_t r_b, void* keypts, float* src_cat, double* moved,
                                  void* stream) {
  DVCP_REQUIRE(fe_xyz && fe_feat && topk && kstart && R_init && keypts && src_cat && moved,
               "dvcp_src_keypoints: null pointer");
  DVCP_REQUIRE(K > 0 && K <= dvcp::kKpMaxK && K <= S, "dvcp_src_keypoints: K=%d unsupported (1..256, <= S)", K);
  DVCP_REQUIRE(nsample > 0 && nsample <= dvcp::kKpMaxNs, "dvcp_src_keypoints: nsample=%d unsupported", nsample);
  // With K < nsample the reference's slice (pointnet2_utils.py:103) yields K columns and its
  // DFE MaxPool1d(32) then rejects the input; keep that case an error here too.
  DVCP_REQUIRE(K >= nsample, "dvcp_src_keypoints: K=%d < nsample=%d", K, nsample);
  if (B == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_kp<float>(fe_xyz, fe_feat, S, topk, B, K, kstart, radius, nsample, R_init, r_b, keypts,
                                  src_cat, moved, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_kp<double>(fe_xyz, fe_feat, S, topk, B, K, kstart, radius, nsample, R_init, r_b, keypts,
                                   src_cat, moved, st);
  dvcp::set_error("dvcp_src_keypoints: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

// Backward of the key-point stage's feature rows: grad_cat (B x K x ns x 35, the src_cat gradient)
// -> grad_feat (B x S x 32 fp32, accumulated: zero it first).  Re-runs steps 1-4 (key-point FPS,
// ball query, distance weights) exactly as the forward; only the 32 feature columns carry a
// gradient (the coordinates come from index ops).
extern "C" int dvcp_src_keypoints_backward(int dtype, const void* fe_xyz, int S, const int64_t* topk, int B, int K,
                                           const int64_t* kstart, double radius, int nsample, const float* grad_cat,
                                           float* grad_feat, void* stream) {
  DVCP_REQUIRE(K > 0 && K <= dvcp::kKpMaxK && K <= S && nsample > 0 && nsample <= dvcp::kKpMaxNs && K >= nsample,
               "dvcp_src_keypoints_backward: K=%d nsample=%d unsupported", K, nsample);
  if (B == 0) return DVCP_OK;
  DVCP_REQUIRE(fe_xyz && topk && kstart && grad_cat && grad_feat, "dvcp_src_keypoints_backward: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32) {
    const float r2 = static_cast<float>(radius * radius);
    hipLaunchKernelGGL((dvcp::src_keypoints_kernel<float>), dim3(B), dim3(dvcp::kKpThreads), 0, st,
                       static_cast<const float*>(fe_xyz), nullptr, S, topk, K, kstart, r2, nsample, nullptr, 0,
                       nullptr, nullptr, nullptr, grad_cat, grad_feat);
  } else if (dtype == DVCP_F64) {
    const double r2 = radius * radius;
    hipLaunchKernelGGL((dvcp::src_keypoints_kernel<double>), dim3(B), dim3(dvcp::kKpThreads), 0, st,
                       static_cast<const double*>(fe_xyz), nullptr, S, topk, K, kstart, r2, nsample, nullptr, 0,
                       nullptr, nullptr, nullptr, grad_cat, grad_feat);
  } else {
    dvcp::set_error("dvcp_src_keypoints_backward: bad dtype %d", dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_src_keypoints_backward");
}
