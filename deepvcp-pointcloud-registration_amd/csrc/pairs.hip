// pairs.hip -- rigid transform of point clouds for training-pair synthesis on the GPU.
//
// Replaces the numpy transform of the reference's datasets:
//   KITTIDataset.py:80-81       target_points = R @ src_points + t          (src fp32, R/t fp64)
//   ModelNet40Dataset.py:74-85  target_points = R @ src_points (+ t later), target_normal = R @ src_normals
// numpy promotes the fp32 source to fp64 and multiplies through BLAS; the K = 3 product here is
// the same fma chain the fp64 gemm kernels use, fma(R2, x2, fma(R1, x1, R0 * x0)), then + t.
#include "common.h"

namespace dvcp {

template <typename T>
__global__ void rigid_apply_kernel(PointsView<T> in, int N, int C, const double* __restrict__ R,
                                   const double* __restrict__ t, int64_t t_b, double* __restrict__ out) {
  const int b = blockIdx.y;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const double* Rb = R + static_cast<int64_t>(b) * 9;
  double* ob = out + static_cast<int64_t>(b) * C * N;
  for (int g = 0; g < C; g += 3) {  // channel groups: xyz (+ t), then normals (rotated only)
    const double x = static_cast<double>(in.at(b, g, n)), y = static_cast<double>(in.at(b, g + 1, n)),
                 z = static_cast<double>(in.at(b, g + 2, n));
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double v = __fma_rn(Rb[3 * c + 2], z, __fma_rn(Rb[3 * c + 1], y, Rb[3 * c] * x));
      if (g == 0 && t) v += t[b * t_b + c];
      ob[static_cast<int64_t>(g + c) * N + n] = v;
    }
  }
}

}  // namespace dvcp

extern "C" int dvcp_rigid_apply(int dtype, const void* in, int64_t ib, int64_t ic, int64_t in_n, int B, int N, int C,
                                const double* R, const double* t, int64_t t_b, double* out, void* stream) {
  DVCP_REQUIRE(in && R && out, "dvcp_rigid_apply: null pointer");
  DVCP_REQUIRE(C == 3 || C == 6, "dvcp_rigid_apply: C=%d (3 = xyz, 6 = xyz + normals)", C);
  DVCP_REQUIRE(B >= 0 && B <= 65535 && N >= 0, "dvcp_rigid_apply: bad sizes");
  if (B == 0 || N == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid(dvcp::ceil_div(N, 256), B);
  if (dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::rigid_apply_kernel<float>), grid, dim3(256), 0, st,
                       dvcp::PointsView<float>{static_cast<const float*>(in), ib, ic, in_n}, N, C, R, t, t_b, out);
  else if (dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::rigid_apply_kernel<double>), grid, dim3(256), 0, st,
                       dvcp::PointsView<double>{static_cast<const double*>(in), ib, ic, in_n}, N, C, R, t, t_b, out);
  else {
    dvcp::set_error("dvcp_rigid_apply: bad dtype %d", dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_rigid_apply");
}
