// fps.hip -- farthest point sampling (replaces pointnet2_utils.py:63-84).
//
// One 1024-thread workgroup per cloud; FPS is a strictly serial chain of `npoint` argmax
// steps, so the design minimises the latency of one step:
//   * every point lives in VGPRs for the whole launch (PPT points per thread, strided by
//     1024 so each thread scans its points in ascending index order);
//   * the running minimum is fp32 for both coordinate dtypes (:74, :82) and is updated
//     with a strict '<' (:81);
//   * argmax = one 64-bit key max (value, then lowest index: torch.max's first index,
//     :83) by wave shuffles, then ONE barrier per step: each wave publishes {key, x, y, z}
//     of its winner into a double-buffered LDS slot and every thread reduces the 16 slots,
//     so the next centre's coordinates never come from global memory.
#include "common.h"

namespace dvcp {

template <typename T>
struct alignas(16) FpsSlot {
  uint64_t key;
  T x, y, z;
};

template <typename T, int PPT>
__global__ __launch_bounds__(1024) void fps_kernel(PointsView<T> pts, int N, int npoint,
                                                   const int64_t* __restrict__ start,
                                                   int64_t* __restrict__ out_idx,
                                                   T* __restrict__ out_xyz) {
  constexpr int NT = 1024;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6;
  __shared__ FpsSlot<T> slots[2][NT / kWave];

  T px[PPT], py[PPT], pz[PPT];
  float dmin[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int n = tid + p * NT;
    if (n < N) {
      px[p] = pts.at(b, 0, n);
      py[p] = pts.at(b, 1, n);
      pz[p] = pts.at(b, 2, n);
      dmin[p] = 1e10f;  // torch.ones(B, N) * 1e10 (fp32), :74
    } else {
      px[p] = py[p] = pz[p] = static_cast<T>(0);
      dmin[p] = -1.0f;  // never updated (d >= 0) and never selected
    }
  }

  int64_t cur = start[b];
  if (cur < 0 || cur >= N) cur = 0;  // host validates; keep the kernel in bounds regardless
  T cx = pts.at(b, 0, cur), cy = pts.at(b, 1, cur), cz = pts.at(b, 2, cur);

  int64_t* oi = out_idx + static_cast<int64_t>(b) * npoint;
  T* ox = out_xyz ? out_xyz + static_cast<int64_t>(b) * 3 * npoint : nullptr;

  for (int step = 0; step < npoint; ++step) {
    if (tid == 0) {
      oi[step] = cur;
      if (ox) {
        ox[step] = cx;
        ox[npoint + step] = cy;
        ox[2 * npoint + step] = cz;
      }
    }
    float bestv = -1.0f;
    int bestp = 0;
    T bx = 0, by = 0, bz = 0;
#pragma unroll
    for (int p = 0; p < PPT; ++p) {
      const T dx = px[p] - cx, dy = py[p] - cy, dz = pz[p] - cz;
      const T d = (dx * dx + dy * dy) + dz * dz;  // torch.sum((xyz - c) ** 2, -1), :80
      if (d < static_cast<T>(dmin[p])) dmin[p] = static_cast<float>(d);
      if (dmin[p] > bestv) {  // strict: the earlier (lower) index keeps a tie
        bestv = dmin[p];
        bestp = p;
        bx = px[p];
        by = py[p];
        bz = pz[p];
      }
    }
    const uint64_t mine = bestv >= 0.0f ? argmax_key(bestv, static_cast<uint32_t>(tid + bestp * NT)) : 0ull;
    const uint64_t wmax = wave_max_u64(mine);
    FpsSlot<T>* buf = slots[step & 1];
    if (mine == wmax) {
      buf[wave].key = wmax;
      buf[wave].x = bx;
      buf[wave].y = by;
      buf[wave].z = bz;
    }
    __syncthreads();
    uint64_t best = buf[0].key;
    int wsel = 0;
#pragma unroll
    for (int w = 1; w < NT / kWave; ++w) {
      const uint64_t k = buf[w].key;
      if (k > best) {
        best = k;
        wsel = w;
      }
    }
    cur = static_cast<int64_t>(key_index(best));
    cx = buf[wsel].x;
    cy = buf[wsel].y;
    cz = buf[wsel].z;
  }
}

template <typename T>
static int launch_fps(const T* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                      const int64_t* start, int64_t* out_idx, T* out_xyz, hipStream_t st) {
  PointsView<T> v{xyz, sb, sc, sn};
  const int ppt = ceil_div(N, 1024);
  dim3 grid(B), block(1024);
#define DVCP_FPS_CASE(P)                                                                          \
  if (ppt <= P) {                                                                                 \
    hipLaunchKernelGGL((fps_kernel<T, P>), grid, block, 0, st, v, N, npoint, start, out_idx, out_xyz); \
    return launch_status("dvcp_fps");                                                             \
  }
  DVCP_FPS_CASE(1)
  DVCP_FPS_CASE(2)
  DVCP_FPS_CASE(4)
  DVCP_FPS_CASE(8)
  DVCP_FPS_CASE(12)
  DVCP_FPS_CASE(16)
#undef DVCP_FPS_CASE
  set_error("dvcp_fps: N=%d exceeds the register-resident limit of 16384 points per cloud", N);
  return DVCP_EINVAL;
}

}  // namespace dvcp

extern "C" int dvcp_fps(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                        int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz,
                        void* stream) {
  DVCP_REQUIRE(xyz && start && out_idx, "dvcp_fps: null pointer");
  DVCP_REQUIRE(B >= 0 && N > 0 && npoint >= 0, "dvcp_fps: bad sizes B=%d N=%d npoint=%d", B, N, npoint);
  if (B == 0 || npoint == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_fps<float>(static_cast<const float*>(xyz), sb, sc, sn, B, N, npoint, start,
                                   out_idx, static_cast<float*>(out_xyz), st);
  if (dtype == DVCP_F64)
    return dvcp::launch_fps<double>(static_cast<const double*>(xyz), sb, sc, sn, B, N, npoint, start,
                                    out_idx, static_cast<double*>(out_xyz), st);
  dvcp::set_error("dvcp_fps: bad dtype %d", dtype);
  return DVCP_EINVAL;
}
