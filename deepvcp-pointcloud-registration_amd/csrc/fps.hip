// fps.hip -- farthest point sampling (replaces pointnet2_utils.py:63-84).
//
// Semantics (bit-exact with the reference): running minimum stored in fp32 for both coordinate
// dtypes (:74, :82), distance ((dx*dx + dy*dy) + dz*dz) in the coordinate dtype (:80), strict
// '<' update (:81), argmax = largest running minimum, ties to the LOWEST original index (:83).
//
// FPS is a serial chain of `npoint` dependent argmax steps per cloud, so the kernel is built
// around the latency of one step.  One 1024-thread workgroup per cloud (16 waves):
//   * Setup: the cloud is counting-sorted in LDS by a 12-bit Morton cell (16^3 cells), and wave
//     w takes sorted positions [w*64*PPT, (w+1)*64*PPT): every wave owns a compact region and
//     keeps its points, running minima and original indices in VGPRs for the whole launch.
//   * Exact pruning: a wave skips a step when lb2(centre, wave box) >= its current max running
//     minimum.  lb2 is computed with the same ops as a point distance on box-face coordinates,
//     and round-to-nearest is monotone, so every point of the box then has d >= lb2 >= its
//     running minimum: the reference's strict '<' would not update any of them.  A skipped wave
//     re-publishes its cached best.  Late in the chain only waves near the new centre work.
//   * One barrier per step: wave argmax by DPP (row_shr / row_bcast) + ballot tie-break, each
//     wave publishes {value, index, x, y, z} to a double-buffered LDS slot, and every wave
//     reduces the 16 slots with a 16-lane DPP max.  No global memory in the loop except the
//     output stores.
#include <cstdlib>

#include "common.h"

namespace dvcp {

// ------------------------------------------------------------------------------- DPP helpers
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ float dpp_maxf(float v) {
  const int o = __builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWS, 0xF, false);
  return fmaxf(v, __int_as_float(o));
}
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ int dpp_mini(int v) {
  const int o = __builtin_amdgcn_update_dpp(v, v, CTRL, ROWS, 0xF, false);
  return min(v, o);
}
// row_shr:1,2,4,8 then row_bcast:15 (rows 1,3) and row_bcast:31 (rows 2,3): lane 63 holds the
// reduction of all 64 lanes.
__device__ __forceinline__ float wave_maxf_dpp(float v) {
  v = dpp_maxf<0x111>(v);
  v = dpp_maxf<0x112>(v);
  v = dpp_maxf<0x114>(v);
  v = dpp_maxf<0x118>(v);
  v = dpp_maxf<0x142, 0xA>(v);
  v = dpp_maxf<0x143, 0xC>(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ int wave_mini_dpp(int v) {
  v = dpp_mini<0x111>(v);
  v = dpp_mini<0x112>(v);
  v = dpp_mini<0x114>(v);
  v = dpp_mini<0x118>(v);
  v = dpp_mini<0x142, 0xA>(v);
  v = dpp_mini<0x143, 0xC>(v);
  return __builtin_amdgcn_readlane(v, 63);
}
template <typename T>
__device__ __forceinline__ T readlane_t(T v, int lane);
template <>
__device__ __forceinline__ float readlane_t<float>(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
template <>
__device__ __forceinline__ double readlane_t<double>(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b & 0xFFFFFFFFll), lane);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), lane);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Lower bound of the distance from c to an axis-aligned box, rounded like a point distance
// (branch-free: outside the slab exactly one difference is positive, inside both are <= 0).
template <typename T>
__device__ __forceinline__ T box_lb2(T cx, T cy, T cz, const T (&bx)[6]) {
  const T ex = fmax(fmax(bx[0] - cx, cx - bx[3]), static_cast<T>(0));
  const T ey = fmax(fmax(bx[1] - cy, cy - bx[4]), static_cast<T>(0));
  const T ez = fmax(fmax(bx[2] - cz, cz - bx[5]), static_cast<T>(0));
  return (ex * ex + ey * ey) + ez * ez;
}

template <typename T>
struct alignas(16) FpsSlot {
  float v;
  int i;
  T x, y, z;
};

constexpr int kFpsThreads = 1024;
constexpr int kFpsWaves = kFpsThreads / kWave;
constexpr int kMortonBins = 4096;

__device__ __forceinline__ uint32_t spread4(uint32_t v) {  // 4 bits -> every third bit
  v &= 0xF;
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4) | ((v & 8u) << 6);
}

template <typename T, int PPT, bool PRUNE = true>
__global__ __launch_bounds__(kFpsThreads) void fps_kernel(PointsView<T> pts, int N, int npoint,
                                                          const int64_t* __restrict__ start,
                                                          int64_t* __restrict__ out_idx, T* __restrict__ out_xyz) {
  __shared__ uint32_t bins[kMortonBins];
  __shared__ uint16_t perm[kFpsThreads * PPT];
  __shared__ FpsSlot<T> slots[2][kFpsWaves];
  __shared__ T red[2][6][kFpsWaves];
  __shared__ uint32_t wsum[kFpsWaves];

  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- setup 1: cloud bounding box (natural layout) ----------------------------------------
  T lo[3] = {static_cast<T>(__builtin_huge_val()), static_cast<T>(__builtin_huge_val()),
             static_cast<T>(__builtin_huge_val())};
  T hi[3] = {-lo[0], -lo[1], -lo[2]};
  for (int n = tid; n < N; n += kFpsThreads) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const T v = pts.at(b, a, n);
      lo[a] = v < lo[a] ? v : lo[a];
      hi[a] = v > hi[a] ? v : hi[a];
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    for (int off = 32; off > 0; off >>= 1) {
      const T ol = __shfl_xor(lo[a], off, kWave), oh = __shfl_xor(hi[a], off, kWave);
      lo[a] = ol < lo[a] ? ol : lo[a];
      hi[a] = oh > hi[a] ? oh : hi[a];
    }
    if (lane == 0) {
      red[0][a][wave] = lo[a];
      red[1][a][wave] = hi[a];
    }
  }
  for (int i = tid; i < kMortonBins; i += kFpsThreads) bins[i] = 0u;
  __syncthreads();
  T blo[3], bscale[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    T l = red[0][a][0], h = red[1][a][0];
    for (int w = 1; w < kFpsWaves; ++w) {
      l = red[0][a][w] < l ? red[0][a][w] : l;
      h = red[1][a][w] > h ? red[1][a][w] : h;
    }
    blo[a] = l;
    bscale[a] = h > l ? static_cast<T>(16) / (h - l) : static_cast<T>(0);
  }

  // ---- setup 2: counting sort by Morton cell (only the point->slot map depends on it) --------
  auto cell_of = [&](int n) -> uint32_t {
    uint32_t c = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      int q = static_cast<int>((pts.at(b, a, n) - blo[a]) * bscale[a]);
      q = q < 0 ? 0 : (q > 15 ? 15 : q);
      c |= spread4(static_cast<uint32_t>(q)) << a;
    }
    return c;
  };
  for (int n = tid; n < N; n += kFpsThreads) atomicAdd(&bins[cell_of(n)], 1u);
  __syncthreads();
  {  // exclusive scan of 4096 bins: 4 per thread, wave scan, then across waves
    uint32_t v[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = bins[tid * 4 + k];
      s += v[k];
    }
    uint32_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t u = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < wave; ++w) base += wsum[w];
    uint32_t run = base + incl - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bins[tid * 4 + k] = run;
      run += v[k];
    }
  }
  __syncthreads();
  for (int n = tid; n < N; n += kFpsThreads) perm[atomicAdd(&bins[cell_of(n)], 1u)] = static_cast<uint16_t>(n);
  __syncthreads();

  // ---- setup 3: this thread's points (wave-contiguous sorted ranges) and the wave's box ------
  T px[PPT], py[PPT], pz[PPT];
  float dmin[PPT];
  int pid[PPT];
  T wb[6];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    wb[a] = static_cast<T>(__builtin_huge_val());
    wb[3 + a] = -wb[a];
  }
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int pos = wave * (kWave * PPT) + p * kWave + lane;
    if (pos < N) {
      const int n = perm[pos];
      pid[p] = n;
      px[p] = pts.at(b, 0, n);
      py[p] = pts.at(b, 1, n);
      pz[p] = pts.at(b, 2, n);
      dmin[p] = 1e10f;  // torch.ones(B, N) * 1e10 (fp32), :74
      wb[0] = px[p] < wb[0] ? px[p] : wb[0];
      wb[1] = py[p] < wb[1] ? py[p] : wb[1];
      wb[2] = pz[p] < wb[2] ? pz[p] : wb[2];
      wb[3] = px[p] > wb[3] ? px[p] : wb[3];
      wb[4] = py[p] > wb[4] ? py[p] : wb[4];
      wb[5] = pz[p] > wb[5] ? pz[p] : wb[5];
    } else {
      pid[p] = 0x7FFFFFFF;
      px[p] = py[p] = pz[p] = static_cast<T>(0);
      dmin[p] = -1.0f;  // never updated (d >= 0) and never selected
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    for (int off = 32; off > 0; off >>= 1) {
      const T ol = __shfl_xor(wb[a], off, kWave), oh = __shfl_xor(wb[3 + a], off, kWave);
      wb[a] = ol < wb[a] ? ol : wb[a];
      wb[3 + a] = oh > wb[3 + a] ? oh : wb[3 + a];
    }
  }

  int64_t cur = start[b];
  if (cur < 0 || cur >= N) cur = 0;  // host validates; keep the kernel in bounds regardless
  T cx = pts.at(b, 0, cur), cy = pts.at(b, 1, cur), cz = pts.at(b, 2, cur);

  int64_t* oi = out_idx + static_cast<int64_t>(b) * npoint;
  T* ox = out_xyz ? out_xyz + static_cast<int64_t>(b) * 3 * npoint : nullptr;

  // the wave's cached best (wave-uniform): value, original index, coordinates
  float wv = __builtin_huge_valf();  // forces the first step to update
  int wi = 0x7FFFFFFF;
  T wx = 0, wy = 0, wz = 0;
  const bool empty_wave = wave * (kWave * PPT) >= N;

  for (int step = 0; step < npoint; ++step) {
    if (tid == 0) {
      oi[step] = cur;
      if (ox) {
        ox[step] = cx;
        ox[npoint + step] = cy;
        ox[2 * npoint + step] = cz;
      }
    }
    const bool active = !empty_wave && (!PRUNE || !(box_lb2(cx, cy, cz, wb) >= static_cast<T>(wv)));
    if (active) {
      float bv = -1.0f;
      int bi = 0x7FFFFFFF;
      T bx = 0, by = 0, bz = 0;
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        const T dx = px[p] - cx, dy = py[p] - cy, dz = pz[p] - cz;
        const T d = (dx * dx + dy * dy) + dz * dz;  // torch.sum((xyz - c) ** 2, -1), :80
        dmin[p] = d < static_cast<T>(dmin[p]) ? static_cast<float>(d) : dmin[p];
        // branch-free lexicographic (value desc, original index asc): bitwise, not short-circuit
        const bool better = (dmin[p] > bv) | ((dmin[p] == bv) & (pid[p] < bi));
        bv = better ? dmin[p] : bv;
        bi = better ? pid[p] : bi;
        bx = better ? px[p] : bx;
        by = better ? py[p] : by;
        bz = better ? pz[p] : bz;
      }
      wv = wave_maxf_dpp(bv);
      const uint64_t tied = __ballot(bv == wv);
      int wl;
      if ((tied & (tied - 1)) == 0) {
        wl = __ffsll(static_cast<long long>(tied)) - 1;
      } else {  // equal maxima in several lanes: lowest original index
        const int mi = wave_mini_dpp(bv == wv ? bi : 0x7FFFFFFF);
        wl = __ffsll(static_cast<long long>(__ballot(bv == wv && bi == mi))) - 1;
      }
      wi = __builtin_amdgcn_readlane(bi, wl);
      wx = readlane_t(bx, wl);
      wy = readlane_t(by, wl);
      wz = readlane_t(bz, wl);
    }
    FpsSlot<T>* buf = slots[step & 1];
    if (lane == 0) buf[wave] = FpsSlot<T>{empty_wave ? -2.0f : wv, empty_wave ? 0x7FFFFFFF : wi, wx, wy, wz};
    lds_barrier();  // the output stores above stay in flight across the barrier
    // block argmax over the 16 slots in lanes 0..15 (row 0): value desc, then index asc
    const FpsSlot<T> mine = buf[lane & (kFpsWaves - 1)];
    float v = mine.v;
    v = dpp_maxf<0x111, 0x1>(v);
    v = dpp_maxf<0x112, 0x1>(v);
    v = dpp_maxf<0x114, 0x1>(v);
    v = dpp_maxf<0x118, 0x1>(v);
    const float gv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 15));
    const uint64_t tied = __ballot(lane < kFpsWaves && mine.v == gv);
    int ws;
    if ((tied & (tied - 1)) == 0) {
      ws = __ffsll(static_cast<long long>(tied)) - 1;
    } else {
      int ii = (lane < kFpsWaves && mine.v == gv) ? mine.i : 0x7FFFFFFF;
      ii = dpp_mini<0x111, 0x1>(ii);
      ii = dpp_mini<0x112, 0x1>(ii);
      ii = dpp_mini<0x114, 0x1>(ii);
      ii = dpp_mini<0x118, 0x1>(ii);
      const int mi = __builtin_amdgcn_readlane(ii, 15);
      ws = __ffsll(static_cast<long long>(__ballot(lane < kFpsWaves && mine.v == gv && mine.i == mi))) - 1;
    }
    cur = buf[ws].i;
    cx = buf[ws].x;
    cy = buf[ws].y;
    cz = buf[ws].z;
  }
}

// Dense fallback (no sort, no pruning) for clouds larger than the sorted kernel's VGPR budget.
template <typename T>
__global__ __launch_bounds__(kFpsThreads) void fps_dense_kernel(PointsView<T> pts, int N, int npoint,
                                                                const int64_t* __restrict__ start,
                                                                int64_t* __restrict__ out_idx, T* __restrict__ out_xyz,
                                                                float* __restrict__ ws) {
  __shared__ FpsSlot<T> slots[2][kFpsWaves];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* dmin = ws + static_cast<int64_t>(b) * N;
  for (int n = tid; n < N; n += kFpsThreads) dmin[n] = 1e10f;
  int64_t cur = start[b];
  if (cur < 0 || cur >= N) cur = 0;
  T cx = pts.at(b, 0, cur), cy = pts.at(b, 1, cur), cz = pts.at(b, 2, cur);
  for (int step = 0; step < npoint; ++step) {
    if (tid == 0) {
      out_idx[static_cast<int64_t>(b) * npoint + step] = cur;
      if (out_xyz) {
        T* ox = out_xyz + static_cast<int64_t>(b) * 3 * npoint;
        ox[step] = cx;
        ox[npoint + step] = cy;
        ox[2 * npoint + step] = cz;
      }
    }
    float bv = -1.0f;
    int bi = 0x7FFFFFFF;
    for (int n = tid; n < N; n += kFpsThreads) {  // ascending n per thread: strict '>' keeps the lower index
      const T dx = pts.at(b, 0, n) - cx, dy = pts.at(b, 1, n) - cy, dz = pts.at(b, 2, n) - cz;
      const T d = (dx * dx + dy * dy) + dz * dz;
      float m = dmin[n];
      if (d < static_cast<T>(m)) {
        m = static_cast<float>(d);
        dmin[n] = m;
      }
      if (m > bv) {
        bv = m;
        bi = n;
      }
    }
    const float wvv = wave_maxf_dpp(bv);
    const int mi = wave_mini_dpp(bv == wvv ? bi : 0x7FFFFFFF);
    if (lane == 0) {
      slots[step & 1][wave].v = wvv;
      slots[step & 1][wave].i = mi;
    }
    __syncthreads();
    float gv = -2.0f;
    int gi = 0x7FFFFFFF;
    for (int w = 0; w < kFpsWaves; ++w) {
      const float v = slots[step & 1][w].v;
      const int i = slots[step & 1][w].i;
      if (v > gv || (v == gv && i < gi)) {
        gv = v;
        gi = i;
      }
    }
    cur = gi;
    cx = pts.at(b, 0, cur);
    cy = pts.at(b, 1, cur);
    cz = pts.at(b, 2, cur);
  }
}

template <typename T>
static int launch_fps(const T* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                      const int64_t* start, int64_t* out_idx, T* out_xyz, float* ws, hipStream_t st) {
  PointsView<T> v{xyz, sb, sc, sn};
  const int ppt = ceil_div(N, kFpsThreads);
  dim3 grid(B), block(kFpsThreads);
  // diagnostics only: DVCP_FPS_NOPRUNE=1 disables the exact box pruning (identical results)
  static const bool noprune = [] {
    const char* e = getenv("DVCP_FPS_NOPRUNE");
    return e && e[0] == '1';
  }();
#define DVCP_FPS_CASE(P)                                                                                      \
  if (ppt <= P) {                                                                                             \
    if (noprune)                                                                                              \
      hipLaunchKernelGGL((fps_kernel<T, P, false>), grid, block, 0, st, v, N, npoint, start, out_idx, out_xyz); \
    else                                                                                                      \
      hipLaunchKernelGGL((fps_kernel<T, P, true>), grid, block, 0, st, v, N, npoint, start, out_idx, out_xyz);  \
    return launch_status("dvcp_fps");                                                                         \
  }
  DVCP_FPS_CASE(1)
  DVCP_FPS_CASE(2)
  DVCP_FPS_CASE(4)
  DVCP_FPS_CASE(8)
  if (sizeof(T) == 4 || N <= 12 * kFpsThreads) {
    DVCP_FPS_CASE(12)
  }
  if (sizeof(T) == 4) {
    DVCP_FPS_CASE(16)
  }
#undef DVCP_FPS_CASE
  if (!ws) {
    set_error("dvcp_fps: N=%d needs the dense path and its B x N fp32 workspace (dvcp_fps_ws)", N);
    return DVCP_EINVAL;
  }
  hipLaunchKernelGGL((fps_dense_kernel<T>), grid, block, 0, st, v, N, npoint, start, out_idx, out_xyz, ws);
  return launch_status("dvcp_fps(dense)");
}

}  // namespace dvcp

extern "C" int dvcp_fps_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                           const int64_t* start, int64_t* out_idx, void* out_xyz, float* ws, void* stream) {
  DVCP_REQUIRE(xyz && start && out_idx, "dvcp_fps: null pointer");
  DVCP_REQUIRE(B >= 0 && N > 0 && npoint >= 0, "dvcp_fps: bad sizes B=%d N=%d npoint=%d", B, N, npoint);
  DVCP_REQUIRE(N <= 65535 || ws, "dvcp_fps: N=%d needs a workspace", N);
  if (B == 0 || npoint == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_fps<float>(static_cast<const float*>(xyz), sb, sc, sn, B, N, npoint, start, out_idx,
                                   static_cast<float*>(out_xyz), ws, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_fps<double>(static_cast<const double*>(xyz), sb, sc, sn, B, N, npoint, start, out_idx,
                                    static_cast<double*>(out_xyz), ws, st);
  dvcp::set_error("dvcp_fps: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

extern "C" int dvcp_fps(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                        const int64_t* start, int64_t* out_idx, void* out_xyz, void* stream) {
  return dvcp_fps_ws(dtype, xyz, sb, sc, sn, B, N, npoint, start, out_idx, out_xyz, nullptr, stream);
}
