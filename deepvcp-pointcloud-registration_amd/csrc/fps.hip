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

template <typename T>
__device__ __forceinline__ T readfirstlane_t(T v) {
  return readlane_t(v, 0);
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

constexpr int kFpsThreads = 512;  // 8 waves: 2 per SIMD, up to 256 VGPRs each
constexpr int kMortonBins = 4096;
constexpr int kFpsProf = 8;       // timing probe words per wave (fps_kernel<..., TIMING=true>)

__device__ __forceinline__ uint32_t spread4(uint32_t v) {  // 4 bits -> every third bit
  v &= 0xF;
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4) | ((v & 8u) << 6);
}

__device__ __forceinline__ uint64_t fps_clock() {
  const uint64_t t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

// THREADS threads (W = THREADS/64 waves) per cloud; PPT points per lane in VGPRs.
// TIMING (diagnostics, tools/fps_lab): per-wave sums of the step phases in shader clocks.
template <typename T, int THREADS, int PPT, bool PRUNE, bool TIMING = false>
__global__ __launch_bounds__(THREADS) void fps_kernel(PointsView<T> pts, int N, int npoint,
                                                      const int64_t* __restrict__ start,
                                                      int64_t* __restrict__ out_idx, T* __restrict__ out_xyz,
                                                      unsigned long long* __restrict__ prof) {
  constexpr int W = THREADS / kWave;
  constexpr int RANGE = kWave * PPT;  // sorted positions per wave
  static_assert(W <= 16 && (W & (W - 1)) == 0, "slot reduction covers one DPP row");
  static_assert(PPT % 2 == 0 || PPT == 1, "original indices are packed two per VGPR");
  __shared__ uint32_t bins[kMortonBins];
  __shared__ uint16_t perm[THREADS * PPT];
  __shared__ uint8_t owner[THREADS * PPT];
  __shared__ FpsSlot<T> slots[2][W];
  __shared__ T red[2][3][W];
  __shared__ uint32_t wsum[W];

  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- setup 1: cloud bounding box ------------------------------------------------------------
  T lo[3] = {static_cast<T>(__builtin_huge_val()), static_cast<T>(__builtin_huge_val()),
             static_cast<T>(__builtin_huge_val())};
  T hi[3] = {-lo[0], -lo[1], -lo[2]};
  for (int n = tid; n < N; n += THREADS) {
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
  for (int i = tid; i < kMortonBins; i += THREADS) bins[i] = 0u;
  __syncthreads();
  T blo[3], bscale[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    T l = red[0][a][0], h = red[1][a][0];
    for (int w = 1; w < W; ++w) {
      l = red[0][a][w] < l ? red[0][a][w] : l;
      h = red[1][a][w] > h ? red[1][a][w] : h;
    }
    blo[a] = l;
    bscale[a] = h > l ? static_cast<T>(16) / (h - l) : static_cast<T>(0);
  }

  // ---- setup 2: counting sort by Morton cell -> each wave owns a compact region ---------------
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
  for (int n = tid; n < N; n += THREADS) atomicAdd(&bins[cell_of(n)], 1u);
  __syncthreads();
  {  // exclusive scan of the bins: PER per thread, wave scan, then across waves
    constexpr int PER = kMortonBins / THREADS;
    uint32_t v[PER], s = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      v[k] = bins[tid * PER + k];
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
    for (int k = 0; k < PER; ++k) {
      bins[tid * PER + k] = run;
      run += v[k];
    }
  }
  __syncthreads();
  for (int n = tid; n < N; n += THREADS) perm[atomicAdd(&bins[cell_of(n)], 1u)] = static_cast<uint16_t>(n);
  __syncthreads();
  for (int pos = tid; pos < N; pos += THREADS) owner[perm[pos]] = static_cast<uint8_t>(pos / RANGE);
  __syncthreads();
  // ---- setup 3: each wave lists its points in ascending original index (stream compaction) ---
  // Slot p of a lane then holds the wave's (p*64 + lane)-th smallest index, so a lane meets its
  // points in index order and a strict '>' keeps the lowest index among equal maxima (:83).
  {
    int k = 0;
    for (int base = 0; base < N; base += kWave) {
      const int n = base + lane;
      const bool mine = (n < N) && owner[n] == wave;
      const uint64_t m = __ballot(mine);
      if (mine) perm[wave * RANGE + k + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0))] =
          static_cast<uint16_t>(n);
      k += __popcll(m);
    }
  }
  __syncthreads();

  // ---- setup 4: this lane's points, running minima, packed indices; the wave's box -----------
  const int count = min(RANGE, max(0, N - wave * RANGE));
  T px[PPT], py[PPT], pz[PPT];
  float dmin[PPT];
  uint32_t pidp[(PPT + 1) / 2];
  T wb[6];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    wb[a] = static_cast<T>(__builtin_huge_val());
    wb[3 + a] = -wb[a];
  }
#pragma unroll
  for (int p = 0; p < (PPT + 1) / 2; ++p) pidp[p] = 0u;
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int k = p * kWave + lane;
    if (k < count) {
      const uint32_t n = perm[wave * RANGE + k];
      pidp[p >> 1] |= n << ((p & 1) * 16);
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
    wb[a] = readfirstlane_t(wb[a]);
    wb[3 + a] = readfirstlane_t(wb[3 + a]);
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
  const bool empty_wave = count == 0;
  uint64_t ph[4] = {0, 0, 0, 0}, nact = 0;

  for (int step = 0; step < npoint; ++step) {
    uint64_t t0 = 0, t1 = 0, t2 = 0;
    if constexpr (TIMING) t0 = fps_clock();
    if (tid == 0) {
      oi[step] = cur;
      if (ox) {
        ox[step] = cx;
        ox[npoint + step] = cy;
        ox[2 * npoint + step] = cz;
      }
    }
    const bool active = !empty_wave & (!PRUNE || !(box_lb2(cx, cy, cz, wb) >= static_cast<T>(wv)));
    if (active) {
      float bv = -1.0f;
      int bp = 0;
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        const T dx = px[p] - cx, dy = py[p] - cy, dz = pz[p] - cz;
        const T d = (dx * dx + dy * dy) + dz * dz;  // torch.sum((xyz - c) ** 2, -1), :80
        if constexpr (sizeof(T) == 4) {
          dmin[p] = fminf(d, dmin[p]);  // == (d < dmin ? d : dmin) for finite values, :81-82
        } else {
          dmin[p] = d < static_cast<T>(dmin[p]) ? static_cast<float>(d) : dmin[p];
        }
        const bool c = dmin[p] > bv;  // strict: the first (lowest-index) of equal maxima stays
        bp = c ? p : bp;
        bv = c ? dmin[p] : bv;
      }
      if constexpr (TIMING) t1 = fps_clock();
      wv = wave_maxf_dpp(bv);
      const uint64_t tied = __ballot(bv == wv);
      int wl;
      if ((tied & (tied - 1)) == 0) {
        wl = __ffsll(static_cast<long long>(tied)) - 1;
      } else {  // equal maxima in several lanes: the lowest original index among them
        uint32_t mine = 0x7FFFFFFFu;
#pragma unroll
        for (int p = 0; p < PPT; ++p) mine = bp == p ? ((pidp[p >> 1] >> ((p & 1) * 16)) & 0xFFFFu) : mine;
        const int mi = wave_mini_dpp(bv == wv ? static_cast<int>(mine) : 0x7FFFFFFF);
        wl = __ffsll(static_cast<long long>(__ballot((bv == wv) & (static_cast<int>(mine) == mi)))) - 1;
      }
      // the winning lane's slot index is wave-uniform: indexed register reads (s_set_gpr_idx)
      const int wp = __builtin_amdgcn_readlane(bp, wl);
      wi = static_cast<int>((static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pidp[wp >> 1]), wl)) >>
                             ((wp & 1) * 16)) & 0xFFFFu);
      wx = readlane_t(px[wp], wl);
      wy = readlane_t(py[wp], wl);
      wz = readlane_t(pz[wp], wl);
      if constexpr (TIMING) ++nact;
    } else if constexpr (TIMING) {
      t1 = fps_clock();
    }
    FpsSlot<T>* buf = slots[step & 1];
    if (lane == 0) buf[wave] = FpsSlot<T>{empty_wave ? -2.0f : wv, empty_wave ? 0x7FFFFFFF : wi, wx, wy, wz};
    if constexpr (TIMING) t2 = fps_clock();
    lds_barrier();  // the output stores above stay in flight across the barrier
    uint64_t t3 = 0;
    if constexpr (TIMING) t3 = fps_clock();
    // block argmax over the W slots in lanes 0..W-1 (row 0): value desc, then index asc
    const FpsSlot<T> mine = buf[lane & (W - 1)];
    float v = mine.v;
    if constexpr (W > 1) v = dpp_maxf<0x111, 0x1>(v);
    if constexpr (W > 2) v = dpp_maxf<0x112, 0x1>(v);
    if constexpr (W > 4) v = dpp_maxf<0x114, 0x1>(v);
    if constexpr (W > 8) v = dpp_maxf<0x118, 0x1>(v);
    const float gv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), W - 1));
    const uint64_t tied = __ballot((lane < W) & (mine.v == gv));
    int ws;
    if ((tied & (tied - 1)) == 0) {
      ws = __ffsll(static_cast<long long>(tied)) - 1;
    } else {
      int ii = ((lane < W) & (mine.v == gv)) ? mine.i : 0x7FFFFFFF;
      if constexpr (W > 1) ii = dpp_mini<0x111, 0x1>(ii);
      if constexpr (W > 2) ii = dpp_mini<0x112, 0x1>(ii);
      if constexpr (W > 4) ii = dpp_mini<0x114, 0x1>(ii);
      if constexpr (W > 8) ii = dpp_mini<0x118, 0x1>(ii);
      const int mi = __builtin_amdgcn_readlane(ii, W - 1);
      ws = __ffsll(static_cast<long long>(__ballot((lane < W) & (mine.v == gv) & (mine.i == mi)))) - 1;
    }
    cur = __builtin_amdgcn_readlane(mine.i, ws);
    cx = readlane_t(mine.x, ws);
    cy = readlane_t(mine.y, ws);
    cz = readlane_t(mine.z, ws);
    if constexpr (TIMING) {
      const uint64_t t4 = fps_clock();
      ph[0] += t1 - t0;  // box test + point update
      ph[1] += t2 - t1;  // wave argmax + slot publish
      ph[2] += t3 - t2;  // barrier wait
      ph[3] += t4 - t3;  // slot reduction
    }
  }
  if constexpr (TIMING) {
    if (prof && lane == 0) {
      unsigned long long* o = prof + (static_cast<int64_t>(b) * W + wave) * kFpsProf;
      o[0] = ph[0];
      o[1] = ph[1];
      o[2] = ph[2];
      o[3] = ph[3];
      o[4] = nact;
      o[5] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_ID: wave slot, SIMD, CU
      o[6] = static_cast<unsigned long long>(count);
      o[7] = 0;
    }
  }
}

// Dense fallback (no sort, no pruning) for clouds larger than the sorted kernel's VGPR budget.
template <typename T>
__global__ __launch_bounds__(kFpsThreads) void fps_dense_kernel(PointsView<T> pts, int N, int npoint,
                                                                const int64_t* __restrict__ start,
                                                                int64_t* __restrict__ out_idx, T* __restrict__ out_xyz,
                                                                float* __restrict__ ws) {
  constexpr int kDenseWaves = kFpsThreads / kWave;
  __shared__ FpsSlot<T> slots[2][kDenseWaves];
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
    for (int w = 0; w < kDenseWaves; ++w) {
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
#define DVCP_FPS_CASE(P)                                                                             \
  if (ppt <= P) {                                                                                    \
    if (noprune)                                                                                     \
      hipLaunchKernelGGL((fps_kernel<T, kFpsThreads, P, false>), grid, block, 0, st, v, N, npoint, start, \
                         out_idx, out_xyz, nullptr);                                                 \
    else                                                                                             \
      hipLaunchKernelGGL((fps_kernel<T, kFpsThreads, P, true>), grid, block, 0, st, v, N, npoint, start,  \
                         out_idx, out_xyz, nullptr);                                                 \
    return launch_status("dvcp_fps");                                                                \
  }
  DVCP_FPS_CASE(2)
  DVCP_FPS_CASE(4)
  DVCP_FPS_CASE(8)
  DVCP_FPS_CASE(16)
  if constexpr (sizeof(T) == 4) {
    DVCP_FPS_CASE(24)
    DVCP_FPS_CASE(32)
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
