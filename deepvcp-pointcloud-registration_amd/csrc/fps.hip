// fps.hip -- farthest point sampling (replaces pointnet2_utils.py:63-84).
//
// Semantics (bit-exact with the reference): running minimum stored in fp32 for both coordinate
// dtypes (:74, :82), distance ((dx*dx + dy*dy) + dz*dz) in the coordinate dtype (:80), strict
// '<' update (:81), argmax = largest running minimum, ties to the LOWEST original index (:83).
//
// FPS is a serial chain of `npoint` dependent argmax steps per cloud.  Kernels by cloud size:
//   * N < 2048: fps_kernel, one centre per step (one workgroup, per-step DPP argmax + one barrier,
//     wave-box pruning);
//   * 2048 <= N <= 16384 (8192 fp64): fps_select_kernel, which certifies a whole prefix of the
//     serial chain per round (~27 centres on C3 clouds) from a threshold-selected candidate list;
//   * larger, fp32 up to 65536: the split select (fps_part_kernel: 8 workgroups per cloud run
//     the select rounds together, one candidate-list exchange per round; opt-in below 16384);
//     else fps_split_kernel (S workgroups per cloud exchanging one key per step), then
//     fps_dense_kernel.
// Every kernel keeps each cloud's coordinates and running minima in VGPRs (Morton-sorted for the
// first two), so the loop touches no global memory except the output stores.
#include <type_traits>

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
constexpr int kFpsSel1024 = 1024;  // the fp32 select kernel's workgroup: 16 waves, 4 per SIMD
constexpr int kMortonBins = 4096;
constexpr int kFpsProf = 13;      // timing probe words per wave (fps_kernel<..., TIMING=true>)

__device__ __forceinline__ uint32_t spread4(uint32_t v) {  // 4 bits -> every third bit
  v &= 0xF;
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4) | ((v & 8u) << 6);
}

__device__ __forceinline__ uint64_t fps_clock() {
  const uint64_t t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

// Setup shared by the FPS kernels: counting sort of the cloud by 12-bit Morton cell (16^3 cells
// over its bounding box): put(pos, n) for each point n and its sorted position pos.  Only the
// point -> wave/group assignment depends on it, never a result.
template <typename T, int THREADS, typename Put>
__device__ void fps_morton_sort(const PointsView<T>& pts, int b, int N, uint32_t* bins, Put put,
                                T (*red)[3][THREADS / kWave], uint32_t* wsum) {
  constexpr int W = THREADS / kWave;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
  for (int n = tid; n < N; n += THREADS) put(atomicAdd(&bins[cell_of(n)], 1u), n);
  __syncthreads();
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
  fps_morton_sort<T, THREADS>(pts, b, N, bins, [&](uint32_t pos, int n) { perm[pos] = static_cast<uint16_t>(n); },
                              red, wsum);
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

// ---------------------------------------------------------------------------------------------
// Helpers of the threshold-select kernel below.
// Below this cloud size the one-centre-per-step kernel is faster (few groups, short steps; and
// npoint > N tails, where every running minimum is 0, give rounds of one) -- tools/fps_lab.
constexpr int kFpsBatchedMinN = 2048;

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_umax(uint32_t v) {
  return max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROWS, 0xF, false)));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_umin(uint32_t v) {
  return min(v, static_cast<uint32_t>(
                    __builtin_amdgcn_update_dpp(static_cast<int>(0xFFFFFFFFu), static_cast<int>(v), CTRL, ROWS, 0xF, false)));
}
__device__ __forceinline__ uint32_t wave_umax(uint32_t v) {
  v = dpp_umax<0x111, 0xF>(v);
  v = dpp_umax<0x112, 0xF>(v);
  v = dpp_umax<0x114, 0xF>(v);
  v = dpp_umax<0x118, 0xF>(v);
  v = dpp_umax<0x142, 0xA>(v);
  v = dpp_umax<0x143, 0xC>(v);
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}
// Two independent wave maxima; the DPP chains interleave, so they cost about one chain's latency.
__device__ __forceinline__ void wave_umax2(uint32_t a, uint32_t b, uint32_t& ma, uint32_t& mb) {
  a = dpp_umax<0x111, 0xF>(a);
  b = dpp_umax<0x111, 0xF>(b);
  a = dpp_umax<0x112, 0xF>(a);
  b = dpp_umax<0x112, 0xF>(b);
  a = dpp_umax<0x114, 0xF>(a);
  b = dpp_umax<0x114, 0xF>(b);
  a = dpp_umax<0x118, 0xF>(a);
  b = dpp_umax<0x118, 0xF>(b);
  a = dpp_umax<0x142, 0xA>(a);
  b = dpp_umax<0x142, 0xA>(b);
  a = dpp_umax<0x143, 0xC>(a);
  b = dpp_umax<0x143, 0xC>(b);
  ma = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(a), 63));
  mb = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(b), 63));
}
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
  v = dpp_umin<0x111, 0xF>(v);
  v = dpp_umin<0x112, 0xF>(v);
  v = dpp_umin<0x114, 0xF>(v);
  v = dpp_umin<0x118, 0xF>(v);
  v = dpp_umin<0x142, 0xA>(v);
  v = dpp_umin<0x143, 0xC>(v);
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_uadd(uint32_t v) {
  return v + static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROWS, 0xF, false));
}
// Inclusive prefix sum over the wave on DPP (row_shr 1, 2, 4, 8 inside each 16-lane row, then
// row_bcast 15 / 31 across rows): no ds_bpermute round trips in the per-round critical path.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v = dpp_uadd<0x111, 0xF>(v);
  v = dpp_uadd<0x112, 0xF>(v);
  v = dpp_uadd<0x114, 0xF>(v);
  v = dpp_uadd<0x118, 0xF>(v);
  v = dpp_uadd<0x142, 0xA>(v);
  v = dpp_uadd<0x143, 0xC>(v);
  return v;
}
__device__ __forceinline__ float float_unorder_fps(uint32_t u) {  // inverse of float_order
  const uint32_t flip = (u >> 31) ? 0x80000000u : 0xFFFFFFFFu;
  return __uint_as_float(u ^ flip);
}

// Rounding-safe upper bound of the computed d2(p, c) over p in [lo, hi]: per axis the larger of
// |fl(lo - c)| and |fl(hi - c)| (round-to-nearest is monotone), then the d2 formula.
template <typename T>
__device__ __forceinline__ T box_ub2(T cx, T cy, T cz, const T (&bx)[6]) {
  const T ex = fmax(fabs(bx[0] - cx), fabs(bx[3] - cx));
  const T ey = fmax(fabs(bx[1] - cy), fabs(bx[4] - cy));
  const T ez = fmax(fabs(bx[2] - cz), fabs(bx[5] - cz));
  return (ex * ex + ey * ey) + ez * ez;
}

// (Round 5, measured and not kept: the update's x / y differences and squares as packed fp32 pairs,
// v_pk_add_f32 / v_pk_mul_f32, 13 instead of 15 VALU per pair -- 2.99 -> 3.02 ms at 10000,
// profiles/round5/r5bh_fps_pk.log.)
// DVCP_FPS_IMIN: the running-minimum update as an integer min of the bit patterns (see fps_update).
// Non-finite coordinates are outside the parity contract: a NaN point keeps 1e10 in the reference
// (NaN < m is false), which then picks it at every later step (its own distance never drops); the
// select kernels certify prefixes on d(c, c) = 0 and diverge there, as does the integer min on a
// NaN with the sign bit set (it is stored; the reference keeps m).  Callers pass finite clouds.
#ifndef DVCP_FPS_IMIN
#define DVCP_FPS_IMIN 1
#endif

// The reference's running-minimum update (:80-82): d in the coordinate dtype, strict '<', stored fp32.
template <typename T>
__device__ __forceinline__ float fps_update(float m, T px, T py, T pz, T cx, T cy, T cz) {
  const T dx = px - cx, dy = py - cy, dz = pz - cz;
  const T d = (dx * dx + dy * dy) + dz * dz;
  if constexpr (sizeof(T) == 4) {
#if DVCP_FPS_IMIN
    // = (d < m ? d : m) as one signed-integer min of the bit patterns: d >= +0 (a sum of squares;
    // a NaN d has a larger pattern than any m and keeps m) and m is 1e10, a kept d, or -1 on a
    // padding lane -- all ordered like their patterns.  (fminf adds a canonicalizing v_max.)
    return __int_as_float(min(__float_as_int(d), __float_as_int(m)));
#else
    return d < m ? d : m;
#endif
  } else {
    return d < static_cast<T>(m) ? static_cast<float>(d) : m;
  }
}

// ---------------------------------------------------------------------------------------------
// Threshold-select FPS (the default for 2048 <= N <= 16384 fp32 / 8192 fp64 points per cloud).
//
// Same point layout as the batched kernel (Morton-sorted 64-point groups, coordinates and running
// minima in VGPRs), except that the groups are dealt to the waves round robin -- slot p of wave w
// holds sorted positions (p*W + w)*64 + lane -- so every wave owns groups all over the cloud and
// the update of a round's accepted centres (which land in the cloud's largest holes, wherever
// they are) is spread evenly instead of falling on the few waves whose region holds them.  A
// round is decided without a serial walk:
//   1. scan: every point above a floor f is appended to an LDS list (value, position, xyz) and
//      counted in a 256-bin histogram of its float bits over (f, vmax]; T_f = the largest
//      running minimum at or below f (the floor adapts: raised from the histogram when more than
//      kSelCap points lie above it, lowered when fewer than kSelMin do);
//   2. the histogram gives a bin edge with about kSelTarget points above it: those are the
//      listed candidates (at most kSelMax), every other point's running minimum is <= T, the
//      largest unlisted value (exact: T_f and the list entries below the edge);
//   3. candidates are ranked by (value desc, original index asc) -- the reference's argmax
//      order (:83) -- and the longest prefix c_0..c_{k-1} is accepted such that for every j >= 1
//      v_j > T and no c_i (i < j) lowers c_j's running minimum (every d(c_i, c_j) >= v_j, the
//      same float formula as the point update).  Then c_j keeps v_j while c_0..c_{j-1} are
//      applied, every other listed value can only have dropped (to at most v_j, ties ordered
//      by index) and every unlisted one stays <= T < v_j, so c_j is exactly the serial FPS's
//      j-th next centre;
//   4. all waves apply the k accepted centres to their points (wave- and group-box pruning
//      against each group's exact maximum, re-reduced for the groups whose minima dropped).
// Ties beyond kSelMax points at one value (dyadic grids, npoint > N tails) fall back to one exact
// block argmax per round.  On uniform C3 clouds a round accepts ~27 centres (~370 rounds for
// 10000; tools/fps_lab), against ~9 for the batched walker.
// DVCP_FPS_ACC4 (default): the round's accepted centres as one LDS row (x, y, z, 0) each; a touched
// (centre, slot) pair of the update reads its centre as one broadcast LDS load instead of three
// v_readlane from the batch's lanes, moving that work off the VALU, which the update is issue-bound
// on (four waves per SIMD hide the load).  Round 5, tools/fps_lab A/B on one box
// (profiles/round5/r5bc_fps_acc4.log): 16384 -> 10000 5.20 -> 4.81 ms, 10000 -> 10000 (1024 x 10)
// 3.25 -> 3.09 ms, 16 clouds, identical indices.
// DVCP_FPS_RECERT: a round whose first pass stops early ranks the candidates left a second time
// (step 5b); 0 = one pass per round
// DVCP_FPS_PRIO: the select kernel's waves raise their issue priority (s_setprio) by this much
#ifndef DVCP_FPS_PRIO
#define DVCP_FPS_PRIO 0
#endif
#ifndef DVCP_FPS_RECERT
#define DVCP_FPS_RECERT 1
#endif
#ifndef DVCP_FPS_ACC4
#define DVCP_FPS_ACC4 1
#endif
constexpr int kSelCap = 1024;    // list capacity
constexpr int kSelBins = 256;
#ifndef DVCP_FPS_SEL_TARGET
#define DVCP_FPS_SEL_TARGET 64
#endif
constexpr int kSelTarget = DVCP_FPS_SEL_TARGET;
constexpr int kSelMax = 128;
constexpr int kSelMin = 16;
constexpr int kSelMaxScans = 8;  // rescans per round before the fallback (a guard)
constexpr int kSelAccept = 64;   // centres accepted per round at most

// this lane's index, computed where it is used (an opaque v_mbcnt pair the compiler cannot hoist)
__device__ __forceinline__ int fresh_lane() {
  int r;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
  return r;
}
__device__ __forceinline__ int sel_shift(uint32_t range) {  // smallest s with (range >> s) < kSelBins
  return range < kSelBins ? 0 : (32 - __clz(range)) - 8;
}
__device__ __forceinline__ float prev_float(float v) {  // largest float below v (v > 0)
  return __uint_as_float(__float_as_uint(v) - 1u);
}
// wave-wide max of max(v, +0) for v not NaN: the clamp and the max on the bit patterns, which order
// non-negative floats like their values (no order transform, no canonicalizing v_max)
__device__ __forceinline__ float wave_fmax_clamp0(float v) {
  return __uint_as_float(wave_umax(static_cast<uint32_t>(max(__float_as_int(v), 0))));
}

// Up to 10 points per lane at 1024 threads (sa2 / sa3 of C3: 10000 points) the kernel fits in 96
// VGPRs (5 waves per SIMD worth), so a fifth wave of up to 128 VGPRs -- a set-abstraction MFMA
// table, a ball query -- can share the FPS workgroup's CU: the chain's four waves per SIMD spend
// ~97 % of their time waiting on barriers and LDS (VALUBusy ~3 %, profiles/pmc_summary.json).
template <int PPT, int THREADS>
constexpr int fps_select_waves_per_eu() { return PPT <= 10 && THREADS == 1024 ? 5 : 1; }

// Paired FPS of two full-permutation layers (FE layers 2 and 3 of C3: 10000 -> 10000 -> 10000).
// Layer 3's FPS runs over layer 2's centres, which are layer 2's points in FPS order: the same
// point set.  FPS over a set is a function of the set and the start point except where an argmax
// ties (ties go to the lowest index, which depends on the order), so layer 3 can run on layer 2's
// points in their own order, from the start point layer 2 picks at step start3, beside layer 2:
//   * fps_pair_kernel, 2B workgroups: the first B tickets run layer 2 (cloud t) and publish the
//     index of their pick number start3[t] in slot[t]; the next B run layer 3 over the same cloud
//     in the same order, waiting only for that slot.  A workgroup's role comes from a ticket taken
//     when it starts, so a waiting workgroup's producer is always already running.  Layer 2 also
//     publishes each point's pick number (inv2), by which layer 3 resolves the ties of its argmax
//     (see the round's tie notes).  flag[t] is raised where neither applies (the one-argmax
//     fallback of either layer, or a wait that gave up); layer 3's indices are into layer 2's points;
//   * fps_pair_remap_kernel maps them into layer 2's FPS order (idx3 = layer 2's pick number of
//     each point) for the clouds without a flag, and orders tie groups (see the round's tie notes);
//   * the gated select kernel recomputes layer 3 in the reference's order for the flagged clouds.
// The results are those of the two serial launches, bit for bit (tests/test_gpu_kernels.py).
template <typename T>
struct FpsPairArgs {
  uint32_t* ticket;       // 0 before the launch
  uint32_t* slot;         // B, 0 before the launch; bit 31 | the point layer 2 picks at step start3
  int32_t* flag;          // B, 0 before the launch: the cloud needs the gated recomputation
  uint32_t* inv2;         // B x N, 0 before the launch; bit 31 | layer 2's pick number of each point
  const int64_t* start3;  // B
  int64_t* out3_idx;      // B x npoint (indices into layer 2's points until the remap)
  T* out3_xyz;            // B x 3 x npoint
};
constexpr uint32_t kFpsPairSpinCap = 1u << 22;

// Split select (MODE 3, round 6): S workgroups per cloud run the select rounds together.  Every
// workgroup takes the 64-point groups g of the cloud's Morton order with g % S == part (then dealt
// round robin over its waves, as above) and, per round:
//   1. scans, decides and lists its OWN points exactly as the one-workgroup kernel does, with a
//      per-workgroup candidate cap of 128 / S: its candidates and T_w, the largest of its running
//      minima it did not list;
//   2. publishes them as 8-byte {data, round} granules (agent-scope, L2-served stores; each
//      granule carries its own tag, so no fence or flag orders them) into its slot of the round's
//      parity, and polls the other workgroups' granules until every one carries the round;
//   3. every workgroup now holds the same merged list (128 slots, part q's at [q cap, (q+1) cap),
//      unused slots v = -1) and the same T = max_w T_w, a bound on every unlisted running
//      minimum of the cloud, and ranks and certifies the same prefix as the one-workgroup kernel
//      would on that list: identical decisions in every workgroup, so they stay in lockstep;
//   4. updates its own points with the accepted centres.
// A workgroup that falls back (ties beyond its cap) or whose points are all at 0 ("empty", after
// every one of its points was picked) publishes no candidates but its best (value, index) key;
// such a round, or one without any candidate, accepts the single global argmax (value desc,
// index asc) -- the reference's step.  Slots are double-buffered by round parity (a workgroup
// can publish round r + 2 only after every peer published r + 1, i.e. finished reading r).
// Roles (default, `ticket`): a workgroup takes ticket t when it starts running, cloud t / S, part
// t % S, so the tickets handed out cover whole clouds plus at most one partly started cloud: a
// waiting workgroup waits only for peers that already run or take the next free slots on the
// device.  (DVCP_FPS_PART_TICKET=0: block b -> cloud (b / 8 / S) * 8 + b % 8, part (b / 8) % S,
// a cloud's workgroups on one XCD under round-robin placement; same speed in the lab and the
// bench.)  The wait is bounded (spin_cap polls) as a guard: a workgroup that gives up raises err
// and the cloud's remaining outputs repeat the start point (in range, finite).  (Early in round 6
// the guard fired with ten batches in flight; the cause was the workspace, not the wait: its
// slots lacked the per-wave T granules, so the last clouds' exchange overran into the flags --
// fps_part_ws, kPartMaxWaves.)
// The Morton order is computed once per cloud, by part 0: its within-cell order comes from LDS
// atomics and differs between workgroups, so independent sorts would deal some points to two parts
// and others to none.  Part 0 writes the order to `perm` (write-through stores, then the cloud's
// flag), once per launch, and each part reads the indices of its own groups into LDS: clouds of
// up to 65536 points (16-bit indices in LDS).
struct FpsPartArgs {
  uint64_t* slots;   // [B][2][S][kPartHdr + W + 5 * (128 / S)] granules, all ones before the launch
  uint32_t* flag;    // [B], all ones before the launch; 1 once part 0 has published the permutation
  uint32_t* perm;    // [B][perm_words]: the cloud's Morton order (original index per sorted position)
  int32_t* err;
  int S;             // workgroups per cloud: 2, 4 or 8
  int B;             // clouds (the grid is ceil(B / 8) * 8 * S blocks; B * S with tickets)
  int perm_words;    // N
  uint32_t spin_cap;
  int target;        // candidates a part aims to list per round (0: min(128 / S, max(kSelMin, 96 / S)))
  uint32_t* ticket;  // all ones before the launch: roles by start order; nullptr: roles by blockIdx
};
// a part's slot: kPartHdr header granules (count | flags << 16, best v, best idx, its x, y, z, two
// spare), then one T granule per wave (the largest running minimum it did not list), then the
// candidates' v, idx, x, y, z (capw each)
constexpr int kPartHdr = 8;
constexpr int kPartMaxWaves = 16;  // the workspace's T granules per slot (fps_part_ws): up to 1024 threads
constexpr int kPartMaxN = 65536;       // 16-bit point indices in LDS
constexpr uint32_t kPartFlagFb = 1u, kPartFlagEmpty = 2u;
__device__ __forceinline__ void granule_put(uint64_t* g, uint32_t data, uint32_t tag) {
  __hip_atomic_store(g, (static_cast<uint64_t>(tag) << 32) | data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// DVCP_FPS_PAIR_DIAG (timing experiments only, wrong results for 1 and 2): 1 layer 3 stops after
// its start; 2 no tie re-ranking; 3 layer 3 leaves its re-ranked round count in slot[b]
#ifndef DVCP_FPS_PAIR_DIAG
#define DVCP_FPS_PAIR_DIAG 0
#endif

// MODE 0: one cloud per workgroup; 1: the paired launch (role from a ticket); 2: only the clouds
// whose pair flag is set (the paired launch's fallback); 3: S workgroups per cloud (FpsPartArgs).
template <typename T, int PPT, bool TIMING, int THREADS, int MODE>
__device__ __forceinline__ void fps_select_body(PointsView<T> pts, int N, int npoint,
                                                const int64_t* __restrict__ start,
                                                int64_t* __restrict__ out_idx,
                                                T* __restrict__ out_xyz,
                                                unsigned long long* __restrict__ prof,
                                                const FpsPairArgs<T>& pa, const FpsPartArgs& qa = FpsPartArgs{}) {
  constexpr int W = THREADS / kWave;
  static_assert(PPT <= 32 && kSelMax == 128 && (THREADS == 256 || THREADS == 512 || THREADS == 1024), "layout");
  static_assert(MODE != 3 || (sizeof(T) == 4 && DVCP_FPS_ACC4), "split select: fp32, centres as LDS rows");
  static_assert(MODE != 3 || THREADS / kWave <= kPartMaxWaves, "split select: slot layout of fps_part_ws");
  // group lanes: lane l holds the box and exact maximum of the wave's group p = l % GP, replicated
  // over the QC = 64 / GP lane blocks, so one update test covers QC (centre, group) pairs per group
  constexpr int GP = PPT <= 2 ? 2 : PPT <= 4 ? 4 : PPT <= 8 ? 8 : PPT <= 16 ? 16 : 32;
  constexpr int QC = kWave / GP;
  __shared__ uint32_t bins[kMortonBins];  // setup; then the list's values [0, kSelCap) and positions
  __shared__ uint16_t perm[THREADS * PPT];  // original index of each of this workgroup's slots
  __shared__ T red[2][3][W];
  __shared__ uint32_t wsum[W];
  __shared__ T lx[kSelCap], ly[kSelCap], lz[kSelCap];
  __shared__ uint32_t hist[kSelBins];
  __shared__ __attribute__((aligned(16))) float cvv[kSelMax];
  __shared__ __attribute__((aligned(16))) int cpid[kSelMax];
  __shared__ __attribute__((aligned(16))) T cxx[kSelMax];
  __shared__ __attribute__((aligned(16))) T cyy[kSelMax];
  __shared__ __attribute__((aligned(16))) T czz[kSelMax];
  // per candidate, summed over the waves' i-ranges by LDS atomics: count of preceding candidates
  // (bits 0-15) + count of waves with a toucher (bits 16+); phase 5 reads one word per candidate
  // instead of one per wave (it ran on every wave, 4 per SIMD, with W reads each)
  __shared__ uint32_t srank[kSelMax];
  __shared__ uint32_t srank2[DVCP_FPS_RECERT ? kSelMax : 1];                   // the second pass's ranks
  __shared__ __attribute__((aligned(16))) float cvv2[DVCP_FPS_RECERT ? kSelMax : 4];  // its values
  __shared__ float vpart[DVCP_FPS_RECERT ? THREADS : 1];  // their partial minima (THREADS / 128 centre strides)
  // MODE 3: the second pass's candidates compacted into a dense list (index, coordinates, merged-
  // list slot; values in cvv2): the merged list's unused slots and dropped candidates leave it
  constexpr int kC2 = DVCP_FPS_RECERT && MODE == 3 ? kSelMax : 4;
  __shared__ __attribute__((aligned(16))) int c2pid[kC2];
  __shared__ __attribute__((aligned(16))) T c2x[kC2];
  __shared__ __attribute__((aligned(16))) T c2y[kC2];
  __shared__ __attribute__((aligned(16))) T c2z[kC2];
  __shared__ int c2slot[kC2];
  __shared__ float wtf[W];
  // T_f and T (non-negative floats as bits) reduced over the waves by LDS atomicMax: every wave
  // reads one word instead of W
  __shared__ uint32_t tf_max, tb_max;
  __shared__ uint32_t wpid[W];
#if DVCP_FPS_ACC4
  struct alignas(4 * sizeof(T)) AccC {
    T x, y, z, w;
  };
  __shared__ AccC acc4[kSelAccept];  // the round's accepted centres, rank order, one row each
#else
  __shared__ T acx[kSelAccept], acy[kSelAccept], acz[kSelAccept];  // the round's accepted centres, rank order
#endif
  __shared__ T gbox[W][6][GP];  // group boxes, read back per round by the update (not held in VGPRs)
  __shared__ uint32_t na_cnt, cand_fill;
  __shared__ int ckey[MODE == 1 ? kSelMax : 1];  // MODE 1: candidates' point indices in a re-ranked round
  __shared__ int s_gaveup;
  // MODE 3: the round's headers of every part (kPartHdr words each), every part's per-wave T, and
  // this part's empty-key
  __shared__ uint32_t phdr[MODE == 3 ? 8 : 1][kPartHdr];
  __shared__ uint32_t phdrT[MODE == 3 ? 8 * W : 1];
  __shared__ uint32_t s_minidx;
  float* lv = reinterpret_cast<float*>(bins);
  uint32_t* lpos = bins + kSelCap;

  const int tid = threadIdx.x, lane_outer = tid & 63, lane = lane_outer;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: its LDS addresses stay in SGPRs
  int b = blockIdx.x;
  // MODE 3: this workgroup's part of the cloud (see FpsPartArgs); S = 1, part = 0 otherwise
  int S = 1, part = 0;
  int capw = kSelMax;         // candidates this workgroup may list per round
  int seltarget = kSelTarget;
  uint64_t* qslot = nullptr;  // MODE 3: [2][S][slot] granules of this cloud
  int slotsz = 0;
  if constexpr (MODE == 3) {
    S = qa.S;
    if (qa.ticket) {
      __shared__ uint32_t s_ticket;
      if (tid == 0) s_ticket = __hip_atomic_fetch_add(qa.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
      __syncthreads();
      const int t = __builtin_amdgcn_readfirstlane(static_cast<int>(s_ticket));  // (from all ones: 0, 1, ...)
      b = t / S;
      part = t % S;
    } else {
      const int x = static_cast<int>(blockIdx.x) & 7, q = static_cast<int>(blockIdx.x) >> 3;
      b = (q / S) * 8 + x;
      part = q % S;
    }
    if (b >= qa.B) return;  // grid padding: no partner waits for it (its whole cloud is padding)
    capw = kSelMax / S;
    // (1.5 x the one-workgroup target over the parts: with the second pass, S = 4 ran 10000 ->
    // 10000 in 2.58 instead of 2.89 ms at 24 per part; S = 2 and 8 the same within 1 %,
    // profiles/round6/r6y_fps_target_sweep.log; the one-workgroup kernel is fastest at 64)
    seltarget = qa.target > 0 ? min(qa.target, capw) : min(capw, max(kSelMin, (3 * kSelTarget / 2) / S));
    slotsz = kPartHdr + W + 5 * capw;
    qslot = qa.slots + static_cast<int64_t>(b) * 2 * S * slotsz;
    if (tid == 0) s_gaveup = 0;
  }
  // sorted position of point slot p of `wv`'s lane `ln` (groups dealt to the parts, then the waves)
  auto posof = [&](int p, int wv, int ln) { return ((p * W + wv) * S + part) * kWave + ln; };  // sorted position
  auto locof = [&](int p, int wv, int ln) { return (p * W + wv) * kWave + ln; };  // this part's slot (perm)
  bool consumer = false;  // MODE 1: this workgroup runs layer 3
  int s3 = -1;            // MODE 1, layer 2: the pick number whose index layer 3 waits for
  if constexpr (MODE == 1) {
    __shared__ uint32_t s_ticket;
    if (tid == 0) s_gaveup = 0;
    if (tid == 0) s_ticket = __hip_atomic_fetch_add(pa.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(static_cast<int>(s_ticket));
    const int B = static_cast<int>(gridDim.x) / 2;
    consumer = t >= B;
    b = consumer ? t - B : t;
    if (!consumer) {
      const int64_t s = pa.start3[b];
      s3 = (s < 0 || s >= npoint) ? 0 : static_cast<int>(s);  // (the layer-3 launch clamps the same way)
    }
  }
  if constexpr (MODE == 2) {
    if (pa.flag[b] == 0) return;
  }
  auto publish = [&](int pick, int64_t idx) {  // layer 2: pick number s3 -> layer 3's start; inverse order
    if constexpr (MODE == 1) {
      if (!consumer) {
        __hip_atomic_store(pa.inv2 + static_cast<int64_t>(b) * N + idx, 0x80000000u | static_cast<uint32_t>(pick),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pick == s3)
          __hip_atomic_store(pa.slot + b, 0x80000000u | static_cast<uint32_t>(idx), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  bool tied = false;  // MODE 1: this cloud needs the gated recomputation (see the fallback below)
  [[maybe_unused]] int n_repair = 0;
  [[maybe_unused]] uint64_t rep_clk = 0;
  if constexpr (MODE == 3) {
    // part 0 sorts the whole cloud into the workspace (write-through stores, drained, then the flag);
    // every part then reads its own groups' original indices into perm, by local slot
    uint32_t* const gperm = qa.perm + static_cast<int64_t>(b) * qa.perm_words;
    if (part == 0) {
      fps_morton_sort<T, THREADS>(
          pts, b, N, bins,
          [&](uint32_t pos, int n) {
            __hip_atomic_store(gperm + pos, static_cast<uint32_t>(n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          },
          red, wsum);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(qa.flag + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {  // wait for part 0's flag (one lane)
      if (tid == 0) {
        uint32_t polls = 0;
        while (__hip_atomic_load(qa.flag + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1u) {
          if (++polls > qa.spin_cap) {
            s_gaveup = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
      if (s_gaveup) {  // guard: raise err; part 0 (which never waits here) fills the outputs
        if (tid == 0) __hip_atomic_fetch_or(qa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
#pragma unroll 1
    for (int p = 0; p < PPT; ++p) {
      const int pos = posof(p, wave, lane);
      perm[locof(p, wave, lane)] = static_cast<uint16_t>(
          pos < N ? __hip_atomic_load(gperm + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u);
    }
    __syncthreads();
  } else {
    fps_morton_sort<T, THREADS>(pts, b, N, bins, [&](uint32_t pos, int n) { perm[pos] = static_cast<uint16_t>(n); },
                                red, wsum);
  }

  T px[PPT], py[PPT], pz[PPT];
  float dmin[PPT];
  T gb[6];  // lane l: box of group (wave, l % GP)
  const int gl = lane & (GP - 1);  // this lane's group
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    gb[a] = static_cast<T>(__builtin_huge_val());
    gb[3 + a] = -static_cast<T>(__builtin_huge_val());
  }
#pragma unroll 1
  for (int p = 0; p < PPT; ++p) {
    const int pos = posof(p, wave, lane);  // groups interleaved over the (parts and) waves
    const bool real = pos < N;
    const uint32_t n = perm[real ? locof(p, wave, lane) : 0];
    const T x = pts.at(b, 0, n), y = pts.at(b, 1, n), z = pts.at(b, 2, n);
    px[p] = real ? x : static_cast<T>(0);
    py[p] = real ? y : static_cast<T>(0);
    pz[p] = real ? z : static_cast<T>(0);
    dmin[p] = real ? 1e10f : -1.0f;  // torch.ones(B, N) * 1e10 (fp32), :74; padding: never listed
    const T inf = static_cast<T>(__builtin_huge_val());
    T l[3] = {real ? x : inf, real ? y : inf, real ? z : inf};
    T h[3] = {real ? x : -inf, real ? y : -inf, real ? z : -inf};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      for (int off = 32; off > 0; off >>= 1) {
        const T ol = __shfl_xor(l[a], off, kWave), oh = __shfl_xor(h[a], off, kWave);
        l[a] = ol < l[a] ? ol : l[a];
        h[a] = oh > h[a] ? oh : h[a];
      }
      gb[a] = gl == p ? l[a] : gb[a];
      gb[3 + a] = gl == p ? h[a] : gb[3 + a];
    }
  }
  const bool grp = gl < PPT && posof(gl, wave, 0) < N;  // lane l: a non-empty group
  if (lane < GP) {
#pragma unroll
    for (int a = 0; a < 6; ++a) gbox[wave][a][lane] = gb[a];
  }
  if constexpr (MODE == 3) {
    // the key this part publishes once all its points are at 0: the lowest original index it holds
    // (every point of an empty part has running minimum 0, the argmax's value)
    if (tid == 0) s_minidx = 0xFFFFFFFFu;
    lds_barrier();
    uint32_t mi = 0xFFFFFFFFu;
#pragma unroll 1
    for (int p = 0; p < PPT; ++p) {
      const int pos = posof(p, wave, lane);
      if (pos < N) mi = min(mi, static_cast<uint32_t>(perm[locof(p, wave, lane)]));
    }
    mi = wave_umin(mi);
    if (lane == 0 && mi != 0xFFFFFFFFu) atomicMin(&s_minidx, mi);
  }

  int64_t* const oidx = MODE == 1 && consumer ? pa.out3_idx : out_idx;
  T* const oxyz = MODE == 1 && consumer ? pa.out3_xyz : out_xyz;
  int64_t* oi = oidx + static_cast<int64_t>(b) * npoint;
  T* ox = oxyz ? oxyz + static_cast<int64_t>(b) * 3 * npoint : nullptr;
  int64_t cur;
  if constexpr (MODE == 1) {
    if (consumer) {  // wait for layer 2's pick number start3 (the setup above ran meanwhile)
      __shared__ uint32_t s_start;
      if (tid == 0) {
        uint32_t v = 0, polls = 0;
        for (;;) {
          v = __hip_atomic_load(pa.slot + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v & 0x80000000u) break;
          __builtin_amdgcn_s_sleep(8);
          if (++polls > kFpsPairSpinCap) {
            v = 0u;
            break;
          }
        }
        s_start = v;
      }
      __syncthreads();
      const uint32_t v = s_start;
      if (!(v & 0x80000000u)) {  // gave up waiting: the gated launch recomputes this cloud
        if (tid == 0) __hip_atomic_fetch_or(pa.flag + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      cur = static_cast<int64_t>(v & 0x7FFFFFFFu);
#if DVCP_FPS_PAIR_DIAG == 1
      return;
#endif
    } else {
      cur = start[b];
    }
  } else {
    cur = start[b];
  }
  if (cur < 0 || cur >= N) cur = 0;  // host validates; keep the kernel in bounds regardless
  float gub, vmax;
  {
    const T cx = pts.at(b, 0, cur), cy = pts.at(b, 1, cur), cz = pts.at(b, 2, cur);
    if (tid == 0 && part == 0) {
      oi[0] = cur;
      publish(0, cur);
      if (ox) {
        ox[0] = cx;
        ox[npoint] = cy;
        ox[2 * npoint] = cz;
      }
    }
    float m = -1.0f;
#pragma unroll
    for (int p = 0; p < PPT; ++p) {
      dmin[p] = fps_update<T>(dmin[p], px[p], py[p], pz[p], cx, cy, cz);
      m = fmaxf(m, dmin[p]);
    }
    // exact group maxima (kept exact: groups whose minima drop are re-reduced after each update)
    gub = -1.0f;
#pragma unroll 1
    for (int p = 0; p < PPT; ++p) {
      const float gm = wave_fmax_clamp0(dmin[p]);
      gub = gl == p ? gm : gub;
    }
    gub = grp ? gub : -1.0f;
    m = wave_fmax_clamp0(m);
    if (lane == 0) wtf[wave] = m;
  }
  for (int i = tid; i < kSelBins; i += THREADS) hist[i] = 0u;
  if (tid == 0) {
    na_cnt = 0u;
    cand_fill = 0u;
    tf_max = 0u;
    tb_max = 0u;
  }
  lds_barrier();
  vmax = wtf[0];
#pragma unroll
  for (int w = 1; w < W; ++w) vmax = fmaxf(vmax, wtf[w]);
  lds_barrier();  // wtf is rewritten by the first scan

  float f = 0.0f;  // floor: the first scan lists every positive value and re-derives f
  int step = 1;
  unsigned long long n_round = 0, n_scan = 0, n_fallback = 0;
  [[maybe_unused]] bool part_quit = false;  // MODE 3: gave up waiting for a peer (guard)
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};  // TIMING: scan, decide+list(+exchange), rank, prefix+k, update
  unsigned long long why[4] = {0, 0, 0, 0};       // TIMING: rescans for none above f, > cap, < kSelMin, crowded bin
  uint64_t tp = 0;
  auto tick = [&](int k) {
    if constexpr (TIMING) {
      const uint64_t t = fps_clock();
      if (k >= 0) ph[k] += t - tp;
      tp = t;
    }
  };
  // MODE 3, step 2 of a round.  The granules of the round: wave 0 publishes the header and the
  // unused candidate slots once the round's decision is final (part_publish); every wave its T
  // (part_publish_t, from the list pass); the list pass the candidates.  part_gather then reads
  // every other part's granules of the round into the merged list, phdr and phdrT (the caller's
  // next barrier completes it).
  auto round_slot = [&](int q) { return qslot + (static_cast<int64_t>(n_round & 1) * S + q) * slotsz; };
  auto part_publish = [&](uint32_t flags, int cntw, uint32_t bv_bits, uint32_t best_i) {  // wave 0
    if constexpr (MODE == 3) {
      const uint32_t tag = static_cast<uint32_t>(n_round);
      uint64_t* const mine = round_slot(part);
      if (lane < kPartHdr) {
        uint32_t d = lane == 0 ? (static_cast<uint32_t>(cntw) | (flags << 16)) : lane == 1 ? bv_bits
                                                                               : lane == 2 ? best_i : 0u;
        if (lane >= 3 && lane < 6 && flags != 0u && best_i < static_cast<uint32_t>(N))
          d = __float_as_uint(pts.at(b, lane - 3, static_cast<int>(best_i)));
        phdr[part][lane] = d;
        granule_put(mine + lane, d, tag);
      }
      for (int o = cntw + lane; o < capw; o += kWave) {  // unused slots: v = -1 never ranks or wins
        const int j = part * capw + o;
        cvv[j] = -1.0f;
        cpid[j] = 0x7FFFFFFF;
        cxx[j] = 0.0f;
        cyy[j] = 0.0f;
        czz[j] = 0.0f;
        uint64_t* g = mine + kPartHdr + W + o;
        granule_put(g, __float_as_uint(-1.0f), tag);
        granule_put(g + capw, 0x7FFFFFFFu, tag);
        granule_put(g + 2 * capw, 0u, tag);
        granule_put(g + 3 * capw, 0u, tag);
        granule_put(g + 4 * capw, 0u, tag);
      }
    }
  };
  auto part_publish_t = [&](uint32_t t_bits) {  // lane 0 of every wave: this wave's T
    if constexpr (MODE == 3) {
      phdrT[part * W + wave] = t_bits;
      granule_put(round_slot(part) + kPartHdr + wave, t_bits, static_cast<uint32_t>(n_round));
    }
  };
  auto part_gather = [&]() {
    if constexpr (MODE == 3) {
      const uint32_t tag = static_cast<uint32_t>(n_round);
      const int others = (S - 1) * slotsz;
      for (int t = tid; t < others; t += THREADS) {
        const int qq = t / slotsz, k = t - qq * slotsz;
        const int q = qq + (qq >= part ? 1 : 0);
        const uint64_t* g = round_slot(q) + k;
        uint64_t v = 0;
        uint32_t polls = 0;
        for (;;) {
          v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (static_cast<uint32_t>(v >> 32) == tag) break;
          if (++polls > qa.spin_cap) {
            s_gaveup = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t d = static_cast<uint32_t>(v);
        if (k < kPartHdr) {
          phdr[q][k] = d;
        } else if (k < kPartHdr + W) {
          phdrT[q * W + (k - kPartHdr)] = d;
        } else {
          const int c = (k - kPartHdr - W) / capw, o = (k - kPartHdr - W) - c * capw, j = q * capw + o;
          if (c == 0) cvv[j] = __uint_as_float(d);
          else if (c == 1) cpid[j] = static_cast<int>(d);
          else if (c == 2) cxx[j] = __uint_as_float(d);
          else if (c == 3) cyy[j] = __uint_as_float(d);
          else czz[j] = __uint_as_float(d);
        }
      }
    }
  };
  // MODE 3, after the gather's barrier: T = max over every part's waves, the candidate total, whether
  // some part fell back, and this part's own T (lane-parallel reads, wave reductions; every wave)
  auto part_merge = [&](uint32_t& tg, uint32_t& total, uint32_t& fb, uint32_t& tw) {
    uint32_t t = 0u, tt = 0u, c = 0u, f = 0u;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int i = hh * kWave + lane;
      if (i < S * W) {
        const uint32_t x = phdrT[i];
        t = max(t, x);
        if (i / W == part) tt = max(tt, x);
      }
    }
    if (lane < S) {
      const uint32_t h = phdr[lane][0];
      c = h & 0xFFFFu;
      f = (h >> 16) & kPartFlagFb;
    }
    uint32_t ma, mb;
    wave_umax2(t, tt, ma, mb);
    tg = ma;
    tw = mb;
    fb = wave_umax(f);
    total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wave_incl_scan(c)), 63));
  };
  // MODE 3: a round without certification (some part fell back, or no part listed a candidate)
  // accepts the single global argmax over the listed candidates and the fallen-back / empty parts'
  // keys: value desc, original index asc (:83).  Every wave computes the same key; returns it.
  auto part_argmax = [&]() -> uint32_t {
    uint64_t key = 0;
    if constexpr (MODE != 3) return 0u;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int jj = hh * kWave + lane;
      const float v = cvv[jj];
      if (v >= 0.0f)
        key = max(key, (static_cast<uint64_t>(__float_as_uint(v)) << 32) | (0xFFFFFFFFu - static_cast<uint32_t>(cpid[jj])));
    }
    if (lane < S && (phdr[lane][0] >> 16) != 0u)
      key = max(key, (static_cast<uint64_t>(phdr[lane][1]) << 32) | (0xFFFFFFFFu - phdr[lane][2]));
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t o = __shfl_xor(key, off, kWave);
      key = o > key ? o : key;
    }
    return 0xFFFFFFFFu - static_cast<uint32_t>(key);
  };
  while (step < npoint) {
    // The lane index is re-materialised (v_mbcnt in a volatile asm, fresh_lane) at the start of
    // each scan and of the update: the round's LDS addresses are then recomputed from it (a few
    // VALU ops) instead of being hoisted out of the loop as ~40 lane-dependent constants, and no
    // lane register stays live across the round -- at 1024 threads (128 VGPRs) both were spilled.
    ++n_round;
    int kstar = 0;
    bool raised = false;
    for (int scan = 0;; ++scan) {
      const int lane = fresh_lane();  // (see the round loop)
      ++n_scan;
      tick(-1);
      // ---- 1. scan: list the points above f, histogram their float bits over (f, vmax] ----------
      const uint32_t kf = __float_as_uint(f);
      const uint32_t kv = max(__float_as_uint(vmax), kf + 1u);
      const int shift = sel_shift(kv - kf);
      float tf = 0.0f;
      uint32_t nh = 0;
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        const float v = dmin[p];
        const bool hit = v > f;
        tf = hit ? tf : fmaxf(tf, v);
        nh += hit ? 1u : 0u;
      }
      // this lane's list offset: one wave scan and one LDS atomic per wave
      const uint32_t incl = wave_incl_scan(nh);
      const uint32_t wtot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
      uint32_t wbase = 0;
      if (wtot) {
        if (lane == 0) wbase = atomicAdd(&na_cnt, wtot);
        wbase = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(wbase)));
      }
      uint32_t li = wbase + incl - nh;
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        const float v = dmin[p];
        const bool hit = v > f;
        if (__ballot(hit)) {
          if (hit) {
            const uint32_t bin = min((__float_as_uint(v) - kf) >> shift, static_cast<uint32_t>(kSelBins - 1));
            atomicAdd(&hist[bin], 1u);
            if (li < kSelCap) {
              lv[li] = v;
              lpos[li] = static_cast<uint32_t>(locof(p, wave, lane));
              lx[li] = px[p];
              ly[li] = py[p];
              lz[li] = pz[p];
            }
            ++li;
          }
        }
      }
      tf = wave_fmax_clamp0(tf);
      if (lane == 0) atomicMax(&tf_max, __float_as_uint(tf));
      lds_barrier();
      tick(0);
      // ---- 2. decide (every wave computes the same decision from LDS) -------------------------
      const uint32_t na = na_cnt;
      const float Tf = __uint_as_float(tf_max);
      // suffix counts: lane l holds bins 4l .. 4l+3; suf(k) = hits in bins >= k
      uint32_t h[4], hs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) h[k] = hist[4 * lane + k];
      hs[3] = h[3];
      hs[2] = h[2] + hs[3];
      hs[1] = h[1] + hs[2];
      hs[0] = h[0] + hs[1];
      uint32_t above = 0;  // hits in lanes > this lane: the wave total minus the inclusive prefix
      {
        const uint32_t incl = wave_incl_scan(hs[0]);
        above = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63)) - incl;
      }
      // the largest bin k with suf(k) >= need (suf is non-increasing in k)
      auto last_bin_at_least = [&](uint32_t need) -> int {
        int best = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) best = (hs[k] + above >= need) ? 4 * lane + k : best;
        return static_cast<int>(wave_umax(static_cast<uint32_t>(best + 1))) - 1;
      };
      auto suf_of = [&](int bin) -> uint32_t {  // suf(bin), uniform bin
        const int L = bin >> 2, k = bin & 3;
        const uint32_t mine = (k == 0 ? hs[0] : k == 1 ? hs[1] : k == 2 ? hs[2] : hs[3]) + above;
        return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(mine), L));
      };
      // 0: select, 1: rescan with the new f, 2: fallback (one exact argmax), 3 (MODE 3): every point
      // of this part is at 0 (empty)
      int mode = 0;
      int bsel = 0;
      if (scan >= kSelMaxScans) {
        mode = 2;
      } else if (na == 0) {
        if (Tf > 0.0f) {
          f = prev_float(Tf);
          mode = 1;
          ++why[0];
        } else {
          mode = MODE == 3 ? 3 : 2;
        }
      } else {
        // highest non-empty bin: values lie below its upper edge, a tighter vmax for a rescan
        const int top = last_bin_at_least(1);
        auto tighten = [&]() {
          if (top < kSelBins - 1) vmax = fminf(vmax, __uint_as_float(kf + (static_cast<uint32_t>(top + 1) << shift)));
        };
        auto edge_below = [&](int bin) {  // the f that lists exactly bins >= bin
          return __uint_as_float(kf + (static_cast<uint32_t>(bin) << shift) - 1u);
        };
        if (na > static_cast<uint32_t>(kSelCap)) {
          int bb = max(0, last_bin_at_least(4 * seltarget));
          while (bb + 1 < kSelBins && suf_of(bb) > static_cast<uint32_t>(kSelCap) && suf_of(bb + 1) > 0u) ++bb;
          if (shift == 0 && suf_of(bb) > static_cast<uint32_t>(kSelCap)) {
            mode = 2;  // more than kSelCap points share one value
          } else {
            if (bb > 0) f = edge_below(bb);
            tighten();
            mode = 1;
            raised = true;
            ++why[1];
          }
        } else if (na < static_cast<uint32_t>(kSelMin) && Tf > 0.0f && !raised) {
          f = fminf(f * 0.5f, prev_float(Tf));
          mode = 1;
          ++why[2];
        } else {
          bsel = max(0, last_bin_at_least(min(static_cast<uint32_t>(seltarget), na)));
          while (bsel + 1 < kSelBins && suf_of(bsel) > static_cast<uint32_t>(capw) && suf_of(bsel + 1) > 0u) ++bsel;
          if (suf_of(bsel) > static_cast<uint32_t>(capw)) {  // a crowded top bin
            if (shift == 0) {
              mode = 2;
            } else {
              if (bsel > 0) f = edge_below(bsel);
              tighten();
              mode = 1;
              raised = true;
              ++why[3];
            }
          }
        }
      }
      if (mode == 1) {  // rescan: everyone has read hist / na / wtf; clear them
        lds_barrier();
        for (int i = tid; i < kSelBins; i += THREADS) hist[i] = 0u;
        if (tid == 0) {
          na_cnt = 0u;
          tf_max = 0u;
        }
        lds_barrier();
        continue;
      }
      if (mode == 2) {
        // ---- fallback: one exact argmax (value desc, original index asc) over every point ------
        ++n_fallback;
        float bv = -1.0f;  // opaque: the max over dmin is formed here, not hoisted out of the scan loop
        asm volatile("" : "+v"(bv));
#pragma unroll
        for (int p = 0; p < PPT; ++p) bv = fmaxf(bv, dmin[p]);
        bv = wave_fmax_clamp0(bv);
        lds_barrier();  // (wtf / hist reads above are done)
        if (lane == 0) wtf[wave] = bv;
        for (int i = tid; i < kSelBins; i += THREADS) hist[i] = 0u;
        if (tid == 0) {
          na_cnt = 0u;
          tf_max = 0u;
        }
        lds_barrier();
        float gmax = wtf[0];
#pragma unroll
        for (int w = 1; w < W; ++w) gmax = fmaxf(gmax, wtf[w]);
        uint32_t mp = 0xFFFFFFFFu;
#pragma unroll
        for (int p = 0; p < PPT; ++p) {
          if (__ballot(dmin[p] == gmax)) {
            if (dmin[p] == gmax) mp = min(mp, static_cast<uint32_t>(perm[locof(p, wave, lane)]));
          }
        }
        mp = wave_umin(mp);
        if (lane == 0) wpid[wave] = mp;
        lds_barrier();
        uint32_t gp = wpid[0];
#pragma unroll
        for (int w = 1; w < W; ++w) gp = min(gp, wpid[w]);
        if constexpr (MODE == 3) {  // this part's key goes to the others; the round takes the global one
          if (wave == 0) part_publish(kPartFlagFb, 0, __float_as_uint(gmax), gp);
          if (lane == 0) part_publish_t(__float_as_uint(gmax));
          part_gather();
          lds_barrier();
          if (s_gaveup) {
            part_quit = true;
            break;
          }
          gp = part_argmax();
        }
        if (tid == 0) {
          const T gx = pts.at(b, 0, gp), gy = pts.at(b, 1, gp), gz = pts.at(b, 2, gp);
#if DVCP_FPS_ACC4
          acc4[0] = AccC{gx, gy, gz, static_cast<T>(0)};
#else
          acx[0] = gx;
          acy[0] = gy;
          acz[0] = gz;
#endif
          if (part == 0) {
            oi[step] = static_cast<int64_t>(gp);
            publish(step, static_cast<int64_t>(gp));
            if (ox) {
              ox[step] = gx;
              ox[npoint + step] = gy;
              ox[2 * npoint + step] = gz;
            }
          }
        }
        lds_barrier();
        kstar = 1;
        vmax = gmax;  // every value is <= gmax; the new centre's drops to 0
        // MODE 1: layer 3 does not resolve this argmax's ties, and a layer-2 pick at value 0 means
        // layer 2 may repeat points (its centres are then not layer 2's points as a set): the gated
        // launch recomputes such a cloud
        if (consumer || !(gmax > 0.0f)) tied = true;
        if constexpr (MODE == 1) {
          // layer 2 repeating points: raise the cloud's flag now, not at the end, so a layer-3
          // workgroup waiting for a pick number that will never come stops at its next poll
          if (!consumer && !(gmax > 0.0f) && tid == 0)
            __hip_atomic_fetch_or(pa.flag + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
      // ---- 3. list: entries in bins >= bsel are the candidates; T over the rest ---------------
      // (MODE 3: this part's candidates go to its own range of the merged list and out as
      // granules; an empty part lists nothing: na = 0)
      int cnt = static_cast<int>(suf_of(bsel));
      int nreal = cnt;  // candidates in the list (MODE 3: the merged list's, without its unused slots)
      const int cbase = part * capw;
      uint64_t* const cgran = MODE == 3 ? round_slot(part) + kPartHdr + W : nullptr;
      if constexpr (MODE == 3) {  // the decision is final: header and unused slots go out now
        if (wave == 0) part_publish(mode == 3 ? kPartFlagEmpty : 0u, cnt, 0u, mode == 3 ? s_minidx : 0u);
      }
      float tl = Tf;
      for (int i = wave * (kSelCap / W) + lane; i < (wave + 1) * (kSelCap / W); i += kWave) {
        const bool live = i < static_cast<int>(na);
        const float v = live ? lv[i] : 0.0f;
        const bool in = live && static_cast<int>(min((__float_as_uint(v) - kf) >> shift,
                                                     static_cast<uint32_t>(kSelBins - 1))) >= bsel;
        tl = (live && !in) ? fmaxf(tl, v) : tl;
        const uint64_t m = __ballot(in);
        if (m) {
          const int first = __ffsll(static_cast<long long>(m)) - 1;
          uint32_t base = 0;
          if (lane == first) base = atomicAdd(&cand_fill, static_cast<uint32_t>(__popcll(m)));
          base = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(base), first));
          const uint32_t o = base + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0));
          if (in) {
            const int j = cbase + static_cast<int>(o);
            const int pid = static_cast<int>(perm[lpos[i]]);
            cvv[j] = v;
            cpid[j] = pid;
            cxx[j] = lx[i];
            cyy[j] = ly[i];
            czz[j] = lz[i];
            if constexpr (MODE == 3) {
              const uint32_t tag = static_cast<uint32_t>(n_round);
              uint64_t* g = cgran + o;
              granule_put(g, __float_as_uint(v), tag);
              granule_put(g + capw, static_cast<uint32_t>(pid), tag);
              granule_put(g + 2 * capw, __float_as_uint(lx[i]), tag);
              granule_put(g + 3 * capw, __float_as_uint(ly[i]), tag);
              granule_put(g + 4 * capw, __float_as_uint(lz[i]), tag);
            }
          }
        }
      }
      tl = wave_fmax_clamp0(tl);
      if (lane == 0) atomicMax(&tb_max, __float_as_uint(tl));
      if constexpr (MODE == 3) {
        if (lane == 0) part_publish_t(__float_as_uint(tl));
      }
      // next round: keep a few hundred points above the floor.  The decay sets how often a round
      // lists more than kSelCap points and scans again: 0.85 rescanned in ~20 % of the C3 rounds
      // (sa1: 74 of 367), 0.9 in ~2 % (6 of 367; sa2 / sa3 37 -> 4 of 302), with the same rounds
      // (tools/fps_lab/fps_round_sim.py, a CPU model of this round logic; FPS lab: 81 of 382).
      if (na < 4u * static_cast<uint32_t>(seltarget)) f *= 0.9f;
      if (wave * kWave < kSelMax) srank[wave * kWave + lane] = 0u;  // (read last by the previous round)
      if (DVCP_FPS_RECERT && wave * kWave < kSelMax) srank2[wave * kWave + lane] = 0u;
      if constexpr (MODE == 3) {  // ---- MODE 3, step 2: the other parts' granules of the round ------
        tick(1);
        part_gather();
      }
      lds_barrier();
      float Tb = __uint_as_float(tb_max);
      if (tid == 0) {  // (T_f was read by every wave before this barrier)
        na_cnt = 0u;
        tf_max = 0u;
      }
      if (tid == kWave) cand_fill = 0u;
      for (int i = tid; i < kSelBins; i += THREADS) hist[i] = 0u;
      [[maybe_unused]] const float Tw = Tb;  // MODE 3: this part's own T (its next vmax bound)
      if constexpr (MODE == 3) {
        // ---- the merged list: T = max over every part's T, the candidate total, fallbacks --------
        tick(5);
        if (s_gaveup) {
          part_quit = true;
          break;
        }
        uint32_t tg, total, fb, twb;
        part_merge(tg, total, fb, twb);
        if (fb != 0u || total == 0u) {  // one exact argmax for the round
          ++n_fallback;
          const uint32_t gp = part_argmax();
          if (tid == 0) {
            const T gx = pts.at(b, 0, gp), gy = pts.at(b, 1, gp), gz = pts.at(b, 2, gp);
            acc4[0] = AccC{gx, gy, gz, static_cast<T>(0)};
            if (part == 0) {
              oi[step] = static_cast<int64_t>(gp);
              if (ox) {
                ox[step] = gx;
                ox[npoint + step] = gy;
                ox[2 * npoint + step] = gz;
              }
            }
          }
          // this part's values are at most its T and its listed values
          float vm = Tw;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int jj = hh * kWave + lane;
            vm = (jj >= cbase && jj < cbase + capw) ? fmaxf(vm, cvv[jj]) : vm;
          }
          vmax = wave_fmax_clamp0(vm);
          lds_barrier();
          if (tid == 0) tb_max = 0u;  // (every wave read it before this barrier)
          kstar = 1;
          break;
        }
        cnt = S * capw;  // the merged list (unused slots: v = -1)
        nreal = static_cast<int>(total);
        Tb = __uint_as_float(tg);
      }
      tick(1);
      // ---- 4. rank and prefix test in one pass over candidate pairs ----------------------------
      // c_i precedes c_j (value desc, index asc) iff beats(i, j); rank_j = #{i : beats(i, j)}; c_j
      // is "touched" if some c_i preceding it lowers its running minimum (d(c_i, c_j) < v_j, the
      // point update's formula).  Wave w covers i in [16w, 16w + 16) for j = lane and lane + 64:
      // every wave takes part, and each wave-uniform (broadcast) LDS read of four c_i serves both j.
      // MODE 1, layer 3: a round whose steps meet a tie is ranked again with the candidates' layer-2
      // pick numbers as the index (the reference's order for layer 3); cpid then holds those and
      // ckey the point indices.
      bool repaired = false;
      int rk[2];
      bool eqp[2] = {false, false};
      int koff = 0, nreal2 = 0;  // the second pass: centres accepted before it, its candidates
      // phases 4 and 5's decision (twice in a re-ranked round).  P2: the second pass over the
      // candidates left (values cvv2 > T, ranks in srank2, ranks offset by koff)
      auto rank_decide = [&](auto p2c) {
      constexpr bool P2 = decltype(p2c)::value;
      constexpr bool D2 = P2 && MODE == 3;  // MODE 3's second pass: the compacted (dense) list
      float* const cv = P2 ? cvv2 : cvv;
      const int* const cp = D2 ? c2pid : cpid;
      const T* const cX = D2 ? c2x : cxx;
      const T* const cY = D2 ? c2y : cyy;
      const T* const cZ = D2 ? c2z : czz;
      const int cn = D2 ? nreal2 : cnt;
      uint32_t* const sr = P2 ? srank2 : srank;
      {
        const int i_lo = wave * (kSelMax / W);
        int r0 = 0, r1 = 0, t0 = 0, t1 = 0;
        int e0 = 0, e1 = 0;  // MODE 1: c_j has an equal-valued predecessor (bits 24+ of srank)
        if (i_lo < cn) {  // wave-uniform
          const int j0 = lane, j1 = lane + kWave;
          const float v0 = cv[j0], v1 = cv[j1];
          const int p0 = cp[j0], p1 = cp[j1];
          const T x0 = cX[j0], y0 = cY[j0], z0 = cZ[j0];
          const T x1 = cX[j1], y1 = cY[j1], z1 = cZ[j1];
          // rolled at PPT 16 x 1024 threads (128 VGPRs): one batch of four candidates live at a time
          constexpr int kPairUnroll = PPT >= 16 && THREADS == 1024 ? 1 : kSelMax / W / 4;
#pragma unroll kPairUnroll
          for (int c4 = 0; c4 < kSelMax / W / 4; ++c4) {
            const int i0 = i_lo + 4 * c4;
            if (i0 >= cn) break;  // wave-uniform
            const float4 v4 = *reinterpret_cast<const float4*>(&cv[i0]);
            // MODE 3: a part's unused slots (v = -1) follow its candidates; skip all-unused batches
            // (P2: batches with no candidate left)
            if (!D2 && (P2 ? !(fmaxf(fmaxf(v4.x, v4.y), fmaxf(v4.z, v4.w)) > Tb) : (MODE == 3 && v4.x < 0.0f)))
              continue;  // (wave-uniform)
            const int4 p4 = *reinterpret_cast<const int4*>(&cp[i0]);
            const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
            const int pp[4] = {p4.x, p4.y, p4.z, p4.w};
            T xx[4], yy[4], zz[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              xx[k] = cX[i0 + k];
              yy[k] = cY[i0 + k];
              zz[k] = cZ[i0 + k];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const bool in = D2 ? i0 + k < cn : P2 ? vv[k] > Tb : MODE == 3 ? vv[k] >= 0.0f : i0 + k < cnt;
              const bool b0 = in & ((vv[k] > v0) | ((vv[k] == v0) & (pp[k] < p0)));
              const bool b1 = in & ((vv[k] > v1) | ((vv[k] == v1) & (pp[k] < p1)));
              const T ax = x0 - xx[k], ay = y0 - yy[k], az = z0 - zz[k];
              const T bx = x1 - xx[k], by = y1 - yy[k], bz = z1 - zz[k];
              const T d0 = (ax * ax + ay * ay) + az * az;
              const T d1 = (bx * bx + by * by) + bz * bz;
              r0 += b0 ? 1 : 0;
              r1 += b1 ? 1 : 0;
              t0 |= (b0 & (d0 < static_cast<T>(v0))) ? 1 : 0;
              t1 |= (b1 & (d1 < static_cast<T>(v1))) ? 1 : 0;
              if constexpr (MODE == 1) {
                e0 |= (in & (vv[k] == v0) & (pp[k] < p0)) ? 1 : 0;
                e1 |= (in & (vv[k] == v1) & (pp[k] < p1)) ? 1 : 0;
              }
            }
          }
        }
        if (i_lo < cn) {  // wave-uniform
          if (MODE == 3 || P2) {  // (unused slots take no rank; P2: nor the candidates not left)
            const bool in0 = D2 ? lane < cn : P2 ? cv[lane] > Tb : cv[lane] >= 0.0f;
            const bool in1 = D2 ? lane + kWave < cn : P2 ? cv[lane + kWave] > Tb : cv[lane + kWave] >= 0.0f;
            r0 = in0 ? r0 : 0;
            t0 = in0 ? t0 : 0;
            r1 = in1 ? r1 : 0;
            t1 = in1 ? t1 : 0;
          }
          if (r0 | t0 | e0) atomicAdd(&sr[lane], static_cast<uint32_t>(r0 | (t0 << 16) | (e0 << 24)));
          if (r1 | t1 | e1) atomicAdd(&sr[lane + kWave], static_cast<uint32_t>(r1 | (t1 << 16) | (e1 << 24)));
        }
      }
      lds_barrier();
      tick(2);
      // ---- 5. k = the smallest rank that fails; accepted = ranks < k (every wave, redundantly) ----
      if (tid == 0) tb_max = 0u;  // every wave read T before the phase-4 barrier
      const int left = npoint - step - (P2 ? koff : 0);
      eqp[0] = eqp[1] = false;
      uint32_t failr = 0xFFFFFFFFu;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int jj = hh * 64 + lane;
        rk[hh] = 0x7FFFFFFF;
        // (MODE 3: unused slots are no candidates; P2: only those left)
        if (jj < cn && (D2 || (P2 ? cv[jj] > Tb : (MODE != 3 || cv[jj] >= 0.0f)))) {
          const uint32_t e = sr[jj];
          const int r = static_cast<int>(e & 0xFFFFu);
          const bool touched = MODE == 1 ? ((e >> 16) & 0xFFu) != 0u : (e >> 16) != 0u;
          if constexpr (MODE == 1) eqp[hh] = (e >> 24) != 0u;
          rk[hh] = r;
          const bool fail = r >= left || (r > 0 && (touched || !(cv[jj] > Tb)));
          failr = fail ? min(failr, static_cast<uint32_t>(r)) : failr;
        }
      }
      kstar = static_cast<int>(min(min(wave_umin(failr), static_cast<uint32_t>(P2 ? nreal2 : nreal)),
                                   static_cast<uint32_t>(kSelAccept - (P2 ? koff : 0))));
      };
      rank_decide(std::false_type{});
      if constexpr (MODE == 1) {
        // Ties (layer 3).  Values only drop and unlisted ones stay below every listed one, so a
        // step's argmax can only tie with listed candidates of the same round-start value, and
        // equal values are adjacent in rank order.  A tie group inside the accepted prefix (no
        // member lowers another's minimum) leaves the same state after it in any order: its
        // members are marked in the output and reordered by layer 2's pick numbers once layer 2
        // is done (fps_pair_remap_kernel).  A group that reaches the first rejected candidate
        // is left to the next round; one that starts at rank 0 is ranked now by those pick
        // numbers, waiting for them.  (Every wave reads the same srank: uniform decisions.)
        const bool cut = __ballot((eqp[0] && rk[0] == kstar) || (eqp[1] && rk[1] == kstar)) != 0ull;
        int g0 = 0;  // the group's first rank: the last rank <= k without an equal-valued predecessor
        if (consumer && cut && !repaired) {
          int m = -1;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) m = (rk[hh] <= kstar && !eqp[hh]) ? max(m, rk[hh]) : m;
          g0 = static_cast<int>(wave_umax(static_cast<uint32_t>(m + 1))) - 1;
          if (g0 > 0) kstar = g0;
        }
        if (consumer && cut && !repaired && g0 == 0 && DVCP_FPS_PAIR_DIAG != 2) {
#if DVCP_FPS_PAIR_DIAG == 3
          const uint64_t t_rep = fps_clock();
#endif
          lds_barrier();  // every wave has read srank and cpid
          if (tid < cnt) {
            const int n = cpid[tid];
            ckey[tid] = n;
            uint32_t v = 0, polls = 0;
            for (;;) {  // layer 2 picks every point (else it flags the cloud): wait for this one
              v = __hip_atomic_load(pa.inv2 + static_cast<int64_t>(b) * N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (v & 0x80000000u) break;
              // layer 2 flagged the cloud (it repeats points: this one may never be picked)
              if (__hip_atomic_load(pa.flag + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                  ++polls > kFpsPairSpinCap) {
                s_gaveup = 1;
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
            cpid[tid] = static_cast<int>(v & 0x7FFFFFFFu);
          }
          if (tid < kSelMax) srank[tid] = 0u;
          lds_barrier();
          if (s_gaveup) {  // the gated launch recomputes this cloud
            if (tid == 0) __hip_atomic_fetch_or(pa.flag + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
          }
          repaired = true;
          ++n_repair;
          rank_decide(std::false_type{});
#if DVCP_FPS_PAIR_DIAG == 3
          rep_clk += fps_clock() - t_rep;
#endif
        }
      }
      // the accepted centres in rank order, for the update: every wave writes the same values
      // (its own reads below follow its own writes in LDS order); wave 0 of part 0 writes the
      // outputs.  base: the ranks' offset (the second pass's follow the first's)
      // (d2c: MODE 3's second pass, whose candidates are the compacted c2 rows)
      auto accept = [&](int base, auto d2c) {
        constexpr bool D2 = decltype(d2c)::value;
        const int* const cp = D2 ? c2pid : cpid;
        const T* const cX = D2 ? c2x : cxx;
        const T* const cY = D2 ? c2y : cyy;
        const T* const cZ = D2 ? c2z : czz;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int jj = hh * 64 + lane;
          if (rk[hh] < kstar) {
#if DVCP_FPS_ACC4
            acc4[base + rk[hh]] = AccC{cX[jj], cY[jj], cZ[jj], static_cast<T>(0)};
#else
            acx[base + rk[hh]] = cX[jj];
            acy[base + rk[hh]] = cY[jj];
            acz[base + rk[hh]] = cZ[jj];
#endif
          }
        }
        if (wave == 0 && part == 0) {  // outputs in rank order
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int jj = hh * 64 + lane;
            if (rk[hh] < kstar) {
              const int n = MODE == 1 && repaired ? ckey[jj] : cp[jj];
              // MODE 1, layer 3: bit 62 marks a member of a tie group after its first
              const bool mk = MODE == 1 && consumer && !repaired && eqp[hh];
              const int o = step + base + rk[hh];
              oi[o] = static_cast<int64_t>(n) | (mk ? (int64_t(1) << 62) : int64_t(0));
              publish(o, n);
              if (ox) {
                ox[o] = cX[jj];
                ox[npoint + o] = cY[jj];
                ox[2 * npoint + o] = cZ[jj];
              }
            }
          }
        }
      };
      accept(0, std::false_type{});
      // upper bound of every running minimum after this round: T, and the listed not accepted
      // (MODE 3: this part's own -- its T_w and its own listed values -- for a tighter histogram)
      float vm = MODE == 3 ? Tw : Tb;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int jj = hh * 64 + lane;
        const bool mine = MODE != 3 || (jj >= cbase && jj < cbase + capw);
        vm = (mine && jj < cnt && rk[hh] >= kstar) ? fmaxf(vm, cvv[jj]) : vm;
      }
#if DVCP_FPS_RECERT
      // ---- 5b. the second pass: the first pass stops at the first candidate whose order it cannot
      // certify, usually one its accepted centres moved.  The candidates left, with their values
      // after those centres (the update's formula: exactly the points' minima after this round's
      // first pass), are ranked and tested again under the same T -- rank 0 of them is the next
      // step's argmax (above T, hence above every unlisted point) -- so one round accepts more
      // centres for one more pair pass.  (Not for layer 3 of the paired launch: its tie handling
      // ranks by layer 2's pick numbers.)
      if constexpr (MODE == 0 || MODE == 1 || MODE == 3) {
        const bool may = MODE != 1 || !consumer;
        if (may && kstar < nreal && kstar < kSelAccept && kstar < npoint - step) {  // (uniform)
          koff = kstar;
          {  // thread t: candidate t % 128 against centres t / 128, + THREADS / 128, ...
            // (the thread index re-materialised: hoisted out of the round loop, the addresses below
            // stayed live in VGPRs and spilled)
            constexpr int G = THREADS / kSelMax;
            const int t = wave * kWave + fresh_lane();
            const int j = t % kSelMax;
            float m = cvv[j];
            const T qx = cxx[j], qy = cyy[j], qz = czz[j];
            for (int i = t / kSelMax; i < koff; i += G) {  // (acc4: this wave's own rows)
#if DVCP_FPS_ACC4
              const AccC c = acc4[i];
              m = fps_update<T>(m, qx, qy, qz, c.x, c.y, c.z);
#else
              m = fps_update<T>(m, qx, qy, qz, acx[i], acy[i], acz[i]);
#endif
            }
            vpart[t] = m;
          }
          lds_barrier();
          int n2 = 0;
          const int ln2 = fresh_lane();
          [[maybe_unused]] float vmd = 0.0f;  // MODE 3: this part's candidates dropped at or below T
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int jj = hh * 64 + ln2;
            float v2 = -1.0f;  // (no candidate: unused slots, beyond the list, accepted)
            if (jj < cnt && rk[hh] != 0x7FFFFFFF && rk[hh] >= koff) {
              v2 = vpart[jj];
#pragma unroll
              for (int g = 1; g < THREADS / kSelMax; ++g) v2 = fminf(v2, vpart[g * kSelMax + jj]);
            }
            const uint64_t m = __ballot(v2 > Tb);
            if constexpr (MODE == 3) {
              // compacted in list order (every wave writes the same rows of the c2 arrays, which
              // no wave reads before its own writes): the merged list's unused slots and the
              // dropped candidates leave the pair pass
              if (v2 > Tb) {
                const int o = n2 + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                       static_cast<uint32_t>(m >> 32),
                                       __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0)));
                cvv2[o] = v2;
                c2pid[o] = cpid[jj];
                c2x[o] = cxx[jj];
                c2y[o] = cyy[jj];
                c2z[o] = czz[jj];
                c2slot[o] = jj;
              }
              const bool mine = jj >= cbase && jj < cbase + capw;
              vmd = mine && !(v2 > Tb) ? fmaxf(vmd, v2) : vmd;
            } else {
              cvv2[jj] = v2;
            }
            n2 += __popcll(m);
          }
          nreal2 = n2;
          if (n2 > 0) {  // (uniform: every wave computed every value)
            rank_decide(std::true_type{});
            if constexpr (MODE == 3) {
              accept(koff, std::true_type{});
              vm = fmaxf(Tw, vmd);
#pragma unroll
              for (int hh = 0; hh < 2; ++hh) {
                const int o = hh * 64 + lane;
                if (o < n2 && rk[hh] >= kstar) {
                  const int jj = c2slot[o];
                  vm = jj >= cbase && jj < cbase + capw ? fmaxf(vm, cvv2[o]) : vm;
                }
              }
            } else {
              accept(koff, std::false_type{});
              vm = Tb;
#pragma unroll
              for (int hh = 0; hh < 2; ++hh) {
                const int jj = hh * 64 + lane;
                vm = (jj < cnt && rk[hh] >= kstar) ? fmaxf(vm, cvv2[jj]) : vm;
              }
            }
            kstar += koff;
          }
        }
      }
#endif
      vmax = wave_fmax_clamp0(vm);
      tick(3);
      break;
    }
    if constexpr (MODE == 3) {
      if (part_quit) break;
    }
    // ---- the update: apply the accepted centres ----------------------------------------------
    tick(-1);
    // Lane l tests its group l % GP against centre c0 + l / GP: QC (centre, group) pairs per group
    // lane and wave instruction (one centre per instruction left 64 - PPT lanes idle, and the
    // update was bound by those box tests: 16 waves x ~26 centres per round on 4 SIMDs).
    const int lane = fresh_lane();
    uint32_t dirty = 0u;
    T gbl[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) gbl[a] = gbox[wave][a][lane & (GP - 1)];
    for (int c0 = 0; c0 < kstar; c0 += QC) {
      const int cq = c0 + static_cast<int>(static_cast<unsigned>(lane) / GP);
      const int ci = cq < kstar ? cq : kstar - 1;
#if DVCP_FPS_ACC4
      const AccC cc = acc4[ci];
      const T cx = cc.x, cy = cc.y, cz = cc.z;
#else
      const T cx = acx[ci], cy = acy[ci], cz = acz[ci];
#endif
      uint64_t m = __ballot(cq < kstar && grp && !(box_lb2(cx, cy, cz, gbl) >= static_cast<T>(gub)));
      // (Round 5, tools/fps_lab A/B, profiles/round5/r5bb_fps_updgrp.log: taking each slot's pairs of
      // the batch together -- one indexed read and write of the slot for all its centres -- ran
      // 5.23 -> 5.45 ms (16384 -> 10000) and 3.25 -> 3.32 ms (10000): few pairs share a slot.)
      while (m) {  // touched (centre, slot) pairs; p is wave-uniform -> indexed register access
        const int k = __ffsll(static_cast<long long>(m)) - 1;
        m &= m - 1;
        const int p = k & (GP - 1);
        dirty |= 1u << p;
#if DVCP_FPS_ACC4
        const AccC sc = acc4[c0 + k / GP];  // (a broadcast LDS read: the LDS pipe instead of three readlanes)
        dmin[p] = fps_update<T>(dmin[p], px[p], py[p], pz[p], sc.x, sc.y, sc.z);
#else
        const T sx = readlane_t(cx, k), sy = readlane_t(cy, k), sz = readlane_t(cz, k);
        dmin[p] = fps_update<T>(dmin[p], px[p], py[p], pz[p], sx, sy, sz);
#endif
      }
    }
    // re-reduce the touched groups whose maximum point dropped (values only drop: a group keeps
    // its maximum while some point still holds it)
    while (dirty) {
      const int p = __ffs(dirty) - 1;
      dirty &= dirty - 1;
      const float gp = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gub), p));
      if (!__ballot(dmin[p] == gp)) {
        const float gm = wave_fmax_clamp0(dmin[p]);
        gub = (lane & (GP - 1)) == p ? gm : gub;
      }
    }
    tick(4);
    step += kstar;
  }
  if constexpr (MODE == 3) {
    if (part_quit) {  // gave up waiting for a peer: raise err; the remaining outputs repeat the start point
      if (tid == 0) __hip_atomic_fetch_or(qa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (part == 0) {
        int64_t first = start[b];
        if (first < 0 || first >= N) first = 0;
        const T fx = pts.at(b, 0, first), fy = pts.at(b, 1, first), fz = pts.at(b, 2, first);
        for (int k = step + tid; k < npoint; k += THREADS) {
          oi[k] = first;
          if (ox) {
            ox[k] = fx;
            ox[npoint + k] = fy;
            ox[2 * npoint + k] = fz;
          }
        }
      }
    }
  }
  if constexpr (MODE == 1) {
    if (tied && tid == 0) __hip_atomic_fetch_or(pa.flag + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if DVCP_FPS_PAIR_DIAG == 3
    if (consumer && tid == 0) pa.slot[b] = static_cast<uint32_t>(n_repair) | (static_cast<uint32_t>(min(rep_clk >> 10, uint64_t(0xFFFFFF))) << 8);
#endif
  }
  if constexpr (TIMING) {
    if (prof && lane == 0) {  // per wave: [rounds, scans, fallbacks, clk: scan, decide+list, rank, prefix, update]
      unsigned long long* o = prof + ((static_cast<int64_t>(b) * S + part) * W + wave) * kFpsProf;
      o[0] = n_round;
      o[1] = n_scan;
      o[2] = n_fallback;
      for (int k = 0; k < 5; ++k) o[3 + k] = ph[k];
      for (int k = 0; k < 4; ++k) o[8 + k] = why[k];
      o[12] = ph[5];
    }
  }
}

template <typename T, int PPT, bool TIMING = false, int THREADS = kFpsThreads>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(fps_select_waves_per_eu<PPT, THREADS>())))
void fps_select_kernel(PointsView<T> pts, int N, int npoint, const int64_t* __restrict__ start,
                       int64_t* __restrict__ out_idx, T* __restrict__ out_xyz,
                       unsigned long long* __restrict__ prof) {
#if DVCP_FPS_PRIO
  __builtin_amdgcn_s_setprio(DVCP_FPS_PRIO);  // (A/B: issue priority over co-resident waves)
#endif
  fps_select_body<T, PPT, TIMING, THREADS, 0>(pts, N, npoint, start, out_idx, out_xyz, prof, FpsPairArgs<T>{});
}

// Split select (FpsPartArgs): grid ceil(B / 8) * 8 * S, THREADS threads, PPT groups per lane
// slot of a part's share of the cloud.
// TIMING (tools/fps_lab): per-wave round clocks of every part, prof[((b S + part) W + wave) kFpsProf].
template <int PPT, int THREADS, bool TIMING = false>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(THREADS / 256)))
void fps_part_kernel(PointsView<float> pts, int N, int npoint, const int64_t* __restrict__ start,
                     int64_t* __restrict__ out_idx, float* __restrict__ out_xyz, FpsPartArgs qa,
                     unsigned long long* __restrict__ prof) {
  fps_select_body<float, PPT, TIMING, THREADS, 3>(pts, N, npoint, start, out_idx, out_xyz, prof,
                                                  FpsPairArgs<float>{}, qa);
}

// grid 2B: layer 2 (out_idx / out_xyz, start) and layer 3 (pa) of B clouds, see FpsPairArgs.
// (Up to 128 VGPRs: at the select kernel's 96 the tie re-ranking loop spilled 72 B.)
template <typename T, int PPT>
__global__ __launch_bounds__(kFpsSel1024) __attribute__((amdgpu_waves_per_eu(4)))
void fps_pair_kernel(PointsView<T> pts, int N, const int64_t* __restrict__ start, int64_t* __restrict__ out_idx,
                     T* __restrict__ out_xyz, FpsPairArgs<T> pa) {
  fps_select_body<T, PPT, false, kFpsSel1024, 1>(pts, N, N, start, out_idx, out_xyz, nullptr, pa);
}

// grid B: layer 3 in the reference's order for the clouds whose pair flag is set
template <typename T, int PPT>
__global__ __launch_bounds__(kFpsSel1024) __attribute__((amdgpu_waves_per_eu(fps_select_waves_per_eu<PPT, kFpsSel1024>())))
void fps_select_gated_kernel(PointsView<T> pts, int N, const int64_t* __restrict__ start, int64_t* __restrict__ out_idx,
                             T* __restrict__ out_xyz, FpsPairArgs<T> pa) {
  fps_select_body<T, PPT, false, kFpsSel1024, 2>(pts, N, N, start, out_idx, out_xyz, nullptr, pa);
}

// grid B: layer 3's indices (into layer 2's points) -> layer 2's pick numbers (its FPS order), for
// the clouds without a flag (layer 2 then picked every point once).  A tie group (a run of entries
// marked by bit 62 after its first) is put in ascending pick-number order -- the reference's
// lowest-index-first argmax among equal values -- with its centres' coordinates.
constexpr int kFpsRemapThreads = 1024;
__global__ __launch_bounds__(kFpsRemapThreads) void fps_pair_remap_kernel(const uint32_t* __restrict__ inv2,
                                                                          int64_t* __restrict__ idx3,
                                                                          float* __restrict__ xyz3,
                                                                          const int32_t* __restrict__ flag, int N) {
  const int b = blockIdx.x;
  if (flag[b] != 0) return;
  constexpr int64_t kMark = int64_t(1) << 62;
  const uint32_t* inv = inv2 + static_cast<int64_t>(b) * N;
  int64_t* i3 = idx3 + static_cast<int64_t>(b) * N;
  float* x3 = xyz3 + static_cast<int64_t>(b) * 3 * N;
  auto key_of = [&](int64_t v) -> int64_t {
    const int64_t n = v & ~kMark;
    return (n >= 0 && n < N) ? static_cast<int64_t>(inv[n] & 0x7FFFFFFFu) : 0;
  };
  __shared__ uint32_t marks[16384 / 32];  // the marks as written, before any entry is rewritten
  for (int w = threadIdx.x; w < (N + 31) / 32; w += kFpsRemapThreads) marks[w] = 0u;
  __syncthreads();
  for (int j = threadIdx.x; j < N; j += kFpsRemapThreads)
    if (i3[j] & kMark) atomicOr(&marks[j >> 5], 1u << (j & 31));
  __syncthreads();
  auto marked = [&](int j) { return (marks[j >> 5] >> (j & 31)) & 1u; };
  for (int j = threadIdx.x; j < N; j += kFpsRemapThreads) {
    if (marked(j)) continue;  // written by its group's first entry
    const int64_t v = i3[j];
    int e = j;
    while (e + 1 < N && marked(e + 1)) ++e;
    if (e == j) {
      i3[j] = key_of(v);
      continue;
    }
    // group j..e (at most kSelAccept entries): selection sort by pick number, in place
    for (int p = j; p <= e; ++p) {
      int best = p;
      int64_t kb = key_of(i3[p]);
      for (int q = p + 1; q <= e; ++q) {
        const int64_t kq = key_of(i3[q]);
        if (kq < kb) {
          kb = kq;
          best = q;
        }
      }
      const int64_t vp = i3[p];
      i3[best] = vp;  // (an unresolved member: its raw index)
      i3[p] = kb;     // resolved
      for (int a = 0; a < 3; ++a) {
        const float t = x3[a * N + best];
        x3[a * N + best] = x3[a * N + p];
        x3[a * N + p] = t;
      }
    }
  }
}

// Step floor of the FPS chain (bench.py's latency roofline): fps_kernel's per-step
// synchronisation with no point work -- each wave's 64-lane DPP argmax + ballot, one LDS slot per
// wave, one barrier, the W-slot DPP reduction and readlanes -- each step's value depending on the
// previous step's winner, so the steps form one dependent chain as in FPS.
template <int W>
__global__ __launch_bounds__(W * kWave) void fps_floor_kernel(int steps, float* __restrict__ out) {
  __shared__ FpsSlot<float> slots[2][W];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float base = static_cast<float>(lane * 7 % 64) + 64.0f * static_cast<float>(wave * 3 % W);
  int cur = 0;
  for (int step = 0; step < steps; ++step) {
    const float bv = base + static_cast<float>(cur & 1) * 0.5f;
    const float wv = wave_maxf_dpp(bv);
    const uint64_t tied = __ballot(bv == wv);
    const int wl = __ffsll(static_cast<long long>(tied)) - 1;
    FpsSlot<float>* buf = slots[step & 1];
    if (lane == 0) buf[wave] = FpsSlot<float>{wv, wave * kWave + wl, 0.f, 0.f, 0.f};
    lds_barrier();
    const FpsSlot<float> mine = buf[lane & (W - 1)];
    float v = mine.v;
    if constexpr (W > 1) v = dpp_maxf<0x111, 0x1>(v);
    if constexpr (W > 2) v = dpp_maxf<0x112, 0x1>(v);
    if constexpr (W > 4) v = dpp_maxf<0x114, 0x1>(v);
    if constexpr (W > 8) v = dpp_maxf<0x118, 0x1>(v);
    const float gv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), W - 1));
    const int ws = __ffsll(static_cast<long long>(__ballot((lane < W) & (mine.v == gv)))) - 1;
    cur = __builtin_amdgcn_readlane(mine.i, ws) + step;
  }
  if (tid == 0) out[blockIdx.x] = static_cast<float>(cur);
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

// Split FPS for clouds above one CU's register budget (C5: 65536 points): S workgroups per cloud,
// each holding a contiguous chunk of P * NT points (coordinates and running minima in VGPRs, 512
// threads, P = 16 points per lane, or 32 for fp32 clouds above 131072 points).  Every step each workgroup updates its
// minima with the current centre and publishes its best point as one 64-bit key: the fp32 minimum's
// bits (monotonic for values >= 0), then the complemented index (18 bits), then the step's 14-bit
// tag -- so among one step's keys the maximum is the largest minimum with the lowest index, the
// dense kernel's and the reference's argmax rule.  Wave 0 of every workgroup then polls the cloud's
// S key slots, one lane per slot, until all carry this step's tag, and takes their maximum: one
// L2 round trip per poll, no arrival counter (round 4: the counter's release/acquire round trip
// plus a separate read of the keys made a step ~3.6 us).  Slots are double-buffered by step parity:
// a workgroup can only publish step + 2 after every peer has published step + 1, i.e. after every
// peer read step's keys; the slots start invalid (all ones: no minimum has those bits).
//
// Progress does not rest on the whole grid being co-resident.  A workgroup takes its (cloud,
// chunk) from a ticket counter when it starts running, not from blockIdx, so the tickets handed
// out so far cover whole clouds plus at most one partly started cloud per launch: a waiting
// workgroup only ever waits for peers of that one cloud, which take the next free slots on the
// device (S - 1 slots per concurrent launch).  The wait is still bounded (spin_cap polls) as a
// guard: a workgroup that gives up raises the launch's error word, which the host checks
// (dvcp/_lib.py check_device_flags), and writes the start point (index and coordinates) for the
// steps it could not finish, so nothing downstream reads out of bounds or a garbage centre.
constexpr int kFpsSplitMax = 16;
constexpr uint32_t kFpsSpinCap = 1u << 22;
constexpr int kSplitTagBits = 14, kSplitIdxBits = 18;  // N <= 16 x 16384 points per cloud
constexpr uint64_t kSplitTagMask = (1ull << kSplitTagBits) - 1;
constexpr uint32_t kSplitIdxMask = (1u << kSplitIdxBits) - 1;

constexpr int kFpsSplitThreads = 512;  // (1024 threads x 16 points spilled 840 B at 128 VGPRs)
// Points per lane: 16 (chunks of 8192 points: twice the workgroups, half the per-step update)
// while that needs at most kFpsSplitMax workgroups per cloud; fp32 clouds above 131072 points take
// chunks of 16384.  (Chunks of 4096 ran one C5 launch in 19.4 instead of 22.3 ms, but with ten
// batches in flight their spinning workgroups cost the C5 bench 367.7 -> 288.5 pairs/s.)
template <typename T>
inline int fps_split_ppt(int N) {
  return sizeof(T) == 4 && ceil_div(N, 16 * kFpsSplitThreads) > kFpsSplitMax ? 32 : 16;
}
template <typename T>
constexpr int fps_split_max_chunk() { return (sizeof(T) == 4 ? 32 : 16) * kFpsSplitThreads; }

template <typename T, int P, int NT>
__global__ __launch_bounds__(NT) void fps_split_kernel(PointsView<T> pts, int N, int npoint, int S,
                                                       const int64_t* __restrict__ start,
                                                       int64_t* __restrict__ out_idx, T* __restrict__ out_xyz,
                                                       uint64_t* __restrict__ keys, uint32_t* __restrict__ ticket,
                                                       int32_t* __restrict__ err, uint32_t spin_cap) {
  constexpr int kW = NT / kWave;
  constexpr int chunk = P * NT;
  __shared__ uint64_t wbest[kW];
  __shared__ uint64_t gbest;
  __shared__ int timed_out;
  __shared__ uint32_t my_ticket;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    my_ticket = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    timed_out = 0;
  }
  __syncthreads();
  const int b = static_cast<int>(my_ticket) / S, s = static_cast<int>(my_ticket) % S;
  const int n0 = s * chunk, n1 = min(N, n0 + chunk);
  T px[P], py[P], pz[P];
  float dm[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int n = n0 + p * NT + tid;
    const bool ok = n < n1;
    px[p] = ok ? pts.at(b, 0, n) : static_cast<T>(0);
    py[p] = ok ? pts.at(b, 1, n) : static_cast<T>(0);
    pz[p] = ok ? pts.at(b, 2, n) : static_cast<T>(0);
    dm[p] = 1e10f;
  }
  int64_t first = start[b];
  if (first < 0 || first >= N) first = 0;
  int64_t cur = first;
  T cx = pts.at(b, 0, cur), cy = pts.at(b, 1, cur), cz = pts.at(b, 2, cur);
  uint64_t* kb = keys + static_cast<int64_t>(b) * 2 * S;
  int step = 0;
  for (; step < npoint; ++step) {
    if (s == 0 && tid == 0) {
      out_idx[static_cast<int64_t>(b) * npoint + step] = cur;
      if (out_xyz) {
        T* ox = out_xyz + static_cast<int64_t>(b) * 3 * npoint;
        ox[step] = cx;
        ox[npoint + step] = cy;
        ox[2 * npoint + step] = cz;
      }
    }
    uint64_t best = 0;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int n = n0 + p * NT + tid;
      const T dx = px[p] - cx, dy = py[p] - cy, dz = pz[p] - cz;
      const T d = (dx * dx + dy * dy) + dz * dz;
      float m = dm[p];
      if (d < static_cast<T>(m)) m = static_cast<float>(d);
      dm[p] = m;
      const uint64_t key = (static_cast<uint64_t>(__float_as_uint(m)) << 32) |
                           (static_cast<uint64_t>(kSplitIdxMask - static_cast<uint32_t>(n)) << kSplitTagBits);
      best = (n < n1 && key > best) ? key : best;
    }
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t o = __shfl_xor(best, off, kWave);
      best = o > best ? o : best;
    }
    if (lane == 0) wbest[wave] = best;
    __syncthreads();
    if (wave == 0) {
      const uint64_t tag = static_cast<uint64_t>(step) & kSplitTagMask;
      uint64_t* slot = kb + (step & 1) * S;
      if (lane == 0) {
        uint64_t wb = wbest[0];
        for (int w = 1; w < kW; ++w) wb = wbest[w] > wb ? wbest[w] : wb;
        __hip_atomic_store(slot + s, wb | tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      uint64_t v = 0;
      uint32_t polls = 0;
      for (;;) {
        v = lane < S ? __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const bool ok = lane >= S || ((v & kSplitTagMask) == tag && static_cast<uint32_t>(v >> 32) != 0xFFFFFFFFu);
        if (__ballot(!ok) == 0) break;
        __builtin_amdgcn_s_sleep(1);
        if (++polls > spin_cap) {
          if (lane == 0) timed_out = 1;
          break;
        }
      }
      uint64_t g = lane < S ? v : 0ull;
      for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(g, off, kWave);
        g = o > g ? o : g;
      }
      if (lane == 0) gbest = g;
    }
    __syncthreads();
    if (timed_out) break;
    cur = static_cast<int64_t>(kSplitIdxMask - static_cast<uint32_t>((gbest >> kSplitTagBits) & kSplitIdxMask));
    cx = pts.at(b, 0, cur);
    cy = pts.at(b, 1, cur);
    cz = pts.at(b, 2, cur);
    __syncthreads();  // gbest / wbest are rewritten next step
  }
  if (step < npoint) {  // gave up waiting: flag the launch, keep every index and centre valid
    if (tid == 0) __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 0) {
      // the remaining steps repeat the start point: in-range indices AND finite centres, so the
      // ball query / MLP launched behind this one read real points before the host raises
      const T fx = pts.at(b, 0, first), fy = pts.at(b, 1, first), fz = pts.at(b, 2, first);
      T* ox = out_xyz ? out_xyz + static_cast<int64_t>(b) * 3 * npoint : nullptr;
      for (int k = step + tid; k < npoint; k += NT) {
        out_idx[static_cast<int64_t>(b) * npoint + k] = first;
        if (ox) {
          ox[k] = fx;
          ox[npoint + k] = fy;
          ox[2 * npoint + k] = fz;
        }
      }
    }
  }
}

// Workspace of the split kernel, carved from the caller's B x N fp32 buffer (>= 64 KiB per cloud):
// keys [B][2][S] u64 | ticket u32 | err i32 (err is the caller's when given).
struct FpsSplitWs {
  uint64_t* keys;
  uint32_t* ticket;
  int32_t* err;
};
static FpsSplitWs fps_split_ws(float* ws, int B, int S) {
  FpsSplitWs w;
  w.keys = reinterpret_cast<uint64_t*>(ws);
  w.ticket = reinterpret_cast<uint32_t*>(w.keys + static_cast<int64_t>(B) * 2 * S);
  w.err = reinterpret_cast<int32_t*>(w.ticket + 1);
  return w;
}

// Launch the split kernel over B clouds; `withhold` > 0 (tests only) launches that many fewer
// workgroups, so the last cloud never completes and its workgroups must give up.
template <typename T>
static int launch_fps_split(PointsView<T> v, int B, int N, int npoint, const int64_t* start, int64_t* out_idx,
                            T* out_xyz, float* ws, int32_t* err, uint32_t spin_cap, int withhold, hipStream_t st) {
  constexpr int NT = kFpsSplitThreads;
  const int P = fps_split_ppt<T>(N);
  const int S = ceil_div(N, P * NT);
  if (N > S * P * NT || N - 1 > static_cast<int>(kSplitIdxMask)) {
    set_error("dvcp_fps(split): N=%d too large", N);
    return DVCP_EINVAL;
  }
  FpsSplitWs w = fps_split_ws(ws, B, S);
  hipError_t e = hipMemsetAsync(w.keys, 0xFF, sizeof(uint64_t) * 2 * static_cast<size_t>(B) * S, st);  // invalid
  if (e == hipSuccess) e = hipMemsetAsync(w.ticket, 0, sizeof(uint32_t) * 2, st);
  if (e != hipSuccess) return launch_status("dvcp_fps(split memset)");
  if (!err) err = w.err;
  const int grid = B * S - withhold;
  if (grid > 0) {
    if (P == 16)
      hipLaunchKernelGGL((fps_split_kernel<T, 16, NT>), dim3(grid), dim3(NT), 0, st, v, N, npoint, S, start, out_idx,
                         out_xyz, w.keys, w.ticket, err, spin_cap);
    else if constexpr (sizeof(T) == 4)
      hipLaunchKernelGGL((fps_split_kernel<T, 32, NT>), dim3(grid), dim3(NT), 0, st, v, N, npoint, S, start, out_idx,
                         out_xyz, w.keys, w.ticket, err, spin_cap);
  }
  return launch_status("dvcp_fps(split)");
}

// Workgroups per cloud of the select rounds when the caller does not choose (dvcp_fps_ws, parts 0):
// 8 above 16384 points, else one, unless DVCP_FPS_PARTS asks for the split select (2, 4 or 8).
// The split select shortens a lone batch's chain but costs CU time: S full-CU workgroups per
// cloud for 1 / 1.3 / 1.6 the time at S = 2 / 4 / 8 (C3), so with the bench's ten batches in
// flight the one-workgroup kernel gives the most pairs/s (round 6: 2300 against 1630 at S = 4 and
// 1310 at S = 8).  Above 16384 points the alternative is the per-step split kernel, slower still.
// DVCP_FPS_PART_THREADS sets its workgroup size (256, 512 or 1024; A/B runs).
static int fps_env_int(const char* name, int dflt) {
  const char* s = getenv(name);
  return s && *s ? atoi(s) : dflt;
}
static int fps_parts(int N) {
  static const int forced = fps_env_int("DVCP_FPS_PARTS", 0);
  if (forced == 1 || forced == 2 || forced == 4 || forced == 8) return forced;
  // above the one-workgroup kernel's 16384 points: 8 workgroups of up to 8192 (C5's layer 1,
  // 65536 -> 10000: 9.65 ms per launch with the per-step split kernel, 4.4 ms split select)
  return N > 16 * kFpsSel1024 ? 8 : 1;
}

// Launch the split select over B fp32 clouds with S workgroups each; returns 1 (nothing launched)
// when the workspace or the instantiated point slots do not cover this (N, S).
// Workspace of the split select, carved from the caller's buffer: slots [B][2][S][slot] u64 |
// flags [B] u32 + the ticket u32 (padded to 8 bytes) | perm [B][N] u32 | err i32.  The slots,
// flags and ticket are set to all ones per launch.
struct FpsPartWs {
  int64_t slot_bytes, flag_bytes, total;
};
static FpsPartWs fps_part_ws(int B, int N, int S) {
  // a part's slot as fps_select_body lays it out (slotsz there): header, per-wave T, candidates
  const int64_t slotsz = kPartHdr + kPartMaxWaves + 5 * (kSelMax / S);
  FpsPartWs w;
  w.slot_bytes = static_cast<int64_t>(B) * 2 * S * slotsz * 8;
  w.flag_bytes = (static_cast<int64_t>(B) * 4 + 4 + 7) / 8 * 8;  // B flags, the ticket
  w.total = w.slot_bytes + w.flag_bytes + static_cast<int64_t>(B) * N * 4 + 8;
  return w;
}
static int64_t fps_workspace_bytes(int B, int N) {  // the split path's B x N fp32, or the split select's
  int64_t need = static_cast<int64_t>(B) * N * 4;
  for (int S = 2; S <= 8; S *= 2) {
    const int64_t t = fps_part_ws(B, N, S).total;
    need = t > need ? t : need;
  }
  return need;
}

static int launch_fps_part(PointsView<float> v, int B, int N, int npoint, const int64_t* start, int64_t* out_idx,
                           float* out_xyz, float* ws, int64_t ws_bytes, int32_t* err, int S, hipStream_t st) {
  static const int threads = fps_env_int("DVCP_FPS_PART_THREADS", 1024);
  const FpsPartWs w = fps_part_ws(B, N, S);
  if (w.total > ws_bytes || N > kPartMaxN) return 1;
  if (threads / kWave > kPartMaxWaves) return 1;
  uint64_t* slots = reinterpret_cast<uint64_t*>(ws);
  uint32_t* flags = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws) + w.slot_bytes);
  uint32_t* permw = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws) + w.slot_bytes + w.flag_bytes);
  if (!err) err = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(ws) + w.total - 8);
  if (hipMemsetAsync(slots, 0xFF, static_cast<size_t>(w.slot_bytes + w.flag_bytes), st) != hipSuccess)
    return launch_status("dvcp_fps(part memset)");
  static const int target = fps_env_int("DVCP_FPS_PART_TARGET", 0);
  static const bool tickets = fps_env_int("DVCP_FPS_PART_TICKET", 1) != 0;
  const FpsPartArgs qa{slots, flags, permw, err, S, B, N, kFpsSpinCap, target, tickets ? flags + B : nullptr};
  const dim3 grid(tickets ? B * S : ceil_div(B, 8) * 8 * S);
  const int groups = ceil_div(ceil_div(N, kWave), S);  // 64-point groups per part (at most)
#define DVCP_FPS_PART(P, NT)                                                                                  \
  if (threads == NT && groups <= P * (NT / kWave)) {                                                          \
    hipLaunchKernelGGL((fps_part_kernel<P, NT>), grid, dim3(NT), 0, st, v, N, npoint, start, out_idx, out_xyz, qa, \
                       nullptr);                                                                              \
    return launch_status("dvcp_fps(part)");                                                                   \
  }
  DVCP_FPS_PART(2, 1024)
  DVCP_FPS_PART(4, 1024)
  DVCP_FPS_PART(8, 1024)
  DVCP_FPS_PART(4, 512)
  DVCP_FPS_PART(8, 512)
  DVCP_FPS_PART(8, 256)
  DVCP_FPS_PART(16, 256)
#undef DVCP_FPS_PART
  return 1;
}

template <typename T>
static int launch_fps(const T* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                      const int64_t* start, int64_t* out_idx, T* out_xyz, float* ws, int32_t* err, hipStream_t st,
                      int parts = 0, int64_t ws_bytes = -1) {
  if (ws_bytes < 0) ws_bytes = ws ? static_cast<int64_t>(B) * N * 4 : 0;  // dvcp_fps_ws's B x N fp32
  PointsView<T> v{xyz, sb, sc, sn};
  const int ppt = ceil_div(N, kFpsThreads);
  dim3 grid(B), block(kFpsThreads);
  // fp32 clouds of 2048..16384 points with a workspace: the split select, S workgroups per cloud
  if constexpr (sizeof(T) == 4) {
    if (ws && N >= kFpsBatchedMinN && N <= kPartMaxN && npoint > 1) {
      const int S = parts > 0 ? parts : fps_parts(N);  // (parts 1: the one-workgroup kernel below)
      if (S > 1) {
        const int e = launch_fps_part(v, B, N, npoint, start, out_idx, out_xyz, ws, ws_bytes, err, S, st);
        if (e != 1) return e;
      }
    }
  }
  // fp32 clouds of 2048..16384 points: the select kernel with 1024 threads (16 waves, 4 per SIMD,
  // up to 16 points per lane): per-wave scan and update halve while the per-round decisions stay
  // (tools/fps_lab: 16384 -> 10000 5.52 -> 5.07 ms, 10000 -> 10000 4.13 -> 3.30 ms on 16 clouds)
  if constexpr (sizeof(T) == 4) {
    // DVCP_FPS_THREADS=512 (A/B runs): the 512-thread select below instead
    static const bool sel1024 = fps_env_int("DVCP_FPS_THREADS", 1024) != 512;
    if (sel1024 && N >= kFpsBatchedMinN && N <= 16 * kFpsSel1024) {
      const int p16 = ceil_div(N, kFpsSel1024);
      const dim3 blk(kFpsSel1024);
#define DVCP_FPS_SEL1024(P)                                                                                   \
  if (p16 <= P) {                                                                                             \
    hipLaunchKernelGGL((fps_select_kernel<T, P, false, kFpsSel1024>), grid, blk, 0, st, v, N, npoint, start,    \
                       out_idx, out_xyz, nullptr);                                                            \
    return launch_status("dvcp_fps");                                                                         \
  }
      DVCP_FPS_SEL1024(2)
      DVCP_FPS_SEL1024(4)
      DVCP_FPS_SEL1024(8)
      DVCP_FPS_SEL1024(10)
      DVCP_FPS_SEL1024(16)
#undef DVCP_FPS_SEL1024
    }
  }
  // threshold-select kernel from 2048 points; below, the one-centre-per-step kernel (box-pruned)
#define DVCP_FPS_CASE(P)                                                                                   \
  if (ppt <= P) {                                                                                          \
    if (N >= kFpsBatchedMinN)                                                                              \
      hipLaunchKernelGGL((fps_select_kernel<T, P>), grid, block, 0, st, v, N, npoint, start, out_idx, out_xyz, \
                         nullptr);                                                                         \
    else                                                                                                   \
      hipLaunchKernelGGL((fps_kernel<T, kFpsThreads, P, true>), grid, block, 0, st, v, N, npoint, start,        \
                         out_idx, out_xyz, nullptr);                                                       \
    return launch_status("dvcp_fps");                                                                      \
  }
  DVCP_FPS_CASE(2)
  DVCP_FPS_CASE(4)
  DVCP_FPS_CASE(8)
  DVCP_FPS_CASE(16)
  if constexpr (sizeof(T) == 4) {
    DVCP_FPS_CASE(20)  // N = 10000 (the FE layers 2 and 3): no all-padding slots per lane
    DVCP_FPS_CASE(24)
    DVCP_FPS_CASE(32)
  }
#undef DVCP_FPS_CASE
  if (!ws) {
    set_error("dvcp_fps: N=%d needs the split/dense path and its B x N fp32 workspace (dvcp_fps_ws)", N);
    return DVCP_EINVAL;
  }
  if (ceil_div(N, fps_split_max_chunk<T>()) <= kFpsSplitMax)
    return launch_fps_split<T>(v, B, N, npoint, start, out_idx, out_xyz, ws, err, kFpsSpinCap, 0, st);
  hipLaunchKernelGGL((fps_dense_kernel<T>), grid, block, 0, st, v, N, npoint, start, out_idx, out_xyz, ws);
  return launch_status("dvcp_fps(dense)");
}

// Paired launch of two full-permutation fp32 layers (see FpsPairArgs); N in the select kernel's
// 1024-thread range.
static int launch_fps_pair(PointsView<float> v, int B, int N, const int64_t* start2, const int64_t* start3,
                           int64_t* idx2, float* xyz2, int64_t* idx3, float* xyz3, uint32_t* ws, hipStream_t st) {
  // ws: ticket | slot[B] | flag[B] | inv2[B x N], all zero before the launch
  FpsPairArgs<float> pa{ws, ws + 1, reinterpret_cast<int32_t*>(ws + 1 + B), ws + 1 + 2 * static_cast<int64_t>(B),
                        start3, idx3, xyz3};
  if (hipMemsetAsync(ws, 0, sizeof(uint32_t) * (1 + 2 * static_cast<size_t>(B) + static_cast<size_t>(B) * N), st) !=
      hipSuccess)
    return launch_status("dvcp_fps_pair(memset)");
  const PointsView<float> v2{xyz2, 3 * static_cast<int64_t>(N), N, 1};
  const int p16 = ceil_div(N, kFpsSel1024);
#define DVCP_FPS_PAIR(P)                                                                                        \
  if (p16 <= P) {                                                                                               \
    hipLaunchKernelGGL((fps_pair_kernel<float, P>), dim3(2 * B), dim3(kFpsSel1024), 0, st, v, N, start2, idx2,   \
                       xyz2, pa);                                                                               \
    if (int e = launch_status("dvcp_fps_pair")) return e;                                                       \
    hipLaunchKernelGGL(fps_pair_remap_kernel, dim3(B), dim3(kFpsRemapThreads), 0, st, pa.inv2, idx3, xyz3, pa.flag, \
                       N);                                                                                      \
    if (int e = launch_status("dvcp_fps_pair(remap)")) return e;                                                \
    hipLaunchKernelGGL((fps_select_gated_kernel<float, P>), dim3(B), dim3(kFpsSel1024), 0, st, v2, N, start3,    \
                       idx3, xyz3, pa);                                                                         \
    return launch_status("dvcp_fps_pair(gated)");                                                               \
  }
  DVCP_FPS_PAIR(2)
  DVCP_FPS_PAIR(4)
  DVCP_FPS_PAIR(8)
  DVCP_FPS_PAIR(10)
  DVCP_FPS_PAIR(16)
#undef DVCP_FPS_PAIR
  set_error("dvcp_fps_pair: N=%d out of range", N);
  return DVCP_EINVAL;
}

}  // namespace dvcp

// Two chained full-permutation FPS layers in one launch (FE layers 2 and 3): bit-identical to
//   dvcp_fps(xyz, N, start2) -> (idx2, xyz2);  dvcp_fps(xyz2, N, start3) -> (idx3, xyz3).
// fp32, 2048 <= N <= 16384; ws: dvcp_fps_pair_workspace_bytes(B, N) bytes, 4-byte aligned.
extern "C" int64_t dvcp_fps_pair_workspace_bytes(int B, int N) {
  return B < 0 || N < 0 ? -1 : 4 * (1 + 2 * static_cast<int64_t>(B) + static_cast<int64_t>(B) * N);
}

extern "C" int dvcp_fps_pair(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                             const int64_t* start2, const int64_t* start3, int64_t* idx2, void* xyz2, int64_t* idx3,
                             void* xyz3, void* ws, void* stream) {
  DVCP_REQUIRE(xyz && start2 && start3 && idx2 && xyz2 && idx3 && xyz3 && ws, "dvcp_fps_pair: null pointer");
  DVCP_REQUIRE(dtype == DVCP_F32, "dvcp_fps_pair: fp32 only (dtype %d)", dtype);
  DVCP_REQUIRE(B >= 0 && B <= 32767 && N >= dvcp::kFpsBatchedMinN && N <= 16 * dvcp::kFpsSel1024,
               "dvcp_fps_pair: bad sizes B=%d N=%d", B, N);
  DVCP_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 3) == 0, "dvcp_fps_pair: workspace not 4-byte aligned");
  if (B == 0) return DVCP_OK;
  return dvcp::launch_fps_pair(dvcp::PointsView<float>{static_cast<const float*>(xyz), sb, sc, sn}, B, N, start2,
                               start3, idx2, static_cast<float*>(xyz2), idx3, static_cast<float*>(xyz3),
                               static_cast<uint32_t*>(ws), static_cast<hipStream_t>(stream));
}

extern "C" int dvcp_fps_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                           const int64_t* start, int64_t* out_idx, void* out_xyz, float* ws, int32_t* err,
                           void* stream) {
  DVCP_REQUIRE(xyz && start && out_idx, "dvcp_fps: null pointer");
  DVCP_REQUIRE(B >= 0 && N > 0 && npoint >= 0, "dvcp_fps: bad sizes B=%d N=%d npoint=%d", B, N, npoint);
  DVCP_REQUIRE(N <= 65535 || ws, "dvcp_fps: N=%d needs a workspace", N);
  if (B == 0 || npoint == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_fps<float>(static_cast<const float*>(xyz), sb, sc, sn, B, N, npoint, start, out_idx,
                                   static_cast<float*>(out_xyz), ws, err, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_fps<double>(static_cast<const double*>(xyz), sb, sc, sn, B, N, npoint, start, out_idx,
                                    static_cast<double*>(out_xyz), ws, err, st);
  dvcp::set_error("dvcp_fps: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

// Workspace bytes dvcp_fps_parts needs for B clouds of N points (any parts).
extern "C" int64_t dvcp_fps_workspace_bytes(int B, int N) {
  return B < 0 || N < 0 ? -1 : dvcp::fps_workspace_bytes(B, N);
}

// dvcp_fps_ws with a sized workspace and the split select's workgroups per cloud: parts 0 = the
// library's choice (dvcp_fps_ws's), 1 = the one-workgroup select kernel (the per-step split kernel
// above 16384 points), 2 / 4 / 8 = the split select (fp32, 2048 <= N <= 65536, as far as its
// instantiated slots reach).  ws: ws_bytes >= dvcp_fps_workspace_bytes(B, N) bytes (8-aligned).
extern "C" int dvcp_fps_parts(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                              int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz, void* ws,
                              int64_t ws_bytes, int32_t* err, int parts, void* stream) {
  DVCP_REQUIRE(xyz && start && out_idx && ws, "dvcp_fps_parts: null pointer");
  DVCP_REQUIRE(B >= 0 && N > 0 && npoint >= 0, "dvcp_fps_parts: bad sizes B=%d N=%d npoint=%d", B, N, npoint);
  DVCP_REQUIRE(parts == 0 || parts == 1 || parts == 2 || parts == 4 || parts == 8,
               "dvcp_fps_parts: parts=%d not 0, 1, 2, 4 or 8", parts);
  DVCP_REQUIRE(ws_bytes >= dvcp::fps_workspace_bytes(B, N) && (reinterpret_cast<uintptr_t>(ws) & 7) == 0,
               "dvcp_fps_parts: workspace of %lld bytes (need %lld, 8-aligned)", static_cast<long long>(ws_bytes),
               static_cast<long long>(dvcp::fps_workspace_bytes(B, N)));
  if (B == 0 || npoint == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* w = static_cast<float*>(ws);
  if (dtype == DVCP_F32)
    return dvcp::launch_fps<float>(static_cast<const float*>(xyz), sb, sc, sn, B, N, npoint, start, out_idx,
                                   static_cast<float*>(out_xyz), w, err, st, parts, ws_bytes);
  if (dtype == DVCP_F64)
    return dvcp::launch_fps<double>(static_cast<const double*>(xyz), sb, sc, sn, B, N, npoint, start, out_idx,
                                    static_cast<double*>(out_xyz), w, err, st, parts, ws_bytes);
  dvcp::set_error("dvcp_fps_parts: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

extern "C" int dvcp_fps(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N, int npoint,
                        const int64_t* start, int64_t* out_idx, void* out_xyz, void* stream) {
  return dvcp_fps_ws(dtype, xyz, sb, sc, sn, B, N, npoint, start, out_idx, out_xyz, nullptr, nullptr, stream);
}

// bench.py: `blocks` workgroups of 512 threads each run the FPS step floor chain for `steps` steps.
extern "C" int dvcp_fps_step_floor(int steps, int blocks, float* out, void* stream) {
  DVCP_REQUIRE(out && steps >= 0 && blocks > 0 && blocks <= 65535, "dvcp_fps_step_floor: bad arguments");
  hipLaunchKernelGGL((dvcp::fps_floor_kernel<dvcp::kFpsThreads / dvcp::kWave>), dim3(blocks), dim3(dvcp::kFpsThreads),
                     0, static_cast<hipStream_t>(stream), steps, out);
  return dvcp::launch_status("dvcp_fps_step_floor");
}

// Test hook for the split kernel's guard: runs the split path with the given poll cap and
// `withhold` workgroups left out of the grid (so the last cloud cannot complete).
extern "C" int dvcp_fps_split_probe(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int B, int N,
                                    int npoint, const int64_t* start, int64_t* out_idx, void* out_xyz, float* ws,
                                    int32_t* err, uint32_t spin_cap, int withhold, void* stream) {
  DVCP_REQUIRE(xyz && start && out_idx && ws && err, "dvcp_fps_split_probe: null pointer");
  DVCP_REQUIRE(B > 0 && N > 0 && npoint > 0 && withhold >= 0, "dvcp_fps_split_probe: bad sizes");
  const int S = dvcp::ceil_div(N, (dtype == DVCP_F32 ? dvcp::fps_split_ppt<float>(N) : dvcp::fps_split_ppt<double>(N)) *
                                     dvcp::kFpsSplitThreads);
  DVCP_REQUIRE(S >= 2 && S <= dvcp::kFpsSplitMax && withhold < S, "dvcp_fps_split_probe: N=%d is not a split size", N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_fps_split<float>(dvcp::PointsView<float>{static_cast<const float*>(xyz), sb, sc, sn}, B, N,
                                         npoint, start, out_idx, static_cast<float*>(out_xyz), ws, err, spin_cap,
                                         withhold, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_fps_split<double>(dvcp::PointsView<double>{static_cast<const double*>(xyz), sb, sc, sn}, B,
                                          N, npoint, start, out_idx, static_cast<double*>(out_xyz), ws, err, spin_cap,
                                          withhold, st);
  dvcp::set_error("dvcp_fps_split_probe: bad dtype %d", dtype);
  return DVCP_EINVAL;
}
