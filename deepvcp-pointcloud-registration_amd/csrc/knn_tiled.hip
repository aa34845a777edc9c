// knn_tiled.hip -- exact kNN over spatially sorted reference tiles (replaces knn_cuda.KNN at
// get_cat_feat_tgt.py:45,52; same contract as dvcp_knn in knn.hip: fp32 d2 = (dx*dx + dy*dy) +
// dz*dz with dx = ref - query, ascending, ties to the lower index, dist = correctly rounded sqrt).
//
// Why: the brute-force scan meets reference points in index order, so a lane keeps inserting into
// its sorted top-32 and the wave executes the 32-deep insertion network on almost every point.
// Here both sets are sorted by a 12-bit Morton cell, references into 64-point tiles with boxes.
// Each wave takes 64 Morton-consecutive queries (a compact box), sorts the tiles by the lower
// bound of the distance between its query box and each tile box, and scans tiles nearest first:
//   * tile data is wave-uniform, so points come through the scalar cache as SGPR operands;
//   * a tile is skipped when no lane's own lower bound reaches its current k-th distance;
//   * the scan stops when the next tile's bound exceeds every lane's k-th distance.
// Exactness: round-to-nearest is monotone, so a bound computed from box faces with the same
// float ops never exceeds the computed d2 of any point in the box; tiles are dropped only when the
// bound is strictly above the k-th distance, so every point that could enter or tie the top k is
// examined, and insertion orders by (d2, index) explicitly.
#include "common.h"
#include "morton.h"

namespace dvcp {

constexpr int kTile = 16;             // reference points per tile (finer boxes prune and order better)
constexpr int kMaxTiles = 1024;       // per cloud: M <= 16384
constexpr uint32_t kTileIdBits = 0x3FFu;  // tile id in the low bits of a sort key (kMaxTiles - 1)
constexpr int kTiledThreads = 256;    // 4 independent waves per workgroup
constexpr int kBoxBatch = 1;          // tiles whose boxes are read (LDS) and tested together

struct TiledLayout {
  float4* sorted;  // B x T*64: x, y, z, original index bits (padding: NaN, index 0x7FFFFFFF)
  float4* tbox;    // B x T x 2: {lo.xyz, _}, {hi.xyz, _}
  float4* qsorted;  // B x Q: the queries in curve order as (x, y, z, original index bits), fp32
  uint32_t* qbins;  // B x kSortBins: the queries' cell counts, then their running positions
  uint32_t* qbox;   // B x 8: ~float_order(lo.xyz), float_order(hi.xyz) of the queries (atomicMax)
};

inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

inline TiledLayout tiled_layout(void* ws, int B, int M, int Q) {
  const int64_t T = ceil_div(M, kTile);
  char* p = static_cast<char*>(ws);
  TiledLayout L;
  L.sorted = reinterpret_cast<float4*>(p);
  p += align256(16 * int64_t(B) * T * kTile);
  L.tbox = reinterpret_cast<float4*>(p);
  p += align256(32 * int64_t(B) * T);
  L.qsorted = reinterpret_cast<float4*>(p);
  p += align256(16 * int64_t(B) * Q);
  L.qbins = reinterpret_cast<uint32_t*>(p);  // qbins and qbox are one zeroed range
  L.qbox = L.qbins + int64_t(B) * kSortBins;
  return L;
}
inline int64_t tiled_zeroed_bytes(int B) { return 4 * int64_t(B) * (kSortBins + 8); }

// The queries' curve order is a counting sort spread over many workgroups (kQSortItems queries
// each; one workgroup per cloud took ~0.15 ms at C3's 85184 queries): bounding box by atomicMax
// on order keys, per-workgroup LDS histograms added into the cloud's bins, one scan per cloud,
// then a scatter by atomicAdd on the running positions (the order inside a cell is arbitrary:
// the permutation only shapes the query waves, never a result).
constexpr int kQSortItems = 8192;

template <typename CT>
__device__ __forceinline__ void qry_point(const PointsView<CT>& qry, int b, int i, float (&v)[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) v[a] = static_cast<float>(qry.at(b, a, i));  // knn_cuda's .float()
}

__device__ __forceinline__ CurveGrid qry_grid(const uint32_t* qbox, int b) {
  float lo[3], hi[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    lo[a] = float_unorder(~qbox[b * 8 + a]);
    hi[a] = float_unorder(qbox[b * 8 + 3 + a]);
  }
  return curve_grid(lo, hi);
}

template <typename CT>
__global__ __launch_bounds__(kBuildThreads) void knn_qbox_kernel(PointsView<CT> qry, int Q, uint32_t* qbox) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int i0 = blockIdx.x * kQSortItems, i1 = min(Q, i0 + kQSortItems);
  float lo[3], hi[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    lo[a] = __builtin_huge_valf();
    hi[a] = -__builtin_huge_valf();
  }
  for (int i = i0 + threadIdx.x; i < i1; i += kBuildThreads) {
    float v[3];
    qry_point(qry, b, i, v);
#pragma unroll
    for (int a = 0; a < 3; ++a) {  // fminf / fmaxf: NaN coordinates are ignored, as block_bbox
      lo[a] = fminf(lo[a], v[a]);
      hi[a] = fmaxf(hi[a], v[a]);
    }
  }
  // wave, then workgroup reduction: six atomics per workgroup (one per wave serialised ~1400
  // atomics on the same 48 bytes per launch: 43 us)
  __shared__ uint32_t red[kBuildThreads / kWave][6];
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    for (int off = 32; off > 0; off >>= 1) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off, kWave));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off, kWave));
    }
    if (lane == 0) {
      red[wave][a] = ~float_order(lo[a]);
      red[wave][3 + a] = float_order(hi[a]);
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    uint32_t m = 0u;
    for (int w = 0; w < kBuildThreads / kWave; ++w) m = max(m, red[w][threadIdx.x]);
    atomicMax(&qbox[b * 8 + threadIdx.x], m);
  }
}

template <typename CT>
__global__ __launch_bounds__(kBuildThreads) void knn_qhist_kernel(PointsView<CT> qry, int Q, const uint32_t* qbox,
                                                                  uint32_t* qbins) {
  __shared__ uint32_t bins[kSortBins];
  const int b = blockIdx.y;
  const int i0 = blockIdx.x * kQSortItems, i1 = min(Q, i0 + kQSortItems);
  for (int i = threadIdx.x; i < kSortBins; i += kBuildThreads) bins[i] = 0u;
  __syncthreads();
  const CurveGrid g = qry_grid(qbox, b);
  for (int i = i0 + threadIdx.x; i < i1; i += kBuildThreads) {
    float v[3];
    qry_point(qry, b, i, v);
    atomicAdd(&bins[curve_cell(g, v)], 1u);
  }
  __syncthreads();
  uint32_t* gb = qbins + static_cast<int64_t>(b) * kSortBins;
  for (int i = threadIdx.x; i < kSortBins; i += kBuildThreads)
    if (bins[i] != 0u) atomicAdd(&gb[i], bins[i]);
}

__global__ __launch_bounds__(kBuildThreads) void knn_qscan_kernel(uint32_t* qbins) {
  __shared__ uint32_t bins[kSortBins];
  __shared__ uint32_t wsum[16];
  uint32_t* gb = qbins + static_cast<int64_t>(blockIdx.x) * kSortBins;
  for (int i = threadIdx.x; i < kSortBins; i += kBuildThreads) bins[i] = gb[i];
  __syncthreads();
  block_scan_bins(bins, wsum);
  __syncthreads();
  for (int i = threadIdx.x; i < kSortBins; i += kBuildThreads) gb[i] = bins[i];
}

template <typename CT>
__global__ __launch_bounds__(kBuildThreads) void knn_tiled_build_kernel(PointsView<CT> ref, int M, PointsView<CT> qry,
                                                                        int Q, TiledLayout L) {
  __shared__ uint32_t bins[kSortBins];
  __shared__ uint32_t boxk[kMaxTiles][6];  // order-preserving float keys: lo.xyz (min), hi.xyz (max)
  __shared__ uint32_t wsum[16];
  __shared__ float red[2][3][16];
  const int tid = threadIdx.x;
  // With B % 8 == 0 the linear block id is re-mapped so that every block of cloud b runs on XCD
  // b % 8 (blocks reach the XCDs round robin, speed only): the scatter's 16-byte rows of a cloud
  // then meet in one L2 and leave it as whole lines (round 5's 4-byte index scatter from all eight
  // XCDs wrote 34 MB per C3 launch for 2.7 MB of permutation).
  int b = blockIdx.y, bx = blockIdx.x;
  if ((gridDim.y & 7) == 0) {
    const int lin = static_cast<int>(blockIdx.y * gridDim.x + blockIdx.x);
    const int xo = lin & 7, slot = lin >> 3;
    b = xo + 8 * (slot / static_cast<int>(gridDim.x));
    bx = slot % static_cast<int>(gridDim.x);
  }
  if (bx > 0) {  // the queries' scatter into curve order (the scanned bins are running positions)
    const int i0 = (bx - 1) * kQSortItems, i1 = min(Q, i0 + kQSortItems);
    const CurveGrid g = qry_grid(L.qbox, b);
    uint32_t* gb = L.qbins + static_cast<int64_t>(b) * kSortBins;
    float4* qs = L.qsorted + static_cast<int64_t>(b) * Q;
    for (int i = i0 + tid; i < i1; i += kBuildThreads) {
      float v[3];
      qry_point(qry, b, i, v);
      qs[atomicAdd(&gb[curve_cell(g, v)], 1u)] = make_float4(v[0], v[1], v[2], __int_as_float(i));
    }
    return;
  }
  const int T = (M + kTile - 1) / kTile;
  float4* so = L.sorted + static_cast<int64_t>(b) * T * kTile;
  // knn_cuda casts both inputs with .float()
  auto get_ref = [&](int i, float (&v)[3]) {
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] = static_cast<float>(ref.at(b, a, i));
  };
  for (int i = tid; i < T * 6; i += kBuildThreads) boxk[i / 6][i % 6] = (i % 6) < 3 ? 0xFFFFFFFFu : 0u;
  float lo[3], hi[3];
  block_bbox(M, get_ref, lo, hi, red);
  morton_sort(
      M, get_ref,
      [&](int pos, int i, const float (&v)[3]) {
        so[pos] = make_float4(v[0], v[1], v[2], __int_as_float(i));
        const int t = pos / kTile;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          atomicMin(&boxk[t][a], float_order(v[a]));
          atomicMax(&boxk[t][3 + a], float_order(v[a]));
        }
      },
      lo, hi, bins, wsum);
  for (int pos = M + tid; pos < T * kTile; pos += kBuildThreads)
    so[pos] = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __int_as_float(0x7FFFFFFF));
  for (int t = tid; t < T; t += kBuildThreads) {
    float4* tb = L.tbox + (static_cast<int64_t>(b) * T + t) * 2;
    tb[0] = make_float4(float_unorder(boxk[t][0]), float_unorder(boxk[t][1]), float_unorder(boxk[t][2]), 0.f);
    tb[1] = make_float4(float_unorder(boxk[t][3]), float_unorder(boxk[t][4]), float_unorder(boxk[t][5]), 0.f);
  }
}

// Lower bound of the computed d2 between a point in box [a_lo, a_hi] and a point in box
// [b_lo, b_hi] (per axis gap fl(b_lo - a_hi) or fl(a_lo - b_hi), then the d2 formula).
__device__ __forceinline__ float box_box_lb2(float alx, float aly, float alz, float ahx, float ahy, float ahz,
                                             float blx, float bly, float blz, float bhx, float bhy, float bhz) {
  const float gx = fmaxf(fmaxf(blx - ahx, alx - bhx), 0.0f);
  const float gy = fmaxf(fmaxf(bly - ahy, aly - bhy), 0.0f);
  const float gz = fmaxf(fmaxf(blz - ahz, alz - bhz), 0.0f);
  return (gx * gx + gy * gy) + gz * gz;
}

// Tile boxes at half precision, rounded outward (largest half <= lo, smallest half >= hi; NaN
// and +-inf pass through): 8 bytes per corner pair instead of 32, and box_box_lb2 over the widened
// box is still a lower bound of every computed d2 in the tile (the gaps are monotone in the box).
__device__ __forceinline__ uint32_t half_down(float x) {
  const _Float16 h = static_cast<_Float16>(x);
  uint32_t hb = __builtin_bit_cast(uint16_t, h);
  if (static_cast<float>(h) > x) hb = (hb & 0x8000u) ? hb + 1u : (hb == 0u ? 0x8001u : hb - 1u);
  return hb;
}
__device__ __forceinline__ uint32_t half_up(float x) {
  const _Float16 h = static_cast<_Float16>(x);
  uint32_t hb = __builtin_bit_cast(uint16_t, h);
  if (static_cast<float>(h) < x) hb = (hb & 0x8000u) ? (hb == 0x8000u ? 0x0001u : hb - 1u) : hb + 1u;
  return hb;
}
__device__ __forceinline__ float half_lo(uint32_t w) {
  return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(w & 0xFFFFu)));
}
__device__ __forceinline__ float half_hi(uint32_t w) {
  return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(w >> 16)));
}
// {lo.x | lo.y << 16, lo.z | hi.x << 16, hi.y | hi.z << 16}
__device__ __forceinline__ uint3 pack_hbox(const float4& lo, const float4& hi) {
  return make_uint3(half_down(lo.x) | (half_down(lo.y) << 16), half_down(lo.z) | (half_up(hi.x) << 16),
                    half_up(hi.y) | (half_up(hi.z) << 16));
}
__device__ __forceinline__ float hbox_lb2(const uint3& h, float ax, float ay, float az, float bx, float by, float bz) {
  return box_box_lb2(ax, ay, az, bx, by, bz, half_lo(h.x), half_hi(h.x), half_lo(h.y), half_hi(h.y), half_lo(h.z),
                     half_hi(h.z));
}

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_max_u(uint32_t v) {
  return max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROWS, 0xF, false)));
}
// max over the wave of non-negative float bits (k-th distances; +inf allowed)
__device__ __forceinline__ float wave_max_nonneg(float x) {
  uint32_t v = __float_as_uint(x);
  v = dpp_max_u<0x111, 0xF>(v);
  v = dpp_max_u<0x112, 0xF>(v);
  v = dpp_max_u<0x114, 0xF>(v);
  v = dpp_max_u<0x118, 0xF>(v);
  v = dpp_max_u<0x142, 0xA>(v);
  v = dpp_max_u<0x143, 0xC>(v);
  return __uint_as_float(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63)));
}

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_or_u(uint32_t v) {
  return v | static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROWS, 0xF, false));
}
// bitwise or over the wave (wave-uniform result)
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  v = dpp_or_u<0x111, 0xF>(v);
  v = dpp_or_u<0x112, 0xF>(v);
  v = dpp_or_u<0x114, 0xF>(v);
  v = dpp_or_u<0x118, 0xF>(v);
  v = dpp_or_u<0x142, 0xA>(v);
  v = dpp_or_u<0x143, 0xC>(v);
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// max over the wave of any floats (order-preserving bits)
__device__ __forceinline__ float wave_max_nonneg_signed(float x) {
  uint32_t v = float_order(x);
  v = dpp_max_u<0x111, 0xF>(v);
  v = dpp_max_u<0x112, 0xF>(v);
  v = dpp_max_u<0x114, 0xF>(v);
  v = dpp_max_u<0x118, 0xF>(v);
  v = dpp_max_u<0x142, 0xA>(v);
  v = dpp_max_u<0x143, 0xC>(v);
  return float_unorder(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63)));
}
__device__ __forceinline__ uint32_t wave_umax_i(uint32_t v) {
  v = dpp_max_u<0x111, 0xF>(v);
  v = dpp_max_u<0x112, 0xF>(v);
  v = dpp_max_u<0x114, 0xF>(v);
  v = dpp_max_u<0x118, 0xF>(v);
  v = dpp_max_u<0x142, 0xA>(v);
  v = dpp_max_u<0x143, 0xC>(v);
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// This lane's index, formed where it is used (an opaque v_mbcnt pair the compiler cannot hoist):
// a lane-dependent value held across the select kernel's scan was its last scratch spill.
__device__ __forceinline__ int knn_fresh_lane() {
  int r;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
  return r;
}

// Bitonic sort (ascending) of 64*R keys held as keys[r] at position r*64 + lane.
template <int R>
__device__ __forceinline__ void wave_bitonic(uint32_t (&keys)[R]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= 64 * R; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {  // partner is another register of the same lane
        const int jr = j >> 6;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if ((r & jr) == 0) {
            const int i = r * 64 + lane;
            const bool up = (i & k) == 0;
            const uint32_t a = keys[r], c = keys[r + jr];
            const bool sw = up ? (a > c) : (a < c);
            keys[r] = sw ? c : a;
            keys[r + jr] = sw ? a : c;
          }
        }
      } else {  // partner lane = lane ^ j, same register
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int i = r * 64 + lane;
          const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(keys[r]), j, kWave));
          const bool lower = (lane & j) == 0;  // this lane holds the lower index of the pair
          const bool up = (i & k) == 0;
          const uint32_t mn = min(keys[r], o), mx = max(keys[r], o);
          keys[r] = (lower == up) ? mn : mx;
        }
      }
    }
  }
}

template <int KT, int R>
__global__ __launch_bounds__(kTiledThreads) void knn_tiled_query_kernel(const float4* __restrict__ sorted,
                                                                        const float4* __restrict__ tbox,
                                                                        const float4* __restrict__ qsorted, int M,
                                                                        int Q, int k, float* __restrict__ dist,
                                                                        int32_t* __restrict__ idx,
                                                                        int64_t* __restrict__ idx64, int B8) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // Cloud and block within it.  Workgroups reach the 8 XCDs round robin by linear id, so with
  // B % 8 == 0 the linear id is re-mapped to give XCD x the clouds x, x + 8, ...: each cloud's
  // sorted points and boxes are then fetched into one XCD's L2 instead of all eight.
  int b = blockIdx.y, bx = blockIdx.x;
  if ((B8 & 1) != 0) {
    const int lin = static_cast<int>(blockIdx.y * gridDim.x + blockIdx.x);
    const int xo = lin & 7, slot = lin >> 3;
    b = xo + 8 * (slot / static_cast<int>(gridDim.x));
    bx = slot % static_cast<int>(gridDim.x);
  }
  const int T = (M + kTile - 1) / kTile;
  // the cloud's tile boxes in LDS (all four waves scan the same cloud): the per-lane box test
  // then reads LDS broadcasts kBoxBatch tiles at a time instead of waiting on a scalar load per tile
  __shared__ float4 sbox[2 * kMaxTiles];
  {
    const float4* tbg = tbox + static_cast<int64_t>(b) * T * 2;
    for (int i = threadIdx.x; i < 2 * T; i += kTiledThreads) sbox[i] = tbg[i];
    __syncthreads();
  }
  const int sq = (bx * (kTiledThreads / kWave) + wave) * kWave + lane;
  if ((bx * (kTiledThreads / kWave) + wave) * kWave >= Q) return;  // whole wave past the end
  const bool live = sq < Q;
  // this lane's query in curve order: one coalesced 16-byte row (converted to fp32 by the scatter,
  // knn_cuda's .float())
  const float4 qrow = live ? qsorted[static_cast<int64_t>(b) * Q + sq] : make_float4(0.f, 0.f, 0.f, 0.f);
  [[maybe_unused]] const int q = __float_as_int(qrow.w);
  const float qx = qrow.x, qy = qrow.y, qz = qrow.z;
  // the wave's query box (live lanes only)
  float wl[3] = {live ? qx : __builtin_huge_valf(), live ? qy : __builtin_huge_valf(),
                 live ? qz : __builtin_huge_valf()};
  float wh[3] = {live ? qx : -__builtin_huge_valf(), live ? qy : -__builtin_huge_valf(),
                 live ? qz : -__builtin_huge_valf()};
#pragma unroll
  for (int a = 0; a < 3; ++a)
    for (int off = 32; off > 0; off >>= 1) {
      wl[a] = fminf(wl[a], __shfl_xor(wl[a], off, kWave));
      wh[a] = fmaxf(wh[a], __shfl_xor(wh[a], off, kWave));
    }
  const float4* tb = tbox + static_cast<int64_t>(b) * T * 2;
  // tile keys: lb2(query box, tile box) with the low 10 mantissa bits replaced by the tile id.
  // Truncation only lowers a non-negative float, so key value <= the true bound.
  uint32_t keys[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = r * 64 + lane;
    if (t < T) {
      const float4 lo = tb[2 * t], hi = tb[2 * t + 1];
      const float lb = box_box_lb2(wl[0], wl[1], wl[2], wh[0], wh[1], wh[2], lo.x, lo.y, lo.z, hi.x, hi.y, hi.z);
      keys[r] = (__float_as_uint(lb) & ~kTileIdBits) | static_cast<uint32_t>(t);
    } else {
      keys[r] = 0xFFFFFFFFu;
    }
  }
  wave_bitonic<R>(keys);

  // The list is kept as 64-bit keys (d2 bits << 32 | index): d2 >= 0 orders like its bits, so
  // one unsigned compare orders by (d2, index) and an insertion is one compare + two selects
  // per slot.
  // (stored as 32-bit halves: a dynamically indexed 64-bit array is not promoted to registers)
  uint32_t kh[KT], kl[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {  // empty slot: (+inf, 0xFFFFFFFF), above every finite point
    kh[t] = 0x7F800000u;
    kl[t] = ~0u;
  }
  constexpr uint64_t kEmpty = (static_cast<uint64_t>(0x7F800000u) << 32) | 0xFFFFFFFFu;
#define DVCP_KK(t) ((static_cast<uint64_t>(kh[t]) << 32) | kl[t])
  const int kq = k - 1;  // wave-uniform: kh[kq], kl[kq] are indexed register reads
  float kth = live ? __builtin_huge_valf() : 0.0f;  // dead lanes never need more points
  uint64_t kkey = live ? kEmpty : 0ull;
  float wkth = wave_max_nonneg(kth);
  const float4* P = uniform_ptr(sorted + static_cast<int64_t>(b) * T * kTile);
  bool stop = false;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    for (int i0 = 0; i0 < 64 && !stop; i0 += kBoxBatch) {
      if (r * 64 + i0 >= T) break;
      // kBoxBatch tiles of the order: keys, then their boxes (LDS broadcasts) and this lane's bounds
      uint32_t key4[kBoxBatch];
      float lb4[kBoxBatch];
#pragma unroll
      for (int j = 0; j < kBoxBatch; ++j) {
        key4[j] = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(keys[r]), i0 + j));
        const int tj = static_cast<int>(key4[j] & kTileIdBits) < T ? static_cast<int>(key4[j] & kTileIdBits) : 0;
        const float4 lo = sbox[2 * tj], hi = sbox[2 * tj + 1];
        lb4[j] = box_box_lb2(qx, qy, qz, qx, qy, qz, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z);
      }
#pragma unroll
      for (int j = 0; j < kBoxBatch; ++j) {
      if (r * 64 + i0 + j >= T) break;
      const uint32_t key = key4[j];
      if (__uint_as_float(key & ~kTileIdBits) > wkth) {  // every later tile is farther
        stop = true;
        break;
      }
      const int t = static_cast<int>(key & kTileIdBits);
      const float lbq = lb4[j];
      const bool act = live & (lbq <= kth);
      if (__ballot(act) == 0) continue;
      const const_float* tp = (const const_float*)(P + t * kTile);
      uint64_t ins = 0;
      for (int j0 = 0; j0 < kTile; j0 += 16) {
        // the whole 16-point chunk is loaded (scalar loads, one wait) before any branch
        float c[64];
#pragma unroll
        for (int u = 0; u < 64; ++u) c[u] = tp[4 * j0 + u];
        // pass 1 (unrolled): every distance of the chunk, and which points are a candidate for
        // some lane against the k-th key at chunk start (a superset: the key only decreases)
        float d2v[16];
        uint32_t piv[16];
        uint32_t todo = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float dx = c[4 * j] - qx, dy = c[4 * j + 1] - qy, dz = c[4 * j + 2] - qz;
          d2v[j] = (dx * dx + dy * dy) + dz * dz;
          piv[j] = __float_as_uint(c[4 * j + 3]);
          const uint64_t pk = (static_cast<uint64_t>(__float_as_uint(d2v[j])) << 32) | piv[j];
          // d2 < inf also rejects NaN (padding) and infinite distances, as dvcp_knn does
          const bool cand = act & (d2v[j] < __builtin_huge_valf()) & (pk < kkey);
          todo |= __ballot(cand) != 0 ? (1u << j) : 0u;
        }
        // pass 2: those points in order, each re-tested against the current key, then inserted
        // (one compare + two selects per slot)
        while (todo) {
          const int j = __builtin_ctz(todo);
          todo &= todo - 1;
          const float d2 = d2v[j];  // indexed register reads (uniform j)
          const uint32_t pi = piv[j];
          const uint64_t pk = (static_cast<uint64_t>(__float_as_uint(d2)) << 32) | pi;
          const bool cand = act & (d2 < __builtin_huge_valf()) & (pk < kkey);
          const uint64_t m = __ballot(cand);
          if (m == 0) continue;
          ins |= m;
          // a non-candidate lane compares with the all-ones key, which is below no slot
          const uint64_t pkc = cand ? pk : ~0ull;
          bool lt[KT];
#pragma unroll
          for (int u = 0; u < KT; ++u) lt[u] = pkc < DVCP_KK(u);
#pragma unroll
          for (int u = KT - 1; u > 0; --u) {
            kh[u] = lt[u - 1] ? kh[u - 1] : (lt[u] ? __float_as_uint(d2) : kh[u]);
            kl[u] = lt[u - 1] ? kl[u - 1] : (lt[u] ? pi : kl[u]);
          }
          kh[0] = lt[0] ? __float_as_uint(d2) : kh[0];
          kl[0] = lt[0] ? pi : kl[0];
          kkey = live ? (KT == 1 ? DVCP_KK(0) : DVCP_KK(kq)) : 0ull;
          kth = __uint_as_float(static_cast<uint32_t>(kkey >> 32));
        }
      }
      if (ins != 0) wkth = wave_max_nonneg(kth);
      }
    }
  }
  if (!live) return;
  const int64_t o = (static_cast<int64_t>(b) * Q + q) * k;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    if (t < k) {
      const bool ok = DVCP_KK(t) != kEmpty;  // fewer than k finite points: like dvcp_knn (inf, -1)
      const float d2 = __uint_as_float(kh[t]);
      const int i = static_cast<int>(kl[t]);
      if (dist) dist[o + t] = ok ? sqrt_rn(d2) : __builtin_huge_valf();
      if (idx) idx[o + t] = ok ? i : -1;
      if (idx64) idx64[o + t] = ok ? i : -1;
    }
  }
#undef DVCP_KK
}


// ---------------------------------------------------------------------------------------------
// Buffered selection (k in 17..32; the forward's k = 32).  Same tiles, wave-ordered scan, pruning
// and stop rule as knn_tiled_query_kernel, but a lane no longer inserts each candidate into its
// sorted top-32 as it appears (a 32-slot insertion network that the whole wave executes for every
// point that is a candidate for ANY lane: ~220 such steps per wave at C3, the kernel's cost).
// Instead each lane appends its own candidates -- (d2, index) keys below its current k-th key --
// to a private 16-entry LDS buffer, and when some lane's buffer would overflow the wave merges:
// every lane sorts its buffer (16-key bitonic network in registers), folds it into its sorted
// top-32 (C[i] = min(top[i], buf[31 - i]) is bitonic and holds the 32 smallest keys; one
// 32-key bitonic merge sorts it) and re-reads its k-th key.  The wave then pays per merge, ~850
// VALU instructions for up to 16 candidates per lane, instead of ~160 per union candidate.
// Exactness is unchanged: the merged list is always the 32 smallest (d2, index) keys of every
// point appended, and a point is only left out when its key is not below a k-th key that is at
// least the true one (filters and pruning use the last merged, i.e. a stale-high, k-th key).
// DVCP_KNN_SORD: the sorted tile order in LDS (default); DVCP_KNN_STAGE_OUT: coalesced output rows
#ifndef DVCP_KNN_SORD
#define DVCP_KNN_SORD 1
#endif
#ifndef DVCP_KNN_STAGE_OUT
#define DVCP_KNN_STAGE_OUT 2
#endif
constexpr int kSelBufN = 16;   // buffer capacity per lane (>= kTile: a merge makes room for a whole tile)
constexpr int kSelSortN = 16;
constexpr int kSordWords = (kMaxTiles + 2) / 3;  // a wave's sorted tile order, three 10-bit ids per word
// A tile's 256 bytes are loaded once some lane is known to need it (prefetching one sorted position
// ahead made every scanned tile wait for its successor's load at the loop latch, ~660 clk per
// skipped tile under DVCP_KNN_DIAG; round 3).
// DVCP_KNN_CHUNK (default): the sorted order is scanned 64 positions at a time behind a
// tile-parallel prefilter against lane-group boxes (see the scan below).
// (Round 4 measured an exact per-lane bulk test over each 64-position chunk -- every lane's tile
// box against all 64 queries of the wave -- 0.92 against 0.75 ms per C3 batch: not kept.)
#ifndef DVCP_KNN_CHUNK
#define DVCP_KNN_CHUNK 1
#endif
// (Round 4 also measured issuing the tile loads of 2 or 3 surviving positions together before
// their visits: 0.77 / 0.83 against 0.76 ms -- the scan is not waiting on those loads.)
// DVCP_KNN_SLOAD: an active tile's 16 points reach the wave as scalar loads (the tile index is
// wave-uniform, the tile is read-only here) instead of one vector load and 48 readlanes; the
// appends, which index the tile per lane, load their LDS copy from L2 when a lane needs one.
// Round 4, A/B on one box (tools/knn_bench.py --fast, profiles/round4/r4t/r4t_knn_sload_ab.log):
// 0.763 / 0.755 -> 0.751 / 0.742 ms per C3 call, identical results, although the 48 scalar values
// push the kernel to 76 B of scratch at 168 VGPRs (filtering in two 8-point batches, or re-loading
// the tile after a merge instead of holding it, spilled more: 80-624 B).
#ifndef DVCP_KNN_SLOAD
#define DVCP_KNN_SLOAD 1
#endif

// (d2, index) keys packed into doubles of [1, 2) (see knn_sel_query_kernel): 14 index bits
constexpr double kKeyEmpty = __builtin_bit_cast(double, 0x3FF0000000000000ull | (0x7F800000ull << 14) | 0x3FFFull);
__device__ __forceinline__ double key_pack(float d2, uint32_t index) {
  return __builtin_bit_cast(double, 0x3FF0000000000000ull | (static_cast<uint64_t>(__float_as_uint(d2)) << 14) |
                                        static_cast<uint64_t>(index & 0x3FFFu));
}
__device__ __forceinline__ float key_d2(double kd) {
  return __uint_as_float(static_cast<uint32_t>((__builtin_bit_cast(uint64_t, kd) >> 14) & 0x7FFFFFFFull));
}
__device__ __forceinline__ int key_index(double kd) {
  return static_cast<int>(__builtin_bit_cast(uint64_t, kd) & 0x3FFFull);
}
__device__ __forceinline__ void key_ce_f64(double& a, double& b, bool asc) {
  const double lo = __builtin_fmin(a, b), hi = __builtin_fmax(a, b);
  a = asc ? lo : hi;
  b = asc ? hi : lo;
}

__device__ __forceinline__ void key_ce(uint32_t& ah, uint32_t& al, uint32_t& bh, uint32_t& bl, bool asc) {
  const uint64_t a = (static_cast<uint64_t>(ah) << 32) | al, b = (static_cast<uint64_t>(bh) << 32) | bl;
  const bool sw = asc ? (b < a) : (a < b);
  const uint32_t th = ah, tl = al;
  ah = sw ? bh : ah;
  al = sw ? bl : al;
  bh = sw ? th : bh;
  bl = sw ? tl : bl;
}

// Every k in 17..32 selects the 32 nearest keys (the pruning bound is the 32nd) and writes the
// first k: ordered by (d^2, index), the first k of the 32 nearest are the k nearest.  (Round 5
// had a k < 32 instantiation bounding by the k-th key: its select loop over the slots cost 272 B
// of scratch per lane; k = 17..31 are test and API cases, the forward's k is 32.)
template <int R>
__global__ __launch_bounds__(kTiledThreads) __attribute__((amdgpu_waves_per_eu(3))) void knn_sel_query_kernel(const float4* __restrict__ sorted,
                                                                      const float4* __restrict__ tbox,
                                                                      const float4* __restrict__ qsorted, int M,
                                                                      int Q, int k,
                                                                      float* __restrict__ dist,
                                                                      int32_t* __restrict__ idx,
                                                                      int64_t* __restrict__ idx64, int B8) {
  constexpr int KT = 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int b = blockIdx.y, bx = blockIdx.x;
  if ((B8 & 1) != 0) {  // XCD-aware cloud mapping, as knn_tiled_query_kernel
    const int lin = static_cast<int>(blockIdx.y * gridDim.x + blockIdx.x);
    const int xo = lin & 7, slot = lin >> 3;
    b = xo + 8 * (slot / static_cast<int>(gridDim.x));
    bx = slot % static_cast<int>(gridDim.x);
  }
  const int T = (M + kTile - 1) / kTile;
  // 12 + 32 + 5.3 KB of LDS (half-precision boxes, candidate buffers, sorted tile order): three
  // workgroups per CU
  __shared__ uint3 hbox[kMaxTiles];
  // each wave's tile order after the sort, three 10-bit tile ids per word (the chunked scan
  // recomputes the keys from them): 16 key registers held across the scan spilled to scratch and
  // were reloaded every chunk
  __shared__ uint32_t sord[kTiledThreads / kWave][kSordWords];
  __shared__ double sbuf[kTiledThreads / kWave][kSelBufN][kWave];  // lane-private candidate buffers (packed keys)
  __shared__ float4 stile[kTiledThreads / kWave][kTile];            // the wave's current tile (appends)
  {
    const float4* tbg = tbox + static_cast<int64_t>(b) * T * 2;
    for (int i = threadIdx.x; i < T; i += kTiledThreads) hbox[i] = pack_hbox(tbg[2 * i], tbg[2 * i + 1]);
    __syncthreads();
  }
  // the wave's first curve position (wave-uniform) and this lane's
  const int sq0 = __builtin_amdgcn_readfirstlane((bx * (kTiledThreads / kWave) + wave) * kWave);
  const int sq = sq0 + lane;
  if (sq0 >= Q) return;  // whole wave past the end
  const bool live = sq < Q;
  // this lane's query in curve order: one coalesced 16-byte row (converted to fp32 by the scatter,
  // knn_cuda's .float())
  const float4 qrow = live ? qsorted[static_cast<int64_t>(b) * Q + sq] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float qx = qrow.x, qy = qrow.y, qz = qrow.z;
  // the query's output row index, re-read from its curve row where the rows are written (held
  // across the scan, it and the position were spilled)
  auto out_row = [&]() {
    const int sqn = sq0 + knn_fresh_lane();
    return __float_as_int(qsorted[static_cast<int64_t>(b) * Q + sqn].w);
  };
  float wl[3] = {live ? qx : __builtin_huge_valf(), live ? qy : __builtin_huge_valf(),
                 live ? qz : __builtin_huge_valf()};
  float wh[3] = {live ? qx : -__builtin_huge_valf(), live ? qy : -__builtin_huge_valf(),
                 live ? qz : -__builtin_huge_valf()};
#pragma unroll
  for (int a = 0; a < 3; ++a) {  // (wave-uniform: SGPRs)
    wl[a] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(-wave_max_nonneg_signed(-wl[a]))));
    wh[a] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_max_nonneg_signed(wh[a]))));
  }
  uint32_t keys[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = r * 64 + lane;
    if (t < T) {
      const float lb = hbox_lb2(hbox[t], wl[0], wl[1], wl[2], wh[0], wh[1], wh[2]);
      keys[r] = (__float_as_uint(lb) & ~kTileIdBits) | static_cast<uint32_t>(t);
    } else {
      keys[r] = 0xFFFFFFFFu;
    }
  }
  wave_bitonic<R>(keys);

  // This lane's 32 smallest keys so far, ascending.  A key (d2, index) is packed into the mantissa
  // of a double in [1, 2): bits 0x3FF0'0000'0000'0000 | d2_bits << 14 | index (M <= 16384: 14 index
  // bits; non-negative d2 bits order like the values), so doubles order exactly like the keys and
  // a compare-exchange is one v_min_f64 + one v_max_f64 instead of a 64-bit compare and four selects.
  double tk[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) tk[t] = kKeyEmpty;
  float kth = live ? __builtin_huge_valf() : 0.0f;  // dead lanes never take a point
  float wkth = wave_max_nonneg(kth);
  int fill = 0;
  double(*mybuf)[kWave] = sbuf[wave];
#ifdef DVCP_KNN_DIAG  // per-wave counters (diagnostic builds only; written over lane 0's distances)
  uint64_t dg_t0 = __builtin_readcyclecounter(), dg_merge_clk = 0, dg_skip_clk = 0, dg_prev = 0;
  int dg_kind = -1;  // the previous iteration: 0 skipped, 1 processed
  int dg_scanned = 0, dg_active = 0, dg_merges = 0, dg_appends = 0;
#endif

  auto merge = [&]() {
    const int n = static_cast<int>(wave_umax_i(static_cast<uint32_t>(fill)));  // wave-uniform
    if (n == 0) return;
#ifdef DVCP_KNN_DIAG
    const uint64_t dg_m0 = __builtin_readcyclecounter();
    ++dg_merges;
#endif
    double bk[kSelSortN];
#pragma unroll
    for (int i = 0; i < kSelSortN; ++i) {
      bk[i] = kKeyEmpty;
      if (i < kSelBufN && i < n) {
        const double e = mybuf[i][lane];
        bk[i] = i < fill ? e : bk[i];
      }
    }
    // bitonic sort of the 16 buffered keys, ascending
#pragma unroll
    for (int kk = 2; kk <= kSelSortN; kk <<= 1)
#pragma unroll
      for (int j = kk >> 1; j > 0; j >>= 1)
#pragma unroll
        for (int i = 0; i < kSelSortN; ++i) {
          const int l = i ^ j;
          if (l > i) key_ce_f64(bk[i], bk[l], (i & kk) == 0);
        }
    // C[i] = min(top[i], buf[31 - i]) (buf[16..31] = empty): bitonic, the 32 smallest keys
#pragma unroll
    for (int i = KT - kSelSortN; i < KT; ++i) tk[i] = __builtin_fmin(tk[i], bk[KT - 1 - i]);
    // bitonic merge, ascending
#pragma unroll
    for (int j = KT >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        const int l = i ^ j;
        if (l > i) key_ce_f64(tk[i], tk[l], true);
      }
    kth = live ? key_d2(tk[KT - 1]) : 0.0f;
    wkth = wave_max_nonneg(kth);
    fill = 0;
#ifdef DVCP_KNN_DIAG
    dg_merge_clk += __builtin_readcyclecounter() - dg_m0;
#endif
  };

  // A needed tile is one coalesced 256-byte load (16 points x 4 floats: one float per lane) whose
  // coordinates reach every lane by readlane (SGPR operands).
  // (Per-wave counters, DVCP_KNN_DIAG, C3: ~185 tiles pass the wave's bound, ~32 of them have a
  // lane within its own k-th distance, 11 merges = 20-24 % of the wave's clock.  Loading only the
  // tiles some lane needs, found by a look-ahead test, was slower: 0.97 -> 1.11 ms per call,
  // profiles/round3/r3x_knn_diag_*.log.)
  const float* P = reinterpret_cast<const float*>(sorted) + static_cast<int64_t>(b) * T * kTile * 4;
  // Visit the tile of sorted key `key` (its bound already known not to exceed wkth): the per-lane
  // test, then the distances, the filter and the appends.
  // (the tile's float for this lane, loaded by the caller once some lane is active)
  auto visit_loaded = [&](uint32_t key, float lbq, float v_cur) {
    [[maybe_unused]] const int t = static_cast<int>(key & kTileIdBits);  // (DVCP_KNN_SLOAD only)
    const bool act = live & (lbq <= kth);
#ifdef DVCP_KNN_DIAG
    ++dg_scanned;
#endif
    if (__ballot(act) == 0) return;
#ifdef DVCP_KNN_DIAG
    ++dg_active;
    dg_kind = 1;
#endif
    float c[3 * kTile];
#if DVCP_KNN_SLOAD
    {
      const float4* Pt = reinterpret_cast<const float4*>(P) + static_cast<int64_t>(t) * kTile;
#pragma unroll
      for (int j = 0; j < kTile; ++j) {
        const float4 pj = Pt[j];
        c[3 * j] = pj.x;
        c[3 * j + 1] = pj.y;
        c[3 * j + 2] = pj.z;
      }
    }
#else
    auto bc = [&](int u) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v_cur), u)); };
#pragma unroll
    for (int j = 0; j < kTile; ++j) {
      c[3 * j] = bc(4 * j);
      c[3 * j + 1] = bc(4 * j + 1);
      c[3 * j + 2] = bc(4 * j + 2);
    }
#endif
    // d2 is recomputed wherever it is needed (the same expression, the same bits) instead of
    // being held in 16 VGPRs across the merge and the appends
    auto d2_of = [&](int j) {
      const float dx = c[3 * j] - qx, dy = c[3 * j + 1] - qy, dz = c[3 * j + 2] - qz;
      return (dx * dx + dy * dy) + dz * dz;
    };
    uint32_t cm = 0;
    // Filter on the distance alone, d2 <= kf: a superset of the keys below the k-th key (a tie
    // with a higher index is appended too and dropped by the merge, which orders full keys);
    // kf is finite, so inf and NaN (padding) never pass, as in dvcp_knn.
    const float kf = fminf(kth, __builtin_bit_cast(float, 0x7F7FFFFFu));
#pragma unroll
    for (int j = 0; j < kTile; ++j) cm |= (act && d2_of(j) <= kf) ? (1u << j) : 0u;
    if (wave_umax_i(static_cast<uint32_t>(fill + __popc(cm))) > static_cast<uint32_t>(kSelBufN)) {
      merge();  // room for the whole tile; then re-filter against the new k-th key
      const float kf2 = fminf(kth, __builtin_bit_cast(float, 0x7F7FFFFFu));
#pragma unroll
      for (int j = 0; j < kTile; ++j) cm &= d2_of(j) <= kf2 ? ~0u : ~(1u << j);
    }
    // appends: each lane walks its own mask, reading its points from the wave's copy of the tile
    // in LDS (the wave loops max-over-lanes popc(mask) times instead of over the union of the
    // masks with four readlanes per point); the same d2 expression, the same bits
    if (__ballot(cm != 0) != 0) {  // wave-uniform: every lane writes its float of the tile
#if DVCP_KNN_SLOAD
      reinterpret_cast<float*>(stile[wave])[lane] = P[static_cast<int64_t>(t) * (4 * kTile) + lane];
#else
      reinterpret_cast<float*>(stile[wave])[lane] = v_cur;
#endif
      __builtin_amdgcn_wave_barrier();
      uint32_t my = cm;
      while (__ballot(my != 0) != 0) {
        if (my != 0) {
          const int j = __builtin_ctz(my);
          my &= my - 1;
#ifdef DVCP_KNN_DIAG
          ++dg_appends;
#endif
          const float4 pt = stile[wave][j];
          const float dx = pt.x - qx, dy = pt.y - qy, dz = pt.z - qz;
          mybuf[fill][lane] = key_pack((dx * dx + dy * dy) + dz * dz, __float_as_uint(pt.w));
          ++fill;
        }
      }
      __builtin_amdgcn_wave_barrier();  // (the next active tile rewrites stile)
    }
  };
  auto visit = [&](uint32_t key) {
    const int t = static_cast<int>(key & kTileIdBits);
    const float lbq = hbox_lb2(hbox[t], qx, qy, qz, qx, qy, qz);
    float v = 0.0f;
    if (__ballot(live & (lbq <= kth)) != 0) v = P[static_cast<int64_t>(t) * (4 * kTile) + lane];
    visit_loaded(key, lbq, v);
  };

#if DVCP_KNN_CHUNK
  // Chunked scan.  The sorted order is taken 64 positions at a time, one position per lane, and a
  // tile-parallel prefilter drops the positions no query can need: lane i tests its tile's box
  // against the boxes of the wave's kKnnSub lane groups (16 Hilbert-consecutive queries each) with
  // each group's largest k-th distance.  A position survives when some group's bound reaches its
  // k-th distance; only survivors get the per-lane test (visit).  The group bounds come from k-th
  // distances read at chunk start: merges only lower them, so a stale bound keeps a superset and
  // the scan stays exact; the stop rule is re-checked at every surviving position.
  constexpr int kKnnSub = 4, kSubLanes = kWave / kKnnSub;
  float gl[3] = {wl[0], wl[1], wl[2]}, gh[3] = {wh[0], wh[1], wh[2]};  // (overwritten below)
  {
    float a[3] = {live ? qx : __builtin_huge_valf(), live ? qy : __builtin_huge_valf(),
                  live ? qz : __builtin_huge_valf()};
    float z[3] = {live ? qx : -__builtin_huge_valf(), live ? qy : -__builtin_huge_valf(),
                  live ? qz : -__builtin_huge_valf()};
#pragma unroll
    for (int ax = 0; ax < 3; ++ax)
#pragma unroll
      for (int off = kSubLanes / 2; off > 0; off >>= 1) {
        a[ax] = fminf(a[ax], __shfl_xor(a[ax], off, kWave));
        z[ax] = fmaxf(z[ax], __shfl_xor(z[ax], off, kWave));
      }
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      gl[ax] = a[ax];
      gh[ax] = z[ax];
    }
  }
  // every group's box, in LDS (read back as broadcasts per chunk: 24 wave-uniform values held in
  // registers across the scan would spill)
  __shared__ float4 sgbox[kTiledThreads / kWave][kKnnSub][2];
  if ((lane & (kSubLanes - 1)) == 0) {
    sgbox[wave][lane / kSubLanes][0] = make_float4(gl[0], gl[1], gl[2], 0.0f);
    sgbox[wave][lane / kSubLanes][1] = make_float4(gh[0], gh[1], gh[2], 0.0f);
  }
  // the sorted order to LDS; the keys are recomputed per chunk from the tile id (the same
  // expression as above: the same bits)
#if DVCP_KNN_SORD
  for (int i = lane; i < kSordWords; i += kWave) sord[wave][i] = 0u;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p = r * 64 + lane;
    if (p < T) atomicOr(&sord[wave][p / 3], (keys[r] & kTileIdBits) << (10 * (p % 3)));
  }
  __builtin_amdgcn_wave_barrier();
#endif
  bool stop = false;
#pragma unroll 1
  for (int base = 0; base < T && !stop; base += kWave) {
    const bool inr = base + lane < T;
#if DVCP_KNN_SORD
    const int pos = base + lane;
    const int tt = inr ? static_cast<int>((sord[wave][pos / 3] >> (10 * (pos % 3))) & kTileIdBits) : 0;
    const uint3 hb = hbox[tt];
    const uint32_t mykey = inr ? (__float_as_uint(hbox_lb2(hb, wl[0], wl[1], wl[2], wh[0], wh[1], wh[2])) &
                                  ~kTileIdBits) | static_cast<uint32_t>(tt)
                               : 0xFFFFFFFFu;  // lane i: sorted position base + i
#else
    const uint32_t mykey = keys[base >> 6];
    const int tt = inr ? static_cast<int>(mykey & kTileIdBits) : 0;
    const uint3 hb = hbox[tt < T ? tt : 0];
#endif
    const float klb = __uint_as_float(mykey & ~kTileIdBits);
    const uint64_t over = __ballot(!inr || klb > wkth);
    const int lim = over ? __builtin_ctzll(over) : kWave;  // positions past lim are never needed
    // the groups' k-th distances (largest per group) as of now
    float gk = kth;
#pragma unroll
    for (int off = kSubLanes / 2; off > 0; off >>= 1) gk = fmaxf(gk, __shfl_xor(gk, off, kWave));
    float gks[kKnnSub];
#pragma unroll
    for (int g = 0; g < kKnnSub; ++g) gks[g] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gk), g * kSubLanes));
    const float blx = half_lo(hb.x), bly = half_hi(hb.x), blz = half_lo(hb.y);
    const float bhx = half_hi(hb.y), bhy = half_lo(hb.z), bhz = half_hi(hb.z);
    bool pass = false;
#pragma unroll
    for (int g = 0; g < kKnnSub; ++g) {
      const float4 lo = sgbox[wave][g][0], hi = sgbox[wave][g][1];
      pass |= box_box_lb2(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, blx, bly, blz, bhx, bhy, bhz) <= gks[g];
    }
    uint64_t cand = __ballot(pass && inr) & (lim >= kWave ? ~0ull : ((1ull << lim) - 1ull));
    if (lim < kWave) stop = true;
    while (cand) {
      const int i = __builtin_ctzll(cand);
      cand &= cand - 1ull;
      const uint32_t key = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(mykey), i));
      if (__uint_as_float(key & ~kTileIdBits) > wkth) {  // every later tile is farther
        stop = true;
        break;
      }
      visit(key);
    }
  }
#else
  // one flat loop over the sorted tile order (not unrolled over the key registers: the merge is
  // large, and the key register is a wave-uniform indexed read)
  uint32_t key_next = T > 0 ? static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(keys[0]), 0)) : 0u;
#pragma unroll 1
  for (int pos = 0; pos < T; ++pos) {
#ifdef DVCP_KNN_DIAG
    {
      const uint64_t now = __builtin_readcyclecounter();
      if (dg_kind == 0) dg_skip_clk += now - dg_prev;
      dg_prev = now;
      dg_kind = 0;
    }
#endif
    const uint32_t key = key_next;
    if (pos + 1 < T)
      key_next = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(keys[(pos + 1) >> 6]), (pos + 1) & 63));
    if (__uint_as_float(key & ~kTileIdBits) > wkth) break;  // every later tile is farther
    visit(key);
  }
#endif
  merge();
#ifdef DVCP_KNN_DIAG
  const uint64_t dg_total = __builtin_readcyclecounter() - dg_t0;
  uint32_t app_sum = static_cast<uint32_t>(dg_appends);
  for (int off = 32; off > 0; off >>= 1) app_sum += __shfl_xor(app_sum, off, kWave);
#endif
#ifndef DVCP_KNN_DIAG
  if constexpr (DVCP_KNN_STAGE_OUT == 2) {
    if (dist && idx && !idx64 && k == KT) {
      // each lane writes its own 128-B rows as eight 16-byte stores (whole lines per lane)
      if (!live) return;
      const int qo = out_row();
      float4* dr = reinterpret_cast<float4*>(dist + (static_cast<int64_t>(b) * Q + qo) * 32);
      int4* ir = reinterpret_cast<int4*>(idx + (static_cast<int64_t>(b) * Q + qo) * 32);
#pragma unroll
      for (int v = 0; v < KT / 4; ++v) {
        float dv[4];
        int iv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double kv = tk[4 * v + e];
          const bool ok = kv != kKeyEmpty;
          dv[e] = ok ? sqrt_rn(key_d2(kv)) : __builtin_huge_valf();
          iv[e] = ok ? key_index(kv) : -1;
        }
        dr[v] = make_float4(dv[0], dv[1], dv[2], dv[3]);
        ir[v] = make_int4(iv[0], iv[1], iv[2], iv[3]);
      }
      return;
    }
  }
  if constexpr (DVCP_KNN_STAGE_OUT == 1) {
    if (dist && idx && !idx64 && k == KT) {
      // Coalesced output rows (the forward's case).  Each lane's query row is 128 B of distances
      // and 128 B of indices at a scattered position (queries run in curve order); stored straight
      // from the lanes, every store instruction touches 64 lines with 4 bytes each.  Instead the
      // rows go through the wave's candidate buffer in LDS, 32 at a time, and eight lanes store a
      // row as 16-byte pieces: each instruction writes eight whole lines.
      const int qo = live ? out_row() : -1;
      float* stage = reinterpret_cast<float*>(sbuf[wave]);             // 32 rows x 33 (4.2 KB of 8)
#pragma unroll
      for (int part = 0; part < 2; ++part) {      // 0: distances, 1: indices
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          if ((lane >> 5) == half) {
#pragma unroll
            for (int t = 0; t < KT; ++t) {
              const bool ok = tk[t] != kKeyEmpty;  // fewer than k finite points
              const float v = part == 0 ? (ok ? sqrt_rn(key_d2(tk[t])) : __builtin_huge_valf())
                                        : __int_as_float(ok ? key_index(tk[t]) : -1);
              stage[(lane & 31) * 33 + t] = v;     // (row stride 33: no bank conflicts)
            }
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int row = it * 8 + (lane >> 3), piece = lane & 7;
            const int rq = __shfl(qo, half * 32 + row, kWave);
            const float* sr = stage + row * 33 + 4 * piece;
            const float4 v = make_float4(sr[0], sr[1], sr[2], sr[3]);
            if (rq >= 0) {
              float* dst = part == 0 ? dist : reinterpret_cast<float*>(idx);
              reinterpret_cast<float4*>(dst + (static_cast<int64_t>(b) * Q + rq) * 32)[piece] = v;
            }
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
      }
      return;
    }
  }
#endif
  if (!live) return;
  // the query's output row (its index re-read: held across the scan it was spilled)
  const int qo = out_row();
  const int64_t o = (static_cast<int64_t>(b) * Q + qo) * k;
#ifdef DVCP_KNN_DIAG
  if (lane == 0 && dist && k == 32) {
    dist[o + 0] = static_cast<float>(dg_scanned);
    dist[o + 1] = static_cast<float>(dg_active);
    dist[o + 2] = static_cast<float>(dg_merges);
    dist[o + 3] = static_cast<float>(app_sum);
    dist[o + 4] = static_cast<float>(dg_total);
    dist[o + 5] = static_cast<float>(dg_merge_clk);
    dist[o + 6] = static_cast<float>(dg_skip_clk);
    dist[o + 31] = -12345.0f;
    return;
  }
#endif
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    if (t < k) {
      const bool ok = tk[t] != kKeyEmpty;  // fewer than k finite points
      const float d2 = key_d2(tk[t]);
      const int i = key_index(tk[t]);
      if (dist) dist[o + t] = ok ? sqrt_rn(d2) : __builtin_huge_valf();
      if (idx) idx[o + t] = ok ? i : -1;
      if (idx64) idx64[o + t] = ok ? i : -1;
    }
  }
}

}  // namespace dvcp

extern "C" int64_t dvcp_knn_tiled_workspace_bytes(int B, int M, int Q) {
  if (B < 0 || M < 0 || Q < 0) return -1;
  const int64_t T = dvcp::ceil_div(M, dvcp::kTile);
  return dvcp::align256(16 * int64_t(B) * T * dvcp::kTile) + dvcp::align256(32 * int64_t(B) * T) +
         dvcp::align256(16 * int64_t(B) * Q) + dvcp::align256(dvcp::tiled_zeroed_bytes(B));
}

static int knn_tiled_impl(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M, const void* qry,
                          int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k, void* workspace, float* dist,
                          int32_t* idx, int64_t* idx64, void* stream, bool insertion) {
  DVCP_REQUIRE(ref && qry && workspace, "dvcp_knn_tiled: null pointer");
  DVCP_REQUIRE(k > 0 && k <= 32 && M >= 0 && Q >= 0 && B >= 0 && B <= 65535, "dvcp_knn_tiled: bad sizes");
  DVCP_REQUIRE(M <= dvcp::kMaxTiles * dvcp::kTile, "dvcp_knn_tiled: M=%d > %d", M, dvcp::kMaxTiles * dvcp::kTile);
  DVCP_REQUIRE(dtype == DVCP_F32 || dtype == DVCP_F64, "dvcp_knn_tiled: bad dtype %d", dtype);
  if (B == 0 || Q == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dvcp::TiledLayout L = dvcp::tiled_layout(workspace, B, M, Q);
  // queries: bounding box, cell counts, scan, then the scatter beside the reference build
  if (hipMemsetAsync(L.qbins, 0, dvcp::tiled_zeroed_bytes(B), st) != hipSuccess) {
    dvcp::set_error("dvcp_knn_tiled: memset failed");
    return DVCP_EHIP;
  }
  const dim3 qgrid(dvcp::ceil_div(Q, dvcp::kQSortItems), B), bgrid(1 + qgrid.x, B);
  if (dtype == DVCP_F32) {
    const dvcp::PointsView<float> qv{static_cast<const float*>(qry), qb, qc, qn};
    hipLaunchKernelGGL((dvcp::knn_qbox_kernel<float>), qgrid, dim3(dvcp::kBuildThreads), 0, st, qv, Q, L.qbox);
    hipLaunchKernelGGL((dvcp::knn_qhist_kernel<float>), qgrid, dim3(dvcp::kBuildThreads), 0, st, qv, Q, L.qbox,
                       L.qbins);
    hipLaunchKernelGGL(dvcp::knn_qscan_kernel, dim3(B), dim3(dvcp::kBuildThreads), 0, st, L.qbins);
    hipLaunchKernelGGL((dvcp::knn_tiled_build_kernel<float>), bgrid, dim3(dvcp::kBuildThreads), 0, st,
                       dvcp::PointsView<float>{static_cast<const float*>(ref), rb, rc, rn}, M, qv, Q, L);
  } else {
    const dvcp::PointsView<double> qv{static_cast<const double*>(qry), qb, qc, qn};
    hipLaunchKernelGGL((dvcp::knn_qbox_kernel<double>), qgrid, dim3(dvcp::kBuildThreads), 0, st, qv, Q, L.qbox);
    hipLaunchKernelGGL((dvcp::knn_qhist_kernel<double>), qgrid, dim3(dvcp::kBuildThreads), 0, st, qv, Q, L.qbox,
                       L.qbins);
    hipLaunchKernelGGL(dvcp::knn_qscan_kernel, dim3(B), dim3(dvcp::kBuildThreads), 0, st, L.qbins);
    hipLaunchKernelGGL((dvcp::knn_tiled_build_kernel<double>), bgrid, dim3(dvcp::kBuildThreads), 0, st,
                       dvcp::PointsView<double>{static_cast<const double*>(ref), rb, rc, rn}, M, qv, Q, L);
  }
  if (int e = dvcp::launch_status("dvcp_knn_tiled(build)")) return e;
  const int T = dvcp::ceil_div(M, dvcp::kTile);
  dim3 grid(dvcp::ceil_div(Q, dvcp::kTiledThreads), B);
  const int xcd = B % 8 == 0 ? 1 : 0;  // XCD-aware cloud mapping (equal clouds per XCD)
  // k = 17..32 (the forward's 32): the buffered-selection kernel
#define DVCP_KNNS(RR)                                                                                             \
  if (k > 16 && T <= 64 * RR) {                                                                                   \
    hipLaunchKernelGGL((dvcp::knn_sel_query_kernel<RR>), grid, dim3(dvcp::kTiledThreads), 0, st, L.sorted,         \
                       L.tbox, L.qsorted, M, Q, k, dist, idx, idx64, xcd);                                         \
    return dvcp::launch_status("dvcp_knn_tiled(select)");                                                         \
  }
  if (!insertion) {
    DVCP_KNNS(1)
    DVCP_KNNS(2)
    DVCP_KNNS(4)
    DVCP_KNNS(8)
    DVCP_KNNS(16)
  }
#undef DVCP_KNNS
#define DVCP_KNNT(KK, RR)                                                                                          \
  if (k <= KK && T <= 64 * RR) {                                                                                   \
    hipLaunchKernelGGL((dvcp::knn_tiled_query_kernel<KK, RR>), grid, dim3(dvcp::kTiledThreads), 0, st, L.sorted,   \
                       L.tbox, L.qsorted, M, Q, k, dist, idx, idx64, xcd);                                          \
    return dvcp::launch_status("dvcp_knn_tiled(query)");                                                           \
  }
  DVCP_KNNT(1, 1)
  DVCP_KNNT(1, 16)
  DVCP_KNNT(8, 1)
  DVCP_KNNT(8, 16)
  DVCP_KNNT(16, 16)
  DVCP_KNNT(32, 1)
  DVCP_KNNT(32, 2)
  DVCP_KNNT(32, 4)
  DVCP_KNNT(32, 8)
  DVCP_KNNT(32, 16)
#undef DVCP_KNNT
  dvcp::set_error("dvcp_knn_tiled: unsupported k=%d", k);
  return DVCP_EINVAL;
}

extern "C" int dvcp_knn_tiled(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M, const void* qry,
                              int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k, void* workspace, float* dist,
                              int32_t* idx, int64_t* idx64, void* stream) {
  return knn_tiled_impl(dtype, ref, rb, rc, rn, M, qry, qb, qc, qn, Q, B, k, workspace, dist, idx, idx64, stream, false);
}

// The same tiled scan with the per-candidate insertion network for every k (the round-2 kernel):
// kept as a second exact implementation for the parity tests and A/B timing.
extern "C" int dvcp_knn_tiled_insert(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M,
                                     const void* qry, int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k,
                                     void* workspace, float* dist, int32_t* idx, int64_t* idx64, void* stream) {
  return knn_tiled_impl(dtype, ref, rb, rc, rn, M, qry, qb, qc, qn, Q, B, k, workspace, dist, idx, idx64, stream, true);
}
