// ball_query.hip -- pointnet2_utils.py:87-107 query_ball_point (+ :19-40 square_distance).
//
// The reference materialises the S x N expansion-form distance matrix, masks it, and
// fully sorts every row (O(S*N) memory, an N-element sort per centre).  Here one lane owns
// one centre and scans the points in ascending index order, appending hits until
// `nsample` are found -- the same "first nsample ascending indices in radius" set with no
// sort and no S x N buffer.  The workgroup's 256 centres share each point tile through LDS
// (a broadcast read per point) and the workgroup stops as soon as all of its lanes are full.
//
// Rounding matches the reference exactly: d2 = ((-2*dot) + |c|^2) + |p|^2 with
// dot = MKL's fma chain and |.|^2 without fma; the radius test is `!(d2 > fp(r^2))` (:102).
#include "common.h"
#include "morton.h"


namespace dvcp {

template <typename T>
struct alignas(16) PointSS {
  T x, y, z, ss;
};

constexpr int kBqThreads = 256;

template <typename T>
__global__ __launch_bounds__(kBqThreads) void ball_query_kernel(
    PointsView<T> pts, int N, PointsView<T> ctr, int S, T r2, int nsample,
    int32_t* __restrict__ count, int32_t* __restrict__ list, int64_t* __restrict__ padded) {
  constexpr int TILE = (sizeof(T) == 4) ? 1024 : 512;
  __shared__ PointSS<T> tile[TILE];
  const int b = blockIdx.y;
  const int s = blockIdx.x * kBqThreads + threadIdx.x;
  const bool live = s < S;
  T cx = 0, cy = 0, cz = 0;
  if (live) {
    cx = ctr.at(b, 0, s);
    cy = ctr.at(b, 1, s);
    cz = ctr.at(b, 2, s);
  }
  const T ssc = sumsq3(cx, cy, cz);
  const int64_t row = (static_cast<int64_t>(b) * S + s) * nsample;
  int32_t* my_list = list ? list + row : nullptr;
  int64_t* my_pad = padded ? padded + row : nullptr;
  int cnt = 0;
  int first = N;  // reference: a centre with no hit is padded with index N
  bool done = !live;

  for (int t0 = 0; t0 < N; t0 += TILE) {
    const int nt = min(TILE, N - t0);
    __syncthreads();
    for (int j = threadIdx.x; j < nt; j += kBqThreads) {
      const T x = pts.at(b, 0, t0 + j), y = pts.at(b, 1, t0 + j), z = pts.at(b, 2, t0 + j);
      tile[j] = PointSS<T>{x, y, z, sumsq3(x, y, z)};
    }
    __syncthreads();
    if (!done) {
      for (int j = 0; j < nt; ++j) {
        const PointSS<T> p = tile[j];
        const T d2 = expansion_d2(dot3_blas(cx, cy, cz, p.x, p.y, p.z), ssc, p.ss);
        if (!(d2 > r2)) {
          const int n = t0 + j;
          if (cnt == 0) first = n;
          if (my_list) my_list[cnt] = n;
          if (my_pad) my_pad[cnt] = n;
          if (++cnt == nsample) {
            done = true;
            break;
          }
        }
      }
    }
    if (__syncthreads_and(done)) break;
  }
  if (!live) return;
  if (count) count[static_cast<int64_t>(b) * S + s] = cnt;
  if (my_list && cnt == 0) my_list[0] = 0;  // (see bq_tiled_kernel)
  if (my_pad)
    for (int j = cnt; j < nsample; ++j) my_pad[j] = first;
}

// ---------------------------------------------------------------------------------------------
// fp32 paths.  Both produce exactly the index-order result above.
//
// bq_wave_kernel (any N): one wave = 64 centres with its own early exit; points are streamed in
// ascending index order as wave-uniform scalar loads of packed (x, y, z, |p|^2) rows.
//
// bq_tiled_kernel (N <= 65536): a sparse radius (most centres far from nsample hits) makes the
// scan above visit every point for every centre.  bq_build_kernel sorts the points along a Hilbert curve into
// 64-point tiles with boxes and the centres into a Hilbert permutation, so a wave's 64 centres
// have a compact box.  The wave marks, in an LDS bitmap indexed by ORIGINAL point index, every
// point whose distance bound to the wave box passes the radius with a rounding margin, then
// scans the set bits in ascending index order with the same test, append rule and early exit.
// A point left out of the bitmap provably fails the reference's test (see bq_prune_thr), so the
// result is identical, and the scan touches only the neighbourhood of the wave.

// Rows are padded to a multiple of 16 points (zeros) so every 16-point chunk of the wave scan is
// one unconditional scalar burst; the padding never hits because the loop tests n < N.
__host__ __device__ constexpr int bq_padded_n(int N) { return (N + 15) & ~15; }

constexpr int kBqTile = 64;
// DVCP_BQ_ABL (timing experiments only, wrong results): 1 the list stores of the tiled scan skipped
#ifndef DVCP_BQ_ABL
#define DVCP_BQ_ABL 0
#endif
constexpr int kBqMaxTiles = 1024;             // tiled path: N <= 65536
constexpr int kBqSmallTiles = 256;            // N <= 16384: the small-bitmap instantiation (occupancy)
constexpr int kBqCap = 256;                   // candidate points staged in LDS per round

struct BqLayout {
  float4* packed;   // B x Npad: x, y, z, |p|^2 in original order (zero padding)
  float4* sorted;   // B x T*64: x, y, z, original index bits (padding: NaN, 0x7FFFFFFF)
  float4* tbox;     // B x T x 2: lo.xyz, hi.xyz (non-finite member: the whole space)
  int32_t* cperm;   // B x S: centre index by Hilbert position
};

inline int64_t bq_align(int64_t x) { return (x + 255) & ~int64_t(255); }

inline BqLayout bq_layout(void* ws, int B, int N, int S) {
  const int64_t T = ceil_div(N, kBqTile);
  char* p = static_cast<char*>(ws);
  BqLayout L;
  L.packed = reinterpret_cast<float4*>(p);
  p += bq_align(16 * int64_t(B) * bq_padded_n(N));
  L.sorted = reinterpret_cast<float4*>(p);
  p += bq_align(16 * int64_t(B) * T * kBqTile);
  L.tbox = reinterpret_cast<float4*>(p);
  p += bq_align(32 * int64_t(B) * T);
  L.cperm = reinterpret_cast<int32_t*>(p);
  return L;
}

inline int64_t bq_workspace_bytes(int B, int N, int S) {
  const int64_t T = ceil_div(N, kBqTile);
  return bq_align(16 * int64_t(B) * bq_padded_n(N)) + bq_align(16 * int64_t(B) * T * kBqTile) +
         bq_align(32 * int64_t(B) * T) + bq_align(4 * int64_t(B) * S);
}

__global__ void bq_pack_kernel(PointsView<float> pts, int N, float4* __restrict__ packed) {
  const int b = blockIdx.y;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int np = bq_padded_n(N);
  if (n >= np) return;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    const float x = pts.at(b, 0, n), y = pts.at(b, 1, n), z = pts.at(b, 2, n);
    v = make_float4(x, y, z, sumsq3(x, y, z));
  }
  packed[static_cast<int64_t>(b) * np + n] = v;
}

// Two workgroups per cloud: packed rows and point tiles with boxes; the centres' Hilbert permutation.
__global__ __launch_bounds__(kBuildThreads) void bq_build_kernel(PointsView<float> pts, int N, PointsView<float> ctr,
                                                                 int S, BqLayout L, int tiled) {
  __shared__ uint32_t bins[kSortBins];
  __shared__ uint32_t boxk[kBqMaxTiles][6];  // float_order keys: lo.xyz (min), hi.xyz (max)
  __shared__ uint32_t wsum[16];
  __shared__ float red[2][3][16];
  const int b = blockIdx.y, tid = threadIdx.x;
  auto get_ctr = [&](int i, float (&v)[3]) {
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] = ctr.at(b, a, i);
  };
  float lo[3], hi[3];
  if (blockIdx.x == 1) {  // the centres' curve order, beside the point work of block 0
    block_bbox(S, get_ctr, lo, hi, red);
    int32_t* cp = L.cperm + static_cast<int64_t>(b) * S;
    morton_sort(
        S, get_ctr, [&](int pos, int i, const float (&)[3]) { cp[pos] = i; }, lo, hi, bins, wsum);
    return;
  }
  const int np = bq_padded_n(N);
  float4* pk = L.packed + static_cast<int64_t>(b) * np;
  for (int i = tid; i < np; i += kBuildThreads) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < N) {
      const float x = pts.at(b, 0, i), y = pts.at(b, 1, i), z = pts.at(b, 2, i);
      v = make_float4(x, y, z, sumsq3(x, y, z));
    }
    pk[i] = v;
  }
  if (!tiled) return;
  const int T = (N + kBqTile - 1) / kBqTile;
  float4* so = L.sorted + static_cast<int64_t>(b) * T * kBqTile;
  for (int i = tid; i < T * 6; i += kBuildThreads) boxk[i / 6][i % 6] = (i % 6) < 3 ? 0xFFFFFFFFu : 0u;
  auto get_pt = [&](int i, float (&v)[3]) {
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] = pts.at(b, a, i);
  };
  block_bbox(N, get_pt, lo, hi, red);
  morton_sort(
      N, get_pt,
      [&](int pos, int i, const float (&v)[3]) {
        so[pos] = make_float4(v[0], v[1], v[2], __int_as_float(i));
        const int t = pos / kBqTile;
        // a non-finite coordinate can pass the reference's test against any centre (NaN d2
        // is not > r^2), so its tile must never be pruned: give it the whole space
        const bool fin = __builtin_isfinite(v[0]) && __builtin_isfinite(v[1]) && __builtin_isfinite(v[2]);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          atomicMin(&boxk[t][a], float_order(fin ? v[a] : -__builtin_huge_valf()));
          atomicMax(&boxk[t][3 + a], float_order(fin ? v[a] : __builtin_huge_valf()));
        }
      },
      lo, hi, bins, wsum);
  for (int pos = N + tid; pos < T * kBqTile; pos += kBuildThreads)
    so[pos] = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __int_as_float(0x7FFFFFFF));
  for (int t = tid; t < T; t += kBuildThreads) {
    float4* tb = L.tbox + (static_cast<int64_t>(b) * T + t) * 2;
    tb[0] = make_float4(float_unorder(boxk[t][0]), float_unorder(boxk[t][1]), float_unorder(boxk[t][2]), 0.f);
    tb[1] = make_float4(float_unorder(boxk[t][3]), float_unorder(boxk[t][4]), float_unorder(boxk[t][5]), 0.f);
  }
}

__global__ __launch_bounds__(256) void bq_wave_kernel(const float4* __restrict__ packed, int N, PointsView<float> ctr,
                                                      int S, float r2, int nsample, int32_t* __restrict__ count,
                                                      int32_t* __restrict__ list, int64_t* __restrict__ padded) {
  const int b = blockIdx.y;
  const int s = blockIdx.x * 256 + threadIdx.x;
  if ((blockIdx.x * 256 + (threadIdx.x & ~63)) >= S) return;  // whole wave past the end
  const bool live = s < S;
  float cx = 0.f, cy = 0.f, cz = 0.f;
  if (live) {
    cx = ctr.at(b, 0, s);
    cy = ctr.at(b, 1, s);
    cz = ctr.at(b, 2, s);
  }
  const float ssc = sumsq3(cx, cy, cz);
  const int64_t row = (static_cast<int64_t>(b) * S + s) * nsample;
  int cnt = live ? 0 : nsample;
  int first = N;
  const const_float* P = (const const_float*)uniform_ptr(packed + static_cast<int64_t>(b) * bq_padded_n(N));
  for (int n0 = 0; n0 < N; n0 += 16) {
    float c[64];
#pragma unroll
    for (int u = 0; u < 64; ++u) c[u] = P[4 * n0 + u];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = n0 + j;
      const float d2 = expansion_d2(dot3_blas(cx, cy, cz, c[4 * j], c[4 * j + 1], c[4 * j + 2]), ssc, c[4 * j + 3]);
      if ((n < N) & !(d2 > r2) & (cnt < nsample)) {
        first = cnt == 0 ? n : first;
        if (list) list[row + cnt] = n;
        if (padded) padded[row + cnt] = n;
        ++cnt;
      }
    }
    if (__ballot(cnt < nsample) == 0) break;
  }
  if (!live) return;
  if (count) count[static_cast<int64_t>(b) * S + s] = cnt;
  if (list && cnt == 0) list[row] = 0;  // (see bq_tiled_kernel)
  if (padded)
    for (int j = cnt; j < nsample; ++j) padded[row + j] = first;
}

__device__ __forceinline__ float wave_fmin(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ float wave_fmax(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Prune threshold.  The reference's d2 = ((-2 dot) + |c|^2) + |p|^2 (dot an fma chain) differs
// from the exact squared distance by at most ~10 u (|c|^2 + |p|^2) (u = 2^-24; each of the six
// roundings is bounded by u times a magnitude <= 2 (|c|^2 + |p|^2)); a gap-based box bound
// computed in fp32 exceeds the exact bound by at most (1 + 2^-20).  A point whose computed bound
// exceeds (r^2 + 16 u (|c|^2max + |p|^2max)) (1 + 2^-19) therefore has computed d2 > r^2.
__device__ __forceinline__ float bq_prune_thr(float r2, float ssc_max, float ssp_max) {
  return (r2 + 0x1p-20f * (ssc_max + ssp_max)) * (1.0f + 0x1p-19f);
}

// |p|^2 upper bound over a box (per axis the larger endpoint magnitude)
__device__ __forceinline__ float box_ss_max(float lx, float ly, float lz, float hx, float hy, float hz) {
  const float ax = fmaxf(fabsf(lx), fabsf(hx)), ay = fmaxf(fabsf(ly), fabsf(hy)), az = fmaxf(fabsf(lz), fabsf(hz));
  return ((ax * ax + ay * ay) + az * az) * (1.0f + 0x1p-20f);
}

__device__ __forceinline__ float bq_gap(float lo, float hi, float v_lo, float v_hi) {
  return fmaxf(fmaxf(v_lo - hi, lo - v_hi), 0.0f);
}

// MAXT bounds the tile count; the per-wave bitmap holds MAXT * 2 words (one bit per point).
template <int MAXT>
__global__ __launch_bounds__(256) void bq_tiled_kernel(BqLayout L, int N, PointsView<float> ctr, int S, float r2,
                                                       int nsample, int32_t* __restrict__ count,
                                                       int32_t* __restrict__ list, int64_t* __restrict__ padded,
                                                       int xcd) {
  __shared__ uint32_t bm[4][MAXT * 2];
  __shared__ float4 cpt[4][kBqCap];
  __shared__ int32_t cid[4][kBqCap];
  // cloud and block within it; xcd != 0 (B % 8 == 0): workgroups reach the XCDs round robin by
  // linear id, which is re-mapped so XCD x takes clouds x, x + 8, ... (one cloud's tiles and rows
  // per L2)
  int b = blockIdx.y, bx = blockIdx.x;
  if (xcd) {
    const int lin = static_cast<int>(blockIdx.y * gridDim.x + blockIdx.x);
    const int slot = lin >> 3;
    b = (lin & 7) + 8 * (slot / static_cast<int>(gridDim.x));
    bx = slot % static_cast<int>(gridDim.x);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q0 = (bx * 4 + wave) * 64;
  if (q0 >= S) return;
  const int T = (N + kBqTile - 1) / kBqTile;
  const int NW = (N + 31) >> 5;
  const int np = bq_padded_n(N);
  const bool live = q0 + lane < S;
  const int s = live ? L.cperm[static_cast<int64_t>(b) * S + q0 + lane] : 0;
  float cx = 0.f, cy = 0.f, cz = 0.f;
  if (live) {
    cx = ctr.at(b, 0, s);
    cy = ctr.at(b, 1, s);
    cz = ctr.at(b, 2, s);
  }
  const float ssc = sumsq3(cx, cy, cz);
  const bool fin = __builtin_isfinite(cx) && __builtin_isfinite(cy) && __builtin_isfinite(cz);
  const float inf = __builtin_huge_valf();
  // Lane groups.  A run of 64 curve-consecutive centres can straddle a jump of the curve (a few
  // lanes' centres far from the rest): its box, and so the candidate union every lane scans, is
  // then many times that of either part, and such waves set the kernel's duration (C3: median
  // wave ~60 us, the slowest ~300 us with 10x the median's candidates, all in clouds with
  // outliers).  The wave therefore looks for the best single cut of its lane range (the split
  // minimising the summed r-expanded box volumes, by prefix and suffix box scans), keeps it when
  // it saves 30 %, and tries once more inside each part: up to four lane groups, each running the
  // bitmap pass and the scan for its own box while the other lanes idle.  A centre's list
  // depends only on its own tests, so the grouping never changes a result.
  int cut1 = -1, cut2 = -1, cut3 = -1;
  if (__ballot(live && !fin) == 0) {  // (a non-finite centre needs every point anyway)
    const float rr2 = 2.0f * sqrtf(r2);
    const bool bl = live;
    auto box_vol = [&](const float (&lo)[3], const float (&hi)[3]) {
      return !(hi[0] >= lo[0]) ? 0.0f : ((hi[0] - lo[0] + rr2) * (hi[1] - lo[1] + rr2)) * (hi[2] - lo[2] + rr2);
    };
    // the best single cut of lanes [a, e): the first lane of the second part, or -1
    auto best_cut = [&](int a, int e) -> int {
      const bool in = bl && lane >= a && lane < e;
      const float c3[3] = {cx, cy, cz};
      float plo[3], phi[3], slo[3], shi[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        plo[d] = slo[d] = in ? c3[d] : inf;
        phi[d] = shi[d] = in ? c3[d] : -inf;
      }
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const float ul = __shfl_up(plo[d], off, kWave), uh = __shfl_up(phi[d], off, kWave);
          const float dl = __shfl_down(slo[d], off, kWave), dh = __shfl_down(shi[d], off, kWave);
          if (lane >= off) {
            plo[d] = fminf(plo[d], ul);
            phi[d] = fmaxf(phi[d], uh);
          }
          if (lane + off < 64) {
            slo[d] = fminf(slo[d], dl);
            shi[d] = fmaxf(shi[d], dh);
          }
        }
      }
      const float vp = box_vol(plo, phi);  // lanes a..lane
      const float vs = box_vol(slo, shi);  // lanes lane..e-1
      const float vprev = __shfl_up(vp, 1, kWave);
      const float whole = __shfl(vp, 63, kWave);
      const float cost = (lane > a && lane < e) ? vprev + vs : inf;
      float m = cost;
      for (int off = 32; off > 0; off >>= 1) m = fminf(m, __shfl_xor(m, off, kWave));
      if (!(m < 0.7f * whole)) return -1;
      return static_cast<int>(__builtin_ctzll(__ballot(cost == m)));
    };
    cut1 = best_cut(0, 64);
    if (cut1 > 0) {
      cut2 = best_cut(0, cut1);
      cut3 = best_cut(cut1, 64);
    }
  }
  const int ngroups = 1 + (cut1 >= 0) + (cut2 >= 0) + (cut3 >= 0);
  const int gid = (cut2 >= 0 && lane >= cut2) + (cut1 >= 0 && lane >= cut1) + (cut3 >= 0 && lane >= cut3);
  uint32_t* mybm = bm[wave];
  const float4* tb = L.tbox + static_cast<int64_t>(b) * T * 2;
  const float4* so = L.sorted + static_cast<int64_t>(b) * T * kBqTile;
  const float4* pk = L.packed + static_cast<int64_t>(b) * np;
  const int64_t row = (static_cast<int64_t>(b) * S + s) * nsample;
  int cnt = live ? 0 : nsample;
  int first = N;
  float4* mypt = cpt[wave];
  int32_t* myid = cid[wave];
  for (int g = 0; g < ngroups; ++g) {
    const bool act = live && gid == g;
    if (__ballot(act) == 0) continue;
    // the group's box; a non-finite centre needs every point
    const float wlx = wave_fmin(act ? (fin ? cx : -inf) : inf), whx = wave_fmax(act ? (fin ? cx : inf) : -inf);
    const float wly = wave_fmin(act ? (fin ? cy : -inf) : inf), why = wave_fmax(act ? (fin ? cy : inf) : -inf);
    const float wlz = wave_fmin(act ? (fin ? cz : -inf) : inf), whz = wave_fmax(act ? (fin ? cz : inf) : -inf);
    const float ssc_max = wave_fmax(act && fin ? ssc : 0.0f);

    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < NW; i += 64) mybm[i] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + lane;
      bool cand = false;
      if (t < T) {
        const float4 lo = tb[2 * t], hi = tb[2 * t + 1];
        const float gx = bq_gap(lo.x, hi.x, wlx, whx), gy = bq_gap(lo.y, hi.y, wly, why), gz = bq_gap(lo.z, hi.z, wlz, whz);
        const float lb2 = (gx * gx + gy * gy) + gz * gz;
        cand = !(lb2 > bq_prune_thr(r2, ssc_max, box_ss_max(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z)));
      }
      uint64_t mask = __ballot(cand);
      while (mask) {
        // up to four candidate tiles per pass, their loads in flight together
        int tt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          tt[u] = mask ? t0 + __builtin_ctzll(mask) : -1;
          mask &= mask - 1;
        }
        float4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = so[max(tt[u], 0) * kBqTile + lane];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = __float_as_int(q[u].w);
          const float gx = bq_gap(q[u].x, q[u].x, wlx, whx), gy = bq_gap(q[u].y, q[u].y, wly, why),
                      gz = bq_gap(q[u].z, q[u].z, wlz, whz);
          const float lb2 = (gx * gx + gy * gy) + gz * gz;
          const float ssp = ((q[u].x * q[u].x + q[u].y * q[u].y) + q[u].z * q[u].z) * (1.0f + 0x1p-20f);
          // NaN coordinates give NaN bounds, which are kept (never "> thr")
          if (tt[u] >= 0 && idx < N && !(lb2 > bq_prune_thr(r2, ssc_max, ssp)))
            atomicOr(&mybm[idx >> 5], 1u << (idx & 31));
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();

    for (int c0 = 0; c0 < NW; c0 += 64) {
      const uint32_t word = (c0 + lane < NW) ? mybm[c0 + lane] : 0u;
      const int pc = __builtin_popcount(word);
      int incl = pc;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += u;
      }
      const int total = __shfl(incl, 63, kWave);
      const int excl = incl - pc;
      for (int base = 0; base < total; base += kBqCap) {
        // this round's candidates (positions [base, base + kBqCap) in index order): indices first,
        // then the points gathered cooperatively (several loads in flight per lane)
        int p = excl;
        uint32_t wd = word;
        while (wd && p < base + kBqCap) {
          const int bit = __builtin_ctz(wd);
          wd &= wd - 1;
          if (p >= base) myid[p - base] = (c0 + lane) * 32 + bit;
          ++p;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int nc = min(kBqCap, total - base);
#pragma unroll
        for (int u = 0; u < kBqCap / 64; ++u) {
          const int j = u * 64 + lane;
          if (j < nc) mypt[j] = pk[myid[j]];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int j0 = 0; j0 < nc; j0 += 64) {
          const int je = min(nc, j0 + 64);
          for (int j1 = j0; j1 < je; j1 += 8) {
            float4 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) q[u] = mypt[j1 + u];  // j1 + 7 < kBqCap
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float d2 = expansion_d2(dot3_blas(cx, cy, cz, q[u].x, q[u].y, q[u].z), ssc, q[u].w);
              if (act & (j1 + u < je) & !(d2 > r2) & (cnt < nsample)) {
                const int n = myid[j1 + u];
                first = cnt == 0 ? n : first;
#if DVCP_BQ_ABL != 1
                if (list) list[row + cnt] = n;
#endif
                if (padded) padded[row + cnt] = n;
                ++cnt;
              }
            }
          }
          if (__ballot(act && cnt < nsample) == 0) goto group_done;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
  group_done:;
  }
  if (!live) return;
  if (count) count[static_cast<int64_t>(b) * S + s] = cnt;
  // A centre without hits (the reference pads it with index N, :104) gets a valid first list
  // entry, point 0: consumers that clamp count to >= 1 (training passes) then read in bounds, and
  // the forward MLP tables give such a centre a zero row without reading its list.
  if (list && cnt == 0) list[row] = 0;
  if (padded)
    for (int j = cnt; j < nsample; ++j) padded[row + j] = first;
}

template <typename T>
__global__ void square_distance_kernel(PointsView<T> src, int S, PointsView<T> dst, int N, T* __restrict__ out) {
  const int b = blockIdx.z;
  const int s = blockIdx.y;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const T sx = src.at(b, 0, s), sy = src.at(b, 1, s), sz = src.at(b, 2, s);
  const T dx = dst.at(b, 0, n), dy = dst.at(b, 1, n), dz = dst.at(b, 2, n);
  out[(static_cast<int64_t>(b) * S + s) * N + n] =
      expansion_d2(dot3_blas(sx, sy, sz, dx, dy, dz), sumsq3(sx, sy, sz), sumsq3(dx, dy, dz));
}

template <typename T>
static int launch_bq(const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const void* c, int64_t cb,
                     int64_t cc, int64_t cn, int S, int B, double radius, int nsample, int32_t* count,
                     int32_t* list, int64_t* padded, void* workspace, hipStream_t st) {
  PointsView<T> pv{static_cast<const T*>(xyz), sb, sc, sn};
  PointsView<T> cv{static_cast<const T*>(c), cb, cc, cn};
  // torch compares the fp32 tensor against the Python float radius**2 cast to fp32.
  const T r2 = static_cast<T>(radius * radius);
  if constexpr (sizeof(T) == 4) {
    if (workspace) {
      const BqLayout L = bq_layout(workspace, B, N, S);
      const int tiled = N <= kBqMaxTiles * kBqTile;
      hipLaunchKernelGGL(bq_build_kernel, dim3(tiled ? 2 : 1, B), dim3(kBuildThreads), 0, st, pv, N, cv, S, L, tiled);
      if (int e = launch_status("dvcp_ball_query(build)")) return e;
      if (tiled)
        hipLaunchKernelGGL(N <= kBqSmallTiles * kBqTile ? bq_tiled_kernel<kBqSmallTiles> : bq_tiled_kernel<kBqMaxTiles>,
                           dim3(ceil_div(S, 256), B), dim3(256), 0, st, L, N, cv, S, r2, nsample, count, list, padded,
                           B % 8 == 0 ? 1 : 0);
      else
        hipLaunchKernelGGL(bq_wave_kernel, dim3(ceil_div(S, 256), B), dim3(256), 0, st, L.packed, N, cv, S, r2,
                           nsample, count, list, padded);
      return launch_status("dvcp_ball_query");
    }
  }
  dim3 grid(ceil_div(S, kBqThreads), B);
  hipLaunchKernelGGL((ball_query_kernel<T>), grid, dim3(kBqThreads), 0, st, pv, N, cv, S, r2, nsample, count,
                     list, padded);
  return launch_status("dvcp_ball_query");
}

}  // namespace dvcp

extern "C" int dvcp_ball_query_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                  const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                                  double radius, int nsample, int32_t* count, int32_t* list,
                                  int64_t* padded, void* workspace, void* stream) {
  DVCP_REQUIRE(xyz && ctr, "dvcp_ball_query: null pointer");
  DVCP_REQUIRE(N >= 0 && S >= 0 && B >= 0 && nsample > 0, "dvcp_ball_query: bad sizes");
  if (B == 0 || S == 0) return DVCP_OK;
  DVCP_REQUIRE(B <= 65535, "dvcp_ball_query: B too large");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_bq<float>(xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B, radius, nsample, count, list,
                                  padded, workspace, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_bq<double>(xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B, radius, nsample, count, list,
                                   padded, nullptr, st);
  dvcp::set_error("dvcp_ball_query: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

extern "C" int64_t dvcp_ball_query_workspace_bytes(int B, int N, int S) {
  if (B < 0 || N < 0 || S < 0) return -1;
  return dvcp::bq_workspace_bytes(B, N, S);
}

extern "C" int dvcp_ball_query(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                               const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                               double radius, int nsample, int32_t* count, int32_t* list,
                               int64_t* padded, void* stream) {
  return dvcp_ball_query_ws(dtype, xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B, radius, nsample, count, list, padded,
                            nullptr, stream);
}

extern "C" int dvcp_square_distance(int dtype, const void* src, int64_t sb, int64_t sc, int64_t sn, int S,
                                    const void* dst, int64_t db, int64_t dc, int64_t dn, int N, int B,
                                    void* out, void* stream) {
  DVCP_REQUIRE(src && dst && out, "dvcp_square_distance: null pointer");
  if (B == 0 || S == 0 || N == 0) return DVCP_OK;
  DVCP_REQUIRE(S <= 65535 && B <= 65535, "dvcp_square_distance: S/B too large");
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(dvcp::ceil_div(N, 256), S, B);
  if (dtype == DVCP_F32) {
    hipLaunchKernelGGL((dvcp::square_distance_kernel<float>), grid, dim3(256), 0, st,
                       dvcp::PointsView<float>{static_cast<const float*>(src), sb, sc, sn}, S,
                       dvcp::PointsView<float>{static_cast<const float*>(dst), db, dc, dn}, N,
                       static_cast<float*>(out));
  } else if (dtype == DVCP_F64) {
    hipLaunchKernelGGL((dvcp::square_distance_kernel<double>), grid, dim3(256), 0, st,
                       dvcp::PointsView<double>{static_cast<const double*>(src), sb, sc, sn}, S,
                       dvcp::PointsView<double>{static_cast<const double*>(dst), db, dc, dn}, N,
                       static_cast<double*>(out));
  } else {
    dvcp::set_error("dvcp_square_distance: bad dtype %d", dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_square_distance");
}
