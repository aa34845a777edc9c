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

// ------------------------------------------------------------------------------------------
// Exact grid kNN.  The brute-force kernel above spends ~90% of its instructions in the divergent
// top-32 insertion (points arrive in index order, so a lane keeps inserting).  Here the
// reference set is counting-sorted into a uniform cell grid once per cloud, and each query scans
// Chebyshev shells of cells around its home cell -- roughly nearest first, so after the first
// shells insertions become rare.  Termination is exact: after shells 0..r, every unscanned point
// lies in a grid slab beyond the scanned cube; the search stops when the smallest distance to any
// such slab (shrunk by a rounding margin for the float cell assignment) exceeds the current k-th
// distance, so every point that could enter -- or tie -- the top k has been examined.  Ties are
// resolved by (d2, index) explicitly because cells are not in index order.
constexpr int kGridMaxCells = 16384;

struct KnnGridHeader {
  float bmin[3];
  float h;
  int dims[3];
  int ncell;
  float margin;
};

template <typename T>
__global__ __launch_bounds__(1024) void knn_grid_build_kernel(PointsView<T> ref, int M, KnnGridHeader* __restrict__ hdr,
                                                              int32_t* __restrict__ cell_start,
                                                              float4* __restrict__ sorted) {
  __shared__ uint32_t cnt[kGridMaxCells];
  __shared__ float red[2][3][16];
  __shared__ uint32_t wsum[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float lo[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
  float hi[3] = {-lo[0], -lo[1], -lo[2]};
  for (int n = tid; n < M; n += 1024)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float v = static_cast<float>(ref.at(b, a, n));
      lo[a] = fminf(lo[a], v);
      hi[a] = fmaxf(hi[a], v);
    }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    for (int off = 32; off > 0; off >>= 1) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off, kWave));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off, kWave));
    }
    if (lane == 0) {
      red[0][a][wave] = lo[a];
      red[1][a][wave] = hi[a];
    }
  }
  for (int i = tid; i < kGridMaxCells; i += 1024) cnt[i] = 0u;
  __syncthreads();
  float bmin[3], ext[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float l = red[0][a][0], h = red[1][a][0];
    for (int w = 1; w < 16; ++w) {
      l = fminf(l, red[0][a][w]);
      h = fmaxf(h, red[1][a][w]);
    }
    bmin[a] = l;
    ext[a] = h - l;
  }
  const float emax = fmaxf(fmaxf(ext[0], ext[1]), fmaxf(ext[2], 1e-30f));
  // ~2 points per cell over the bounding box; at most kGridMaxCells cells
  const float vol = fmaxf(ext[0], 1e-3f * emax) * fmaxf(ext[1], 1e-3f * emax) * fmaxf(ext[2], 1e-3f * emax);
  float h = cbrtf(vol * 2.0f / fmaxf(static_cast<float>(M), 1.0f));
  int dims[3];
  for (int it = 0; it < 8; ++it) {
    int prod = 1;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      dims[a] = min(64, max(1, static_cast<int>(ceilf(ext[a] / h))));
      prod *= dims[a];
    }
    if (prod <= kGridMaxCells) break;
    h *= 1.3f;
  }
  const int ncell = dims[0] * dims[1] * dims[2];
  const float inv_h = 1.0f / h;
  auto cell_of = [&](float x, float y, float z) -> int {
    const int cx = min(dims[0] - 1, max(0, static_cast<int>((x - bmin[0]) * inv_h)));
    const int cy = min(dims[1] - 1, max(0, static_cast<int>((y - bmin[1]) * inv_h)));
    const int cz = min(dims[2] - 1, max(0, static_cast<int>((z - bmin[2]) * inv_h)));
    return (cz * dims[1] + cy) * dims[0] + cx;
  };
  for (int n = tid; n < M; n += 1024)
    atomicAdd(&cnt[cell_of(static_cast<float>(ref.at(b, 0, n)), static_cast<float>(ref.at(b, 1, n)),
                          static_cast<float>(ref.at(b, 2, n)))], 1u);
  __syncthreads();
  {  // exclusive scan over ncell (<= 16384): 16 per thread
    uint32_t v[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = tid * 16 + k;
      v[k] = c < ncell ? cnt[c] : 0u;
      s += v[k];
    }
    uint32_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t u = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - s;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    int32_t* cs = cell_start + static_cast<int64_t>(b) * (kGridMaxCells + 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = tid * 16 + k;
      if (c < ncell) {
        cnt[c] = run;
        cs[c] = static_cast<int32_t>(run);
      }
      run += v[k];
    }
    if (tid == 0) cs[ncell] = M;
  }
  __syncthreads();
  float4* so = sorted + static_cast<int64_t>(b) * M;
  for (int n = tid; n < M; n += 1024) {
    const float x = static_cast<float>(ref.at(b, 0, n)), y = static_cast<float>(ref.at(b, 1, n)),
                z = static_cast<float>(ref.at(b, 2, n));
    so[atomicAdd(&cnt[cell_of(x, y, z)], 1u)] = make_float4(x, y, z, __int_as_float(n));
  }
  if (tid == 0) {
    KnnGridHeader g;
    for (int a = 0; a < 3; ++a) {
      g.bmin[a] = bmin[a];
      g.dims[a] = dims[a];
    }
    g.h = h;
    g.ncell = ncell;
    // float cell assignment may misplace a point by a few ulps of its coordinates
    g.margin = 8.0f * 1.2e-7f * (emax + fmaxf(fmaxf(fabsf(bmin[0]), fabsf(bmin[1])), fabsf(bmin[2])));
    hdr[b] = g;
  }
}

// kd/ki sorted by (d2, index); insert (d, i) in that order, dropping the last entry.
template <int KT>
__device__ __forceinline__ void topk_insert_lex(float (&kd)[KT], int (&ki)[KT], float d, int i) {
#pragma unroll
  for (int t = KT - 1; t > 0; --t) {
    const bool here = (d < kd[t]) | ((d == kd[t]) & (i < ki[t]));
    const bool before = (d < kd[t - 1]) | ((d == kd[t - 1]) & (i < ki[t - 1]));
    kd[t] = before ? kd[t - 1] : (here ? d : kd[t]);
    ki[t] = before ? ki[t - 1] : (here ? i : ki[t]);
  }
  const bool first = (d < kd[0]) | ((d == kd[0]) & (i < ki[0]));
  kd[0] = first ? d : kd[0];
  ki[0] = first ? i : ki[0];
}

__device__ __forceinline__ float axis_gap(float q, float lo, float hi) {
  return q < lo ? lo - q : (q > hi ? q - hi : 0.0f);
}

template <typename T, int KT>
__global__ __launch_bounds__(kKnnThreads) void knn_grid_query_kernel(const KnnGridHeader* __restrict__ hdr,
                                                                     const int32_t* __restrict__ cell_start,
                                                                     const float4* __restrict__ sorted, int M,
                                                                     PointsView<T> qry, int Q, int k,
                                                                     float* __restrict__ dist, int32_t* __restrict__ idx,
                                                                     int64_t* __restrict__ idx64) {
  __shared__ int32_t cs[kGridMaxCells + 1];  // this cloud's cell table (<= 64 KB)
  const int b = blockIdx.y;
  const int q = blockIdx.x * kKnnThreads + threadIdx.x;
  const KnnGridHeader g = hdr[b];
  const int32_t* csg = cell_start + static_cast<int64_t>(b) * (kGridMaxCells + 1);
  for (int c = threadIdx.x; c <= g.ncell; c += kKnnThreads) cs[c] = csg[c];
  __syncthreads();
  if (q >= Q) return;
  const float4* P = sorted + static_cast<int64_t>(b) * M;
  const float qv[3] = {static_cast<float>(qry.at(b, 0, q)), static_cast<float>(qry.at(b, 1, q)),
                       static_cast<float>(qry.at(b, 2, q))};
  float kd[KT];
  int ki[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    kd[t] = __builtin_huge_valf();
    ki[t] = 0x7FFFFFFF;
  }
  int home[3];
  float glo[3], ghi[3], gap[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    home[a] = min(g.dims[a] - 1, max(0, static_cast<int>(floorf((qv[a] - g.bmin[a]) / g.h))));
    glo[a] = g.bmin[a];
    ghi[a] = g.bmin[a] + g.dims[a] * g.h;
    gap[a] = axis_gap(qv[a], glo[a], ghi[a]);
  }
  const int rmax = max(max(g.dims[0], g.dims[1]), g.dims[2]);
  for (int r = 0; r <= rmax; ++r) {
    const int x0 = home[0] - r, x1 = home[0] + r, y0 = home[1] - r, y1 = home[1] + r, z0 = home[2] - r,
              z1 = home[2] + r;
    for (int cz = max(z0, 0); cz <= min(z1, g.dims[2] - 1); ++cz) {
      for (int cy = max(y0, 0); cy <= min(y1, g.dims[1] - 1); ++cy) {
        const bool face = cz == z0 || cz == z1 || cy == y0 || cy == y1;
        // interior rows of the shell only contribute their two x end cells
        const int step = face ? 1 : max(1, x1 - x0);
        for (int cx = x0; cx <= x1; cx += step) {
          if (cx < 0 || cx >= g.dims[0]) continue;
          const int c = (cz * g.dims[1] + cy) * g.dims[0] + cx;
          const int e = cs[c + 1];
          for (int j = cs[c]; j < e; ++j) {
            const float4 p = P[j];
            const float dx = p.x - qv[0], dy = p.y - qv[1], dz = p.z - qv[2];
            const float d2 = (dx * dx + dy * dy) + dz * dz;
            const int pi = __float_as_int(p.w);
            if ((d2 < kd[KT - 1]) | ((d2 == kd[KT - 1]) & (pi < ki[KT - 1]))) topk_insert_lex<KT>(kd, ki, d2, pi);
          }
        }
      }
    }
    // smallest distance from q to any cell outside the scanned cube (inside the grid)
    float lb2 = __builtin_huge_valf();
    bool more = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int b1 = (a + 1) % 3, b2 = (a + 2) % 3;
      const float rest = gap[b1] * gap[b1] + gap[b2] * gap[b2];
      if (home[a] - r - 1 >= 0) {  // low slab: cells <= home - r - 1
        more = true;
        const float face = g.bmin[a] + static_cast<float>(home[a] - r) * g.h;
        const float d = fmaxf(0.0f, qv[a] - face - g.margin);
        lb2 = fminf(lb2, d * d + rest);
      }
      if (home[a] + r + 1 < g.dims[a]) {  // high slab: cells >= home + r + 1
        more = true;
        const float face = g.bmin[a] + static_cast<float>(home[a] + r + 1) * g.h;
        const float d = fmaxf(0.0f, face - qv[a] - g.margin);
        lb2 = fminf(lb2, d * d + rest);
      }
    }
    if (!more) break;
    float kth = kd[0];
#pragma unroll
    for (int t = 1; t < KT; ++t) kth = (t == k - 1) ? kd[t] : kth;
    // every unscanned point has computed d2 >= lb2 * (1 - O(eps)): stop once the k-th distance is
    // strictly below that, so no unscanned point can enter or tie the top k
    if (kth < lb2 * (1.0f - 2.0e-6f)) break;
  }
  const int64_t o = (static_cast<int64_t>(b) * Q + q) * k;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    if (t < k) {
      const bool ok = kd[t] < __builtin_huge_valf();
      if (dist) dist[o + t] = ok ? sqrt_rn(kd[t]) : kd[t];
      if (idx) idx[o + t] = ok ? ki[t] : -1;
      if (idx64) idx64[o + t] = ok ? ki[t] : -1;
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

extern "C" int dvcp_knn_grid(int dtype, const void* ref, int64_t rb, int64_t rc, int64_t rn, int M, const void* qry,
                             int64_t qb, int64_t qc, int64_t qn, int Q, int B, int k, void* workspace, float* dist,
                             int32_t* idx, int64_t* idx64, void* stream) {
  DVCP_REQUIRE(ref && qry && workspace, "dvcp_knn_grid: null pointer");
  DVCP_REQUIRE(k > 0 && k <= 32 && M >= 0 && Q >= 0 && B >= 0 && B <= 65535, "dvcp_knn_grid: bad sizes");
  if (B == 0 || Q == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* ws = static_cast<char*>(workspace);
  auto* hdr = reinterpret_cast<dvcp::KnnGridHeader*>(ws);
  auto* cs = reinterpret_cast<int32_t*>(ws + 64 * static_cast<int64_t>(B));
  auto* so = reinterpret_cast<float4*>(ws + 64 * static_cast<int64_t>(B) +
                                       16 * dvcp::ceil_div(4 * static_cast<int64_t>(B) * (dvcp::kGridMaxCells + 1), 16));
  dim3 qgrid(dvcp::ceil_div(Q, dvcp::kKnnThreads), B);
#define DVCP_KNNG(TT, KK)                                                                                              if (k <= KK) {                                                                                                         hipLaunchKernelGGL((dvcp::knn_grid_query_kernel<TT, KK>), qgrid, dim3(dvcp::kKnnThreads), 0, st, hdr, cs, so, M,                        dvcp::PointsView<TT>{static_cast<const TT*>(qry), qb, qc, qn}, Q, k, dist, idx, idx64);           return dvcp::launch_status("dvcp_knn_grid(query)");                                                               }
  if (dtype == DVCP_F32) {
    hipLaunchKernelGGL((dvcp::knn_grid_build_kernel<float>), dim3(B), dim3(1024), 0, st,
                       dvcp::PointsView<float>{static_cast<const float*>(ref), rb, rc, rn}, M, hdr, cs, so);
    if (int e = dvcp::launch_status("dvcp_knn_grid(build)")) return e;
    DVCP_KNNG(float, 1)
    DVCP_KNNG(float, 8)
    DVCP_KNNG(float, 16)
    DVCP_KNNG(float, 32)
  } else if (dtype == DVCP_F64) {
    hipLaunchKernelGGL((dvcp::knn_grid_build_kernel<double>), dim3(B), dim3(1024), 0, st,
                       dvcp::PointsView<double>{static_cast<const double*>(ref), rb, rc, rn}, M, hdr, cs, so);
    if (int e = dvcp::launch_status("dvcp_knn_grid(build)")) return e;
    DVCP_KNNG(double, 1)
    DVCP_KNNG(double, 8)
    DVCP_KNNG(double, 16)
    DVCP_KNNG(double, 32)
  }
#undef DVCP_KNNG
  dvcp::set_error("dvcp_knn_grid: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

extern "C" int64_t dvcp_knn_grid_workspace_bytes(int B, int M) {
  return 64 * static_cast<int64_t>(B) + 16 * dvcp::ceil_div(4 * static_cast<int64_t>(B) * (dvcp::kGridMaxCells + 1), 16) +
         16 * static_cast<int64_t>(B) * M;
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
