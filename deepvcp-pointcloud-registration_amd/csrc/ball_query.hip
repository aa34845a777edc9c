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
  if (my_pad)
    for (int j = cnt; j < nsample; ++j) my_pad[j] = first;
}

// ---------------------------------------------------------------------------------------------
// fp32 path: one wave = 64 centres with its own early exit, points streamed in ascending index
// order as wave-uniform scalar loads of packed (x, y, z, |p|^2) -- no LDS, no block barrier.  A
// wave stops as soon as each of its centres has `nsample` hits, so dense radii scan only the
// prefix they need and a sparse wave never waits for a dense one.
typedef __attribute__((address_space(4))) const float bq_const_float;

// Rows are padded to a multiple of 16 points (zeros) so every 16-point chunk of the query loop is one
// unconditional scalar burst; the padding never hits because the loop tests n < N.
__host__ __device__ constexpr int bq_padded_n(int N) { return (N + 15) & ~15; }

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

template <typename P>
__device__ __forceinline__ P* bq_uniform_ptr(P* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v & 0xFFFFFFFFull)));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32)));
  return reinterpret_cast<P*>((static_cast<uint64_t>(hi) << 32) | lo);
}

__global__ __launch_bounds__(256) void bq_wave_kernel(const float4* __restrict__ packed, int N, PointsView<float> ctr,
                                                      int S, float r2, int nsample, int32_t* __restrict__ count,
                                                      int32_t* __restrict__ list, int64_t* __restrict__ padded) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
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
  const bq_const_float* P = (const bq_const_float*)bq_uniform_ptr(packed + static_cast<int64_t>(b) * bq_padded_n(N));
  (void)lane;
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
      float4* packed = static_cast<float4*>(workspace);
      hipLaunchKernelGGL(bq_pack_kernel, dim3(ceil_div(bq_padded_n(N), 256), B), dim3(256), 0, st, pv, N, packed);
      if (int e = launch_status("dvcp_ball_query(pack)")) return e;
      hipLaunchKernelGGL(bq_wave_kernel, dim3(ceil_div(S, 256), B), dim3(256), 0, st, packed, N, cv, S, r2,
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
