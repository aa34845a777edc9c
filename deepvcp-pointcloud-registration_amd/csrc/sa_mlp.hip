// sa_mlp.hip -- grouped set-abstraction MLP (pointnet2_utils.py:122-132 + :195-200).
//
// Reference: gather (B, S, nsample, 3+D) (local xyz, features), [Conv2d 1x1 -> BN2d -> ReLU]
// per layer in fp32, then max over nsample.  The padded slots of query_ball_point repeat the
// first hit (:104-106), and a row's MLP output depends only on that row, so the max over the
// distinct hits is bit-identical to the max over all nsample slots.  This kernel therefore
// runs the MLP on the distinct hits only (count/list from dvcp_ball_query): at sa1
// (r = 0.1, ~9 hits of 256 slots) that is ~28x fewer rows than the reference evaluates.
//
// Layout: one workgroup = `cpb` consecutive centres of one cloud; their hit rows are packed
// back to back (prefix sum in LDS) and processed 256 rows per pass, one row per thread, with
// the layer weights read as wave-uniform scalar loads (SGPR operands) and activations in VGPRs.
// The max over a centre's rows is an LDS atomic max on the fp32 bit pattern (outputs are
// post-ReLU, hence >= +0, so unsigned order is float order).

#include "common.h"

namespace dvcp {

template <typename FT>
struct FeatView {
  const FT* p;
  int64_t fb, fd, fn;
  __device__ __forceinline__ float at(int b, int d, int64_t n) const {
    return static_cast<float>(p[b * fb + d * fd + n * fn]);
  }
};

constexpr int kSaThreads = 256;
constexpr int kSaMaxCpb = 64;

// y = relu((W x + bias) * scale + shift).  W (COUT x CIN), bias, scale, shift are packed
// back to back at `p`; every address is wave-uniform and compile-time, so hipcc serves the
// weights through the scalar cache into SGPR operands of v_fma (activations stay in VGPRs).
template <int CIN, int COUT>
__device__ __forceinline__ void sa_layer(const float (&x)[CIN], float (&y)[COUT], const float* __restrict__ p) {
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    float acc = 0.0f;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc = __fmaf_rn(p[co * CIN + ci], x[ci], acc);
    const float v = (acc + p[CIN * COUT + co]) * p[CIN * COUT + COUT + co] + p[CIN * COUT + 2 * COUT + co];
    y[co] = v > 0.0f ? v : 0.0f;
  }
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
__global__ __launch_bounds__(kSaThreads) void sa_mlp_kernel(PointsView<T> pts, PointsView<T> ctr, int S,
                                                            FeatView<FT> feat, const int32_t* __restrict__ count,
                                                            const int32_t* __restrict__ list, int nsample, int cpb,
                                                            const float* __restrict__ params,
                                                            float* __restrict__ out) {
  constexpr int C0 = 3 + D;
  constexpr int CL = C3 > 0 ? C3 : C2;
  __shared__ int pref[kSaMaxCpb + 1];
  __shared__ uint32_t mx[kSaMaxCpb * CL];

  const int b = blockIdx.y;
  const int c0 = blockIdx.x * cpb;
  const int nc = min(cpb, S - c0);
  const int tid = threadIdx.x;

  const float* p2 = params + C0 * C1 + 3 * C1;
  const float* p3 = p2 + C1 * C2 + 3 * C2;
  for (int i = tid; i < nc * CL; i += kSaThreads) mx[i] = 0u;

  if (tid < 64) {  // inclusive scan of the hit counts of this block's centres (nc <= 64)
    int v = 0;
    if (tid < nc) {
      v = count[static_cast<int64_t>(b) * S + c0 + tid];
      v = v < 0 ? 0 : (v > nsample ? nsample : v);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int u = __shfl_up(v, off, kWave);
      if (tid >= off) v += u;
    }
    if (tid < nc) pref[tid + 1] = v;
    if (tid == 0) pref[0] = 0;
  }
  __syncthreads();
  const int R = pref[nc];

  for (int base = 0; base < R; base += kSaThreads) {
    const int r = base + tid;
    if (r < R) {
      int lo = 0, hi = nc - 1;  // largest ci with pref[ci] <= r
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pref[mid] <= r) lo = mid; else hi = mid - 1;
      }
      const int ci = lo, j = r - pref[ci];
      const int c = c0 + ci;
      const int n = list[(static_cast<int64_t>(b) * S + c) * nsample + j];
      float x[C0];
      x[0] = static_cast<float>(pts.at(b, 0, n) - ctr.at(b, 0, c));
      x[1] = static_cast<float>(pts.at(b, 1, n) - ctr.at(b, 1, c));
      x[2] = static_cast<float>(pts.at(b, 2, n) - ctr.at(b, 2, c));
#pragma unroll
      for (int d = 0; d < D; ++d) x[3 + d] = feat.at(b, d, n);
      float y1[C1];
      sa_layer<C0, C1>(x, y1, params);
      float y2[C2];
      sa_layer<C1, C2>(y1, y2, p2);
      uint32_t* m = mx + ci * CL;
      if constexpr (C3 > 0) {
        float y3[C3];
        sa_layer<C2, C3>(y2, y3, p3);
#pragma unroll
        for (int co = 0; co < C3; ++co) atomicMax(m + co, __float_as_uint(y3[co]));
      } else {
#pragma unroll
        for (int co = 0; co < C2; ++co) atomicMax(m + co, __float_as_uint(y2[co]));
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nc * CL; i += kSaThreads) {
    const int ci = i / CL, co = i % CL;
    out[(static_cast<int64_t>(b) * S + c0 + ci) * CL + co] = __uint_as_float(mx[i]);
  }
}

// fp32 MFMA path for the two-layer tables (sa_mlp_mfma.hip)
template <typename T, int D, int C1, int C2>
int launch_sa_mfma(const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const void* c, int64_t cb, int64_t cc,
                   int64_t cn, int S, int B, const float* feat, int64_t fb, int64_t fn, const int32_t* count,
                   const int32_t* list, int nsample, const float* params, float* U, int32_t* order, float* out,
                   const int64_t* rows, int Nf, hipStream_t st);

// the three-layer table (sa1) on the matrix cores (sa_mlp_mfma.hip)
template <typename T, typename FT, int D>
int launch_sa3_mfma(const void* xyz, int64_t sb, int64_t sc, int64_t sn, const void* c, int64_t cb, int64_t cc,
                    int64_t cn, int S, int B, const void* feat, int64_t fb, int64_t fd, int64_t fn, const int32_t* count,
                    const int32_t* list, int nsample, const float* params, float* out, hipStream_t st);

#ifndef DVCP_SA1_MFMA
#define DVCP_SA1_MFMA 1
#endif

template <typename T, typename FT, int D, int C1, int C2, int C3>
static int launch_sa(const void* xyz, int64_t sb, int64_t sc, int64_t sn, const void* c, int64_t cb, int64_t cc,
                     int64_t cn, int S, int B, const void* feat, int64_t fb, int64_t fd, int64_t fn,
                     const int32_t* count, const int32_t* list, int nsample, const float* params, float* out,
                     hipStream_t st) {
  if constexpr (DVCP_SA1_MFMA && C1 == 16 && C2 == 16 && C3 == 32 && (D == 0 || D == 3))
    return launch_sa3_mfma<T, FT, D>(xyz, sb, sc, sn, c, cb, cc, cn, S, B, feat, fb, fd, fn, count, list, nsample,
                                     params, out, st);
  PointsView<T> pv{static_cast<const T*>(xyz), sb, sc, sn};
  PointsView<T> cv{static_cast<const T*>(c), cb, cc, cn};
  FeatView<FT> fv{static_cast<const FT*>(feat), fb, fd, fn};
  const int cpb = nsample > 64 ? 32 : 8;
  dim3 grid(ceil_div(S, cpb), B);
  hipLaunchKernelGGL((sa_mlp_kernel<T, FT, D, C1, C2, C3>), grid, dim3(kSaThreads), 0, st, pv, cv, S, fv, count,
                     list, nsample, cpb, params, out);
  return launch_status("dvcp_sa_group_mlp");
}

}  // namespace dvcp

// Workspace of the two-layer MFMA path: U = W1f f + b1 per input point (B x N x C1 fp32), then
// the centres' curve order (B x S int32).
static bool sa_mfma_table(int nlayer, const int* chans) {
  if (nlayer != 2 || !chans) return false;
  const int D = chans[0] - 3;
  return (D == 32 && chans[1] == 32 && chans[2] == 64) || (D == 64 && chans[1] == 64 && chans[2] == 64);
}
static int64_t sa_u_bytes(int B, int N, const int* chans) {
  return (static_cast<int64_t>(B) * N * chans[1] * 4 + 255) & ~int64_t(255);
}
static int64_t sa_ws_bytes(int B, int N, int S, int nlayer, const int* chans) {
  if (!sa_mfma_table(nlayer, chans)) return 0;
  return sa_u_bytes(B, N, chans) + static_cast<int64_t>(B) * S * 4;
}

static int sa_group_mlp_impl(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const void* ctr,
                             int64_t cb, int64_t cc, int64_t cn, int S, int B, int feat_dtype, const void* feat,
                             int64_t fb, int64_t fd, int64_t fn, int D, const int32_t* count, const int32_t* list,
                             int nsample, int nlayer, const int* chans, const float* params, float* out, void* ws,
                             void* stream, const int64_t* rows = nullptr, int Nf = 0) {
  DVCP_REQUIRE(xyz && ctr && count && list && chans && params && out, "dvcp_sa_group_mlp: null pointer");
  DVCP_REQUIRE(N > 0 || ws == nullptr, "dvcp_sa_group_mlp_ws: N must be given with a workspace");
  DVCP_REQUIRE(D == 0 || feat, "dvcp_sa_group_mlp: D=%d but feat is NULL", D);
  DVCP_REQUIRE(chans[0] == 3 + D, "dvcp_sa_group_mlp: chans[0]=%d != 3+D", chans[0]);
  if (B == 0 || S == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool f64 = dtype == DVCP_F64;
  DVCP_REQUIRE(dtype == DVCP_F32 || f64, "dvcp_sa_group_mlp: bad dtype %d", dtype);
  DVCP_REQUIRE(feat_dtype == DVCP_F32 || feat_dtype == DVCP_F64, "dvcp_sa_group_mlp: bad feat dtype");
  const bool ff64 = feat_dtype == DVCP_F64;
  float* U = ws ? static_cast<float*>(ws) : nullptr;
  int32_t* order = ws ? reinterpret_cast<int32_t*>(static_cast<char*>(ws) + sa_u_bytes(B, N, chans)) : nullptr;
#define DVCP_SA(TT, FF, DD, A, Bc, Cc)                                                                     \
  return dvcp::launch_sa<TT, FF, DD, A, Bc, Cc>(xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, fd, fn, \
                                                count, list, nsample, params, out, st)
#define DVCP_SA_T(DD, A, Bc, Cc)                    \
  do {                                              \
    if (f64) {                                      \
      if (ff64) DVCP_SA(double, double, DD, A, Bc, Cc); \
      DVCP_SA(double, float, DD, A, Bc, Cc);        \
    }                                               \
    if (ff64) DVCP_SA(float, double, DD, A, Bc, Cc); \
    DVCP_SA(float, float, DD, A, Bc, Cc);           \
  } while (0)
  // The three set-abstraction tables of deep_feat_extraction.py:10-13 (+ REF-R R1).
  if (nlayer == 3 && chans[1] == 16 && chans[2] == 16 && chans[3] == 32) {
    if (D == 0) DVCP_SA_T(0, 16, 16, 32);
    if (D == 3) DVCP_SA_T(3, 16, 16, 32);
  }
  // the paper-faithful FE's first table (paper supplement: 32-32 on xyz [+ normals]; dvcp.paper)
  if (nlayer == 2 && chans[1] == 32 && chans[2] == 32) {
    if (D == 0) DVCP_SA_T(0, 32, 32, 0);
    if (D == 3) DVCP_SA_T(3, 32, 32, 0);
  }
  // two-layer tables: fp32 MFMA when each point's features are a contiguous, 16-B aligned fp32 run
  const bool mfma_ok = !ff64 && fd == 1 && fb % 4 == 0 && fn % 4 == 0 &&
                       (reinterpret_cast<uintptr_t>(feat) & 15) == 0;
  // a feature row map is applied by the MFMA tables' per-point pre-pass only
  DVCP_REQUIRE(!rows || (mfma_ok && U && nlayer == 2 && Nf > 0),
               "dvcp_sa_group_mlp_rows_ws: the row map needs a two-layer table, fp32 point-major features "
               "(16-B aligned rows), a workspace and Nf > 0");
#define DVCP_SA_M(DD, A, Bc)                                                                                     \
  return f64 ? dvcp::launch_sa_mfma<double, DD, A, Bc>(xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B,               \
                                                     static_cast<const float*>(feat), fb, fn, count, list,      \
                                                     nsample, params, U, order, out, rows, Nf, st)              \
             : dvcp::launch_sa_mfma<float, DD, A, Bc>(xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B,                \
                                                    static_cast<const float*>(feat), fb, fn, count, list, nsample, \
                                                    params, U, order, out, rows, Nf, st)
  if (nlayer == 2 && D == 32 && chans[1] == 32 && chans[2] == 64) {
    if (mfma_ok) DVCP_SA_M(32, 32, 64);
    DVCP_SA_T(32, 32, 64, 0);
  }
  if (nlayer == 2 && D == 64 && chans[1] == 64 && chans[2] == 64) {
    if (mfma_ok) DVCP_SA_M(64, 64, 64);
    DVCP_SA_T(64, 64, 64, 0);
  }
#undef DVCP_SA_M
#undef DVCP_SA_T
#undef DVCP_SA
  dvcp::set_error("dvcp_sa_group_mlp: unsupported layer table (nlayer=%d, D=%d)", nlayer, D);
  return DVCP_EINVAL;
}

extern "C" int dvcp_sa_group_mlp(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                 const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                                 int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                                 const int32_t* count, const int32_t* list, int nsample, int nlayer,
                                 const int* chans, const float* params, float* out, void* stream) {
  return sa_group_mlp_impl(dtype, xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B, feat_dtype, feat, fb, fd, fn, D, count,
                           list, nsample, nlayer, chans, params, out, nullptr, stream);
}

extern "C" int64_t dvcp_sa_group_mlp_workspace_bytes(int B, int N, int S, int nlayer, const int* chans) {
  return sa_ws_bytes(B, N, S, nlayer, chans);
}

extern "C" int dvcp_sa_group_mlp_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                    const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                                    int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                                    const int32_t* count, const int32_t* list, int nsample, int nlayer,
                                    const int* chans, const float* params, float* out, void* workspace,
                                    void* stream) {
  DVCP_REQUIRE(sa_ws_bytes(B, N, S, nlayer, chans) == 0 || workspace, "dvcp_sa_group_mlp_ws: workspace is NULL");
  DVCP_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "dvcp_sa_group_mlp_ws: workspace not 16-B aligned");
  return sa_group_mlp_impl(dtype, xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B, feat_dtype, feat, fb, fd, fn, D, count,
                           list, nsample, nlayer, chans, params, out,
                           sa_ws_bytes(B, N, S, nlayer, chans) ? workspace : nullptr, stream);
}

extern "C" int dvcp_sa_group_mlp_rows_ws(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                         const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                                         const float* feat, int64_t fb, int64_t fn, int Nf, int D,
                                         const int64_t* feat_rows, const int32_t* count, const int32_t* list,
                                         int nsample, int nlayer, const int* chans, const float* params, float* out,
                                         void* workspace, void* stream) {
  DVCP_REQUIRE(feat && feat_rows, "dvcp_sa_group_mlp_rows_ws: null feature pointer or row map");
  DVCP_REQUIRE(sa_ws_bytes(B, N, S, nlayer, chans) > 0 && workspace,
               "dvcp_sa_group_mlp_rows_ws: needs a two-layer table and its workspace");
  DVCP_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "dvcp_sa_group_mlp_rows_ws: workspace not 16-B aligned");
  return sa_group_mlp_impl(dtype, xyz, sb, sc, sn, N, ctr, cb, cc, cn, S, B, DVCP_F32, feat, fb, 1, fn, D, count, list,
                           nsample, nlayer, chans, params, out, workspace, stream, feat_rows, Nf);
}
