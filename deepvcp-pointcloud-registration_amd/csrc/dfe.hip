// dfe.hip -- deep feature embedding (deep_feat_embedding.py:23-61).
//
//   X.float(); fc1 (35->32), fc2 (32->32), fc3 (32->32), NO nonlinearity (Q14, kept
//   un-collapsed); MaxPool1d(32) over the neighbour axis.
//
// dvcp_dfe     : materialised input rows (the source side, B*K*32 rows).
// dvcp_dfe_tgt : target side fused with get_cat_feat_tgt.py:54-96 -- the (B,K,C,32,35) fp64
//                tensor (763 MB per pair at C=1331) is never materialised; each row is
//                gathered and weighted in registers straight from the kNN output.
//
// One thread = one neighbour row, 8 queries x 32 rows = 256 threads per workgroup.  Weights
// are wave-uniform scalar loads; the max over a query's 32 rows goes through LDS.
#include "common.h"

#include <algorithm>

namespace dvcp {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// dfe_mfma.hip: the target side on fp32 MFMA.  literal = false: the three linear layers collapsed
// into one map (default); true: fc1, fc2, fc3 evaluated one after the other.
template <typename T>
int launch_dfe_tgt_mfma(PointsView<T> ref, const float* feat, int M, const float* cand, const float* dist,
                        const int32_t* idx, int B, int Q, const float* params, float* out, bool literal,
                        hipStream_t st);

// segsum.hip: deterministic per-row sums of keyed 32-float contribution rows.
int64_t segment_sum_workspace_bytes(int64_t E, int64_t nrows);
int segment_sum(const uint32_t* keys, const float* contrib, int64_t E, int64_t nrows, int ncol, float* out, void* ws,
                hipStream_t st);

constexpr int kDfeRowsPerQ = 32;
constexpr int kDfeThreads = 256;
constexpr int kDfeQPerBlock = kDfeThreads / kDfeRowsPerQ;

__device__ __forceinline__ void dfe_mlp(const float (&x)[35], float (&y)[32], const float* __restrict__ params) {
  float h1[32], h2[32];
  linear_sgpr<35, 32>(x, h1, params);
  const float* p2 = params + 35 * 32 + 32;
  linear_sgpr<32, 32>(h1, h2, p2);
  linear_sgpr<32, 32>(h2, y, p2 + 32 * 32 + 32);
}

// rows -> per-query max over the 32 rows (rows of query ql are threads ql*32 .. ql*32+31)
__device__ __forceinline__ void dfe_pool_store(const float (&y)[32], float (*red)[33], int64_t q0, int64_t nq,
                                               float* __restrict__ out) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int c = 0; c < 32; ++c) red[tid][c] = y[c];
  __syncthreads();
  const int ql = tid / 32, c = tid % 32;
  if (q0 + ql < nq) {
    float m = red[ql * 32][c];
#pragma unroll 8
    for (int j = 1; j < 32; ++j) m = fmaxf(m, red[ql * 32 + j][c]);
    out[(q0 + ql) * 32 + c] = m;
  }
}

template <typename XT>
__global__ __launch_bounds__(kDfeThreads) void dfe_kernel(const XT* __restrict__ X, int64_t R,
                                                          const float* __restrict__ params, float* __restrict__ out) {
  __shared__ float red[kDfeThreads][33];
  const int64_t q0 = static_cast<int64_t>(blockIdx.x) * kDfeQPerBlock;
  const int64_t row = q0 * kDfeRowsPerQ + threadIdx.x;
  float x[35];
  if (row < R * kDfeRowsPerQ) {
    const XT* src = X + row * 35;
#pragma unroll
    for (int i = 0; i < 35; ++i) x[i] = static_cast<float>(src[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 35; ++i) x[i] = 0.f;
  }
  float y[32];
  dfe_mlp(x, y, params);
  dfe_pool_store(y, red, q0, R, out);
}

// Row j = tid % 32 of query q (batch b) of get_cat_feat_tgt.py:54-96 -> x[35], for a block of 8
// queries x 32 rows (every thread calls; it synchronises).  dsh: kDfeThreads doubles, wq: [8][32].
template <typename T>
__device__ __forceinline__ void dfe_tgt_row(PointsView<T> ref, const float* __restrict__ feat, int M,
                                            const float* __restrict__ cand, const float* __restrict__ dist,
                                            const int32_t* __restrict__ idx, int Q, int b, int64_t q, bool live,
                                            double* dsh, double (*wq)[32], float (&x)[35]) {
  const int tid = threadIdx.x, ql = tid / 32, j = tid % 32;
  const int64_t kq = (static_cast<int64_t>(b) * Q + (live ? q : 0)) * 32;
  // get_cat_feat_tgt.py:57-58: dist_sum in fp64, w = dist / dist_sum (fp64)
  const float dj = live ? dist[kq + j] : 1.0f;
  double s = static_cast<double>(dj);
  // fixed-order fp64 sum over the query's 32 neighbours (lanes ql*32 .. ql*32+31)
  dsh[tid] = s;
  __syncthreads();
  double acc = 0.0;
  for (int t = 0; t < 32; ++t) acc += dsh[ql * 32 + t];
  wq[ql][j] = static_cast<double>(dj) / acc;
  __syncthreads();

  int n = live ? idx[kq + j] : 0;
  n = n < 0 ? 0 : (n >= M ? M - 1 : n);
  const float* cq = cand + (static_cast<int64_t>(b) * Q + (live ? q : 0)) * 3;
  // candidates_grouped_local = tgt_pts_picked - candidate (tgt xyz dtype, then .float())
  x[0] = static_cast<float>(ref.at(b, 0, n) - static_cast<T>(cq[0]));
  x[1] = static_cast<float>(ref.at(b, 1, n) - static_cast<T>(cq[1]));
  x[2] = static_cast<float>(ref.at(b, 2, n) - static_cast<T>(cq[2]));
  // tgt_feat_norm[j, f] = F[idx_j, f] * w[f]   (Q10: weight indexed by the feature channel)
  const float4* fr = reinterpret_cast<const float4*>(feat + (static_cast<int64_t>(b) * M + n) * 32);
#pragma unroll
  for (int f4 = 0; f4 < 8; ++f4) {
    const float4 v = fr[f4];
    x[3 + 4 * f4 + 0] = static_cast<float>(static_cast<double>(v.x) * wq[ql][4 * f4 + 0]);
    x[3 + 4 * f4 + 1] = static_cast<float>(static_cast<double>(v.y) * wq[ql][4 * f4 + 1]);
    x[3 + 4 * f4 + 2] = static_cast<float>(static_cast<double>(v.z) * wq[ql][4 * f4 + 2]);
    x[3 + 4 * f4 + 3] = static_cast<float>(static_cast<double>(v.w) * wq[ql][4 * f4 + 3]);
  }
}

// ---------------------------------------------------------------------------------------------
// Backward (train.py:121 loss.backward() through deep_feat_embedding.py:23-61).  The three layers
// are linear (Q14), so with g3 the gradient the max-pool routes to the arg-max row of each output
// channel (MaxPool1d: first index among equal values), every weight gradient is a fixed linear
// map of just two sums over all routed rows:
//   Gx[f][c] = sum_q g[q,f] x[q, j*(q,f), c]   (32 x 35),     gs[f] = sum_q g[q,f]
//   Gh1 = Gx W1^T + gs b1^T,  Gh2 = Gh1 W2^T + gs b2^T
//   dW3 = Gh2, db3 = gs;  dW2 = W3^T Gh1, db2 = W3^T gs;  dW1 = W2^T W3^T Gx, db1 = W2^T W3^T gs.
// dfe_bwd_kernel re-runs the forward rows to find j*, as the forward kernel evaluates them: the
// collapsed map y = E x + e (dfe_collapse_kernel forms E, e in fp64 and rounds them once to fp32,
// exactly like dfe_tgt_mfma1_kernel's prologue; 1120 fma per row instead of 3168), and
// accumulates Gx, gs per workgroup (fixed grid, fixed order: deterministic); dfe_bwd_sum_kernel
// sums the workgroup partials in fp64 and dfe_bwd_finish_kernel applies the map.
// Workspace: [nblk][32][36] fp32 partials | [32][36] fp64 sums | [32][36] fp32 (E | e).
constexpr int kDfeGPart = 32 * 36;  // per workgroup: [f][35 Gx + gs]
constexpr int kDfeBwdMaxGrid = 2048;

// E = W3 W2 W1 and e = W3 (W2 b1 + b2) + b3 in fp64, rounded once to fp32 ([f][36]: E | e).
__global__ __launch_bounds__(1024) void dfe_collapse_kernel(const float* __restrict__ params, float* __restrict__ Ee) {
  __shared__ double p[32][36];
  const int tid = threadIdx.x;
  const float* W1 = params;
  const float* b1 = W1 + 32 * 35;
  const float* W2 = b1 + 32;
  const float* b2 = W2 + 32 * 32;
  const float* W3 = b2 + 32;
  const float* b3 = W3 + 32 * 32;
  for (int i = tid; i < 32 * 36; i += 1024) {  // P = W2 W1 | W2 b1 + b2
    const int o = i / 36, c = i % 36;
    double acc = 0.0;
    for (int a = 0; a < 32; ++a)
      acc = __fma_rn(static_cast<double>(W2[o * 32 + a]), static_cast<double>(c < 35 ? W1[a * 35 + c] : b1[a]), acc);
    p[o][c] = c < 35 ? acc : acc + static_cast<double>(b2[o]);
  }
  __syncthreads();
  for (int i = tid; i < 32 * 36; i += 1024) {
    const int o = i / 36, c = i % 36;
    double acc = 0.0;
    for (int a = 0; a < 32; ++a) acc = __fma_rn(static_cast<double>(W3[o * 32 + a]), p[a][c], acc);
    Ee[i] = static_cast<float>(c < 35 ? acc : acc + static_cast<double>(b3[o]));
  }
}

// Gs[e] = sum over workgroups of part[k][e] in fp64: 64 elements x 16 slices per workgroup,
// slices summed in order.
__global__ __launch_bounds__(1024) void dfe_bwd_sum_kernel(const float* __restrict__ part, int nblk,
                                                           double* __restrict__ Gs) {
  __shared__ double sl[16][64];
  const int tid = threadIdx.x, c = tid & 63, slice = tid >> 6;
  const int e = blockIdx.x * 64 + c;
  double s = 0.0;
  if (e < kDfeGPart)
    for (int k = slice; k < nblk; k += 16) s += static_cast<double>(part[static_cast<int64_t>(k) * kDfeGPart + e]);
  sl[slice][c] = s;
  __syncthreads();
  if (tid < 64 && e < kDfeGPart) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += sl[k][c];
    Gs[e] = t;
  }
}

template <int MODE, typename T>  // MODE 0: materialised rows X (R, 32, 35); 1: fused target rows
__global__ __launch_bounds__(kDfeThreads) __attribute__((amdgpu_waves_per_eu(2))) void dfe_bwd_kernel(const T* __restrict__ X, PointsView<T> ref,
                                                              const float* __restrict__ feat, int M,
                                                              const float* __restrict__ cand,
                                                              const float* __restrict__ dist,
                                                              const int32_t* __restrict__ idx, int Q, int64_t R,
                                                              const float* __restrict__ Ee,
                                                              const float* __restrict__ gout, float* __restrict__ part,
                                                              float* __restrict__ gX, float* __restrict__ gF,
                                                              uint32_t* __restrict__ gkey, uint32_t key_none) {
  __shared__ float xs[kDfeThreads][37];
  __shared__ float Es[32][37];  // E (the bias e shifts a channel's rows alike: not needed for the arg-max)
  __shared__ double wq[kDfeQPerBlock][32];
  __shared__ double dsh[kDfeThreads];
  __shared__ int rsel[kDfeThreads];   // input-row gradient: each channel's arg-max row ...
  __shared__ float rg[kDfeThreads];   // ... and its output gradient
  const int tid = threadIdx.x, ql = tid / 32, f = tid % 32, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 32 * 36; i += kDfeThreads) Es[i / 36][i % 36] = Ee[i];
  float acc[36];
#pragma unroll
  for (int i = 0; i < 36; ++i) acc[i] = 0.f;
  for (int64_t q0 = static_cast<int64_t>(blockIdx.x) * kDfeQPerBlock; q0 < R;
       q0 += static_cast<int64_t>(gridDim.x) * kDfeQPerBlock) {
    const int64_t q = q0 + ql;
    const bool live = q < R;
    float x[35];
    if constexpr (MODE == 0) {
      const T* src = X + ((live ? q : 0) * 32 + f) * 35;
#pragma unroll
      for (int i = 0; i < 35; ++i) x[i] = live ? static_cast<float>(src[i]) : 0.f;
    } else {
      const int b = static_cast<int>((live ? q : 0) / Q);
      const int64_t qq = (live ? q : 0) - static_cast<int64_t>(b) * Q;
      dfe_tgt_row(ref, feat, M, cand, dist, idx, Q, b, qq, live, dsh, wq, x);
    }
    __syncthreads();  // the previous group's readers are done
#pragma unroll
    for (int i = 0; i < 35; ++i) xs[tid][i] = x[i];
    __syncthreads();
    // Y = X E^T for this wave's two queries on v_mfma_f32_32x32x2_f32 (18 k-steps over the 35
    // inputs): lane l supplies A = X[row l&31][k], B = E^T[k][channel l&31]; the result holds
    // channel l&31, rows (r&3) + 8(r>>2) + 4(l>>5) in register r.
    int bj = 0;
    {
      const int h = lane >> 5, c32 = lane & 31;
      f32x16 y0 = {}, y1 = {};
#pragma unroll
      for (int s2 = 0; s2 < 18; ++s2) {
        const int k = 2 * s2 + h;
        const float bk = k < 35 ? Es[c32][k] : 0.f;
        const float a0 = k < 35 ? xs[(2 * wave) * 32 + c32][k] : 0.f;
        const float a1 = k < 35 ? xs[(2 * wave + 1) * 32 + c32][k] : 0.f;
        y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bk, y0, 0, 0, 0);
        y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bk, y1, 0, 0, 0);
      }
      // per lane: the best of its 16 rows, then against lane ^ 32's (MaxPool1d: first index)
      float b0 = -__builtin_huge_valf(), bb1 = -__builtin_huge_valf();
      int j0 = 64, j1 = 64;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (y0[r] > b0 || (y0[r] == b0 && row < j0)) {
          b0 = y0[r];
          j0 = row;
        }
        if (y1[r] > bb1 || (y1[r] == bb1 && row < j1)) {
          bb1 = y1[r];
          j1 = row;
        }
      }
      const float ob0 = __shfl_xor(b0, 32, kWave), ob1 = __shfl_xor(bb1, 32, kWave);
      const int oj0 = __shfl_xor(j0, 32, kWave), oj1 = __shfl_xor(j1, 32, kWave);
      if (ob0 > b0 || (ob0 == b0 && oj0 < j0)) j0 = oj0;
      if (ob1 > bb1 || (ob1 == bb1 && oj1 < j1)) j1 = oj1;
      bj = h == 0 ? j0 : j1;  // thread (ql = 2 wave + h, f = lane & 31)
    }
    const float g = live ? gout[q * 32 + f] : 0.f;
#pragma unroll
    for (int i = 0; i < 35; ++i) acc[i] = __fmaf_rn(g, xs[ql * 32 + bj][i], acc[i]);
    acc[35] += g;
    if (gX || gF) {  // block-uniform: the input rows' gradient, dL/dx_j = sum_{f: j*(f) = j} g_f E[f]
      // each thread gathers the channels routed to its own row j (pulled from the per-candidate
      // (j*, g) table; no LDS atomics), in channel order
      rsel[tid] = bj;
      rg[tid] = g;
      __syncthreads();
      const int j = f;  // this thread's own row
      float dx[35];
#pragma unroll
      for (int i = 0; i < 35; ++i) dx[i] = 0.f;
      // the channels routed to row j as a mask, then each lane walks only its own (about one per
      // row; ascending, as before): a wave no longer steps through all 32 channels whenever one
      // of its 64 rows takes each of them
      uint32_t mine = 0u;
#pragma unroll 8
      for (int ff = 0; ff < 32; ++ff) mine |= rsel[ql * 32 + ff] == j ? (1u << ff) : 0u;
      const bool any = mine != 0u;
      while (mine != 0u) {
        const int ff = __builtin_ctz(mine);
        mine &= mine - 1u;
        const float gf = rg[ql * 32 + ff];
#pragma unroll
        for (int i = 0; i < 35; ++i) dx[i] = __fmaf_rn(gf, Es[ff][i], dx[i]);
      }
      if constexpr (MODE == 0) {
        if (live)
          for (int i = 0; i < 35; ++i) gX[(q * 32 + j) * 35 + i] = dx[i];
      } else {
        // get_cat_feat_tgt.py:85,95: x[3 + c] = F[idx_j, c] * w[c] (fp64 weight) -> entry (q, j)
        // contributes dx[3 + c] * w[c] to dF[idx_j, c]: its contribution row and target row are
        // written here and summed per target row by segment_sum (segsum.hip, deterministic)
        if (live) {
          const int64_t e = q * 32 + j;
          const int b = static_cast<int>(q / Q);
          int n = idx[e];
          n = n < 0 ? 0 : (n >= M ? M - 1 : n);
          gkey[e] = any ? static_cast<uint32_t>(static_cast<int64_t>(b) * M + n) : key_none;
          if (any) {
            float4* dst = reinterpret_cast<float4*>(gF + e * 32);
#pragma unroll
            for (int c4 = 0; c4 < 8; ++c4) {
              float v[4];
#pragma unroll
              for (int u = 0; u < 4; ++u)
                v[u] = static_cast<float>(static_cast<double>(dx[3 + 4 * c4 + u]) * wq[ql][4 * c4 + u]);
              dst[c4] = make_float4(v[0], v[1], v[2], v[3]);
            }
          }
        }
      }
      __syncthreads();  // rsel / rg are rewritten by the next group
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 36; ++i) xs[tid][i] = acc[i];
  __syncthreads();
  for (int e = tid; e < kDfeGPart; e += kDfeThreads) {
    const int ff = e / 36, i = e % 36;
    float s = 0.f;
    for (int k = 0; k < kDfeQPerBlock; ++k) s += xs[k * 32 + ff][i];
    part[static_cast<int64_t>(blockIdx.x) * kDfeGPart + e] = s;
  }
}

// One 1024-thread workgroup: partials -> packed parameter gradients (W1, b1, W2, b2, W3, b3).
__global__ __launch_bounds__(1024) void dfe_bwd_finish_kernel(const double* __restrict__ Gsum,
                                                              const float* __restrict__ params,
                                                              float* __restrict__ grad) {
  __shared__ double Gs[kDfeGPart];
  __shared__ double Gh1[32][33];
  __shared__ double U[32][36];  // W3^T [Gx | gs]
  const int tid = threadIdx.x;
  const float* W1 = params;
  const float* b1 = W1 + 32 * 35;
  const float* W2 = b1 + 32;
  const float* b2 = W2 + 32 * 32;
  const float* W3 = b2 + 32;
  float* gW1 = grad;
  float* gb1 = gW1 + 32 * 35;
  float* gW2 = gb1 + 32;
  float* gb2 = gW2 + 32 * 32;
  float* gW3 = gb2 + 32;
  float* gb3 = gW3 + 32 * 32;
  for (int e = tid; e < kDfeGPart; e += 1024) Gs[e] = Gsum ? Gsum[e] : 0.0;
  __syncthreads();
  {  // Gh1[f][k] = sum_c Gx[f][c] W1[k][c] + gs[f] b1[k]
    const int ff = tid / 32, k = tid % 32;
    double v = Gs[ff * 36 + 35] * b1[k];
    for (int c = 0; c < 35; ++c) v += Gs[ff * 36 + c] * W1[k * 35 + c];
    Gh1[ff][k] = v;
  }
  for (int e = tid; e < 32 * 36; e += 1024) {  // U[m][c] = sum_f W3[f][m] [Gx | gs][f][c]
    const int m = e / 36, c = e % 36;
    double v = 0.0;
    for (int ff = 0; ff < 32; ++ff) v += static_cast<double>(W3[ff * 32 + m]) * Gs[ff * 36 + c];
    U[m][c] = v;
  }
  __syncthreads();
  {
    const int ff = tid / 32, m = tid % 32;
    // dW3[f][m] = Gh2[f][m] = sum_k Gh1[f][k] W2[m][k] + gs[f] b2[m]
    double v = Gs[ff * 36 + 35] * b2[m];
    for (int k = 0; k < 32; ++k) v += Gh1[ff][k] * W2[m * 32 + k];
    gW3[ff * 32 + m] = static_cast<float>(v);
    // dW2[m'][k'] = sum_f W3[f][m'] Gh1[f][k']   (thread: m' = ff, k' = m)
    double w = 0.0;
    for (int f2 = 0; f2 < 32; ++f2) w += static_cast<double>(W3[f2 * 32 + ff]) * Gh1[f2][m];
    gW2[ff * 32 + m] = static_cast<float>(w);
  }
  for (int e = tid; e < 32 * 36; e += 1024) {  // dW1[k][c] / db1[k] = sum_m W2[m][k] U[m][c]
    const int k = e / 36, c = e % 36;
    double v = 0.0;
    for (int m = 0; m < 32; ++m) v += static_cast<double>(W2[m * 32 + k]) * U[m][c];
    if (c < 35) gW1[k * 35 + c] = static_cast<float>(v); else gb1[k] = static_cast<float>(v);
  }
  if (tid < 32) {
    gb2[tid] = static_cast<float>(U[tid][35]);
    gb3[tid] = static_cast<float>(Gs[tid * 36 + 35]);
  }
}

}  // namespace dvcp

extern "C" int dvcp_dfe(int x_dtype, const void* X, int64_t R, const float* params, float* out, void* stream) {
  DVCP_REQUIRE(X && params && out, "dvcp_dfe: null pointer");
  if (R <= 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(dvcp::ceil_div(R, dvcp::kDfeQPerBlock));
  if (x_dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::dfe_kernel<float>), grid, dim3(dvcp::kDfeThreads), 0, st, static_cast<const float*>(X), R,
                       params, out);
  else if (x_dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::dfe_kernel<double>), grid, dim3(dvcp::kDfeThreads), 0, st, static_cast<const double*>(X),
                       R, params, out);
  else {
    dvcp::set_error("dvcp_dfe: bad dtype %d", x_dtype);
    return DVCP_EINVAL;
  }
  return dvcp::launch_status("dvcp_dfe");
}

static int dfe_tgt_entry(const char* name, bool literal, int dtype, const void* ref_xyz, int64_t rb, int64_t rc,
                         int64_t rn, int M, const float* ref_feat, const float* cand, const float* dist,
                         const int32_t* idx, int B, int Q, const float* params, float* out, void* stream) {
  DVCP_REQUIRE(ref_xyz && ref_feat && cand && dist && idx && params && out, "%s: null pointer", name);
  DVCP_REQUIRE(M > 0 && B >= 0 && B <= 65535 && Q >= 0, "%s: bad sizes", name);
  if (B == 0 || Q == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DVCP_F32)
    return dvcp::launch_dfe_tgt_mfma<float>(dvcp::PointsView<float>{static_cast<const float*>(ref_xyz), rb, rc, rn},
                                            ref_feat, M, cand, dist, idx, B, Q, params, out, literal, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_dfe_tgt_mfma<double>(dvcp::PointsView<double>{static_cast<const double*>(ref_xyz), rb, rc, rn},
                                             ref_feat, M, cand, dist, idx, B, Q, params, out, literal, st);
  dvcp::set_error("%s: bad dtype %d", name, dtype);
  return DVCP_EINVAL;
}

extern "C" int dvcp_dfe_tgt(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                            const float* ref_feat, const float* cand, const float* dist, const int32_t* idx, int B, int Q,
                            const float* params, float* out, void* stream) {
  return dfe_tgt_entry("dvcp_dfe_tgt", false, dtype, ref_xyz, rb, rc, rn, M, ref_feat, cand, dist, idx, B, Q, params,
                       out, stream);
}

extern "C" int dvcp_dfe_tgt_literal(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                                    const float* ref_feat, const float* cand, const float* dist, const int32_t* idx,
                                    int B, int Q, const float* params, float* out, void* stream) {
  return dfe_tgt_entry("dvcp_dfe_tgt_literal", true, dtype, ref_xyz, rb, rc, rn, M, ref_feat, cand, dist, idx, B, Q,
                       params, out, stream);
}

static int64_t dfe_bwd_blocks(int64_t R) {
  return R <= 0 ? 1 : std::min<int64_t>(dvcp::kDfeBwdMaxGrid, (R + dvcp::kDfeQPerBlock - 1) / dvcp::kDfeQPerBlock);
}

extern "C" int64_t dvcp_dfe_backward_workspace_bytes(int64_t R) {  // (same for the target entry)
  return dfe_bwd_blocks(R) * dvcp::kDfeGPart * static_cast<int64_t>(sizeof(float)) +
         dvcp::kDfeGPart * static_cast<int64_t>(sizeof(double) + sizeof(float));
}

// mode 0: X (R, 32, 35) rows (x_dtype); mode 1: fused target rows (the dvcp_dfe_tgt arguments, R = B*Q).
// Target-feature gradient (mode 1, gF): after the parameter-gradient workspace, the entries'
// target rows (R * 32 u32), their contribution rows (R * 32 * 32 fp32) and segment_sum's own.
static int64_t tgt_feat_ws_offset(int64_t R) { return (dvcp_dfe_backward_workspace_bytes(R) + 255) / 256 * 256; }
static int64_t tgt_contrib_offset(int64_t R) { return tgt_feat_ws_offset(R) + (R * 32 * 4 + 255) / 256 * 256; }
static int64_t tgt_segsum_offset(int64_t R) { return tgt_contrib_offset(R) + R * 32 * 32 * 4; }

extern "C" int64_t dvcp_dfe_tgt_backward_workspace_bytes(int B, int Q, int M, int want_feat_grad) {
  const int64_t R = static_cast<int64_t>(B) * Q;
  if (!want_feat_grad || R <= 0) return dvcp_dfe_backward_workspace_bytes(R);
  const int64_t seg = dvcp::segment_sum_workspace_bytes(R * 32, static_cast<int64_t>(B) * M);
  return seg < 0 ? -1 : tgt_segsum_offset(R) + seg;
}

static int dfe_backward_launch(int mode, int dtype, const void* X, const void* ref_xyz, int64_t rb, int64_t rc,
                               int64_t rn, int M, const float* ref_feat, const float* cand, const float* dist,
                               const int32_t* idx, int Q, int64_t R, const float* params, const float* grad_out,
                               float* ws, float* grad_params, float* gX, float* gF_out, int rows_out, hipStream_t st) {
  if (R <= 0) {  // no rows: zero gradients (the target-feature gradient too: no entry routes to any row)
    hipLaunchKernelGGL(dvcp::dfe_bwd_finish_kernel, dim3(1), dim3(1024), 0, st, nullptr, params, grad_params);
    if (gF_out && M > 0 && rows_out > 0) {
      const hipError_t e = hipMemsetAsync(gF_out, 0, static_cast<size_t>(rows_out) * M * 32 * sizeof(float), st);
      if (e != hipSuccess) {
        dvcp::set_error("dvcp_dfe_tgt_backward: hipMemsetAsync: %s", hipGetErrorString(e));
        return DVCP_EHIP;
      }
    }
    return dvcp::launch_status("dvcp_dfe_backward");
  }
  const int nblk = static_cast<int>(dfe_bwd_blocks(R));
  double* Gs = reinterpret_cast<double*>(ws + static_cast<int64_t>(nblk) * dvcp::kDfeGPart);
  float* Ee = reinterpret_cast<float*>(Gs + dvcp::kDfeGPart);
  hipLaunchKernelGGL(dvcp::dfe_collapse_kernel, dim3(1), dim3(1024), 0, st, params, Ee);
  const dim3 grid(nblk), block(dvcp::kDfeThreads);
  char* wsb = reinterpret_cast<char*>(ws);
  uint32_t* gkey = gF_out ? reinterpret_cast<uint32_t*>(wsb + tgt_feat_ws_offset(R)) : nullptr;
  float* gF = gF_out ? reinterpret_cast<float*>(wsb + tgt_contrib_offset(R)) : nullptr;
  const uint32_t key_none = static_cast<uint32_t>((R / Q) * M);
  if (mode == 0 && dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::dfe_bwd_kernel<0, float>), grid, block, 0, st, static_cast<const float*>(X),
                       dvcp::PointsView<float>{nullptr, 0, 0, 0}, nullptr, 0, nullptr, nullptr, nullptr, 1, R, Ee,
                       grad_out, ws, gX, gF, gkey, key_none);
  else if (mode == 0 && dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::dfe_bwd_kernel<0, double>), grid, block, 0, st, static_cast<const double*>(X),
                       dvcp::PointsView<double>{nullptr, 0, 0, 0}, nullptr, 0, nullptr, nullptr, nullptr, 1, R, Ee,
                       grad_out, ws, gX, gF, gkey, key_none);
  else if (mode == 1 && dtype == DVCP_F32)
    hipLaunchKernelGGL((dvcp::dfe_bwd_kernel<1, float>), grid, block, 0, st, nullptr,
                       dvcp::PointsView<float>{static_cast<const float*>(ref_xyz), rb, rc, rn}, ref_feat, M, cand, dist,
                       idx, Q, R, Ee, grad_out, ws, gX, gF, gkey, key_none);
  else if (mode == 1 && dtype == DVCP_F64)
    hipLaunchKernelGGL((dvcp::dfe_bwd_kernel<1, double>), grid, block, 0, st, nullptr,
                       dvcp::PointsView<double>{static_cast<const double*>(ref_xyz), rb, rc, rn}, ref_feat, M, cand,
                       dist, idx, Q, R, Ee, grad_out, ws, gX, gF, gkey, key_none);
  else {
    dvcp::set_error("dvcp_dfe_backward: bad dtype %d", dtype);
    return DVCP_EINVAL;
  }
  hipLaunchKernelGGL(dvcp::dfe_bwd_sum_kernel, dim3(dvcp::ceil_div(dvcp::kDfeGPart, 64)), dim3(1024), 0, st, ws, nblk,
                     Gs);
  hipLaunchKernelGGL(dvcp::dfe_bwd_finish_kernel, dim3(1), dim3(1024), 0, st, Gs, params, grad_params);
  if (gF_out) {
    const int rc2 = dvcp::launch_status("dvcp_dfe_tgt_backward");
    if (rc2 != DVCP_OK) return rc2;
    return dvcp::segment_sum(gkey, gF, R * 32, static_cast<int64_t>(R / Q) * M, 32, gF_out, wsb + tgt_segsum_offset(R),
                             st);
  }
  return dvcp::launch_status("dvcp_dfe_backward");
}

extern "C" int dvcp_dfe_backward(int x_dtype, const void* X, int64_t R, const float* params, const float* grad_out,
                                 float* ws, float* grad_params, float* grad_X, void* stream) {
  DVCP_REQUIRE(params && grad_params && (R <= 0 || (X && grad_out && ws)), "dvcp_dfe_backward: null pointer");
  return dfe_backward_launch(0, x_dtype, X, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, 1, R, params,
                             grad_out, ws, grad_params, grad_X, nullptr, 0, static_cast<hipStream_t>(stream));
}

extern "C" int dvcp_dfe_tgt_backward(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                                     const float* ref_feat, const float* cand, const float* dist, const int32_t* idx,
                                     int B, int Q, const float* params, const float* grad_out, float* ws,
                                     float* grad_params, float* grad_ref_feat, void* stream) {
  DVCP_REQUIRE(params && grad_params, "dvcp_dfe_tgt_backward: null pointer");
  DVCP_REQUIRE(B == 0 || Q == 0 || (ref_xyz && ref_feat && cand && dist && idx && grad_out && ws),
               "dvcp_dfe_tgt_backward: null pointer");
  DVCP_REQUIRE(M > 0 && B >= 0 && Q >= 0, "dvcp_dfe_tgt_backward: bad sizes");
  // the feature gradient's segment sums use int entry counts and u32 row keys (include/dvcp.h)
  DVCP_REQUIRE(!grad_ref_feat || (static_cast<int64_t>(B) * Q * 32 < (int64_t(1) << 31) &&
                                  static_cast<int64_t>(B) * M < (int64_t(1) << 31)),
               "dvcp_dfe_tgt_backward: B*Q*32 and B*M must stay below 2^31 (B=%d Q=%d M=%d)", B, Q, M);
  return dfe_backward_launch(1, dtype, nullptr, ref_xyz, rb, rc, rn, M, ref_feat, cand, dist, idx, Q > 0 ? Q : 1,
                             static_cast<int64_t>(B) * Q, params, grad_out, ws, grad_params, nullptr, grad_ref_feat, B,
                             static_cast<hipStream_t>(stream));
}
