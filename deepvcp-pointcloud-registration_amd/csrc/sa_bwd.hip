// sa_bwd.hip -- backward of the grouped set-abstraction MLP (pointnet2_utils.py:176-202) and of the
// feature extractor's fc (deep_feat_extraction.py:15), with the BatchNorm layers in eval mode
// (running statistics: the frozen-BN fine-tuning mode, FE1.eval() with trainable parameters).
//
// Forward being differentiated, per centre s and channel c:
//   x_n = [p_n - c_s (3), f_n (D)]     for the grouped rows n (ball-query hits; padding repeats
//                                      the first hit, whose row is identical, so distinct hits only)
//   z_l = W_l h_{l-1} + b_l,  a_l = (z_l - rm_l) * istd_l * gamma_l + beta_l,  h_l = relu(a_l)
//   out[s][c] = max_n h_L[n][c]        (torch.max over nsample, :200)
// Backward: torch.max routes g_out[s][c] to one arg-max row n*(s, c); relu passes it where a > 0
// (threshold_backward: strictly positive), so channels whose maximum is 0 send nothing.  Per
// routed row:
//   g_a_L = g_h_L [a_L > 0];  g_z_l = g_a_l * scale_l;  g_h_{l-1} = W_l^T g_z_l;  g_a_{l-1} = ...
//   dW_l += g_z_l h_{l-1}^T,  db_l += g_z_l,  dgamma_l += g_a_l zhat_l,  dbeta_l += g_a_l,
//   g_f_n += (W_1^T g_z_1)[3:]            (the index_points gather, :59 -- float atomics)
// The coordinates carry no gradient (xyz is input data; centres are index ops).
//
// Kernel layout: one wave per centre, centres in grid stride.  Pass 1 recomputes the centre's rows
// one row per lane (the forward's VALU arithmetic, folded BN), writes the last layer to an LDS tile
// and takes each channel's arg-max (first row among equal maxima, like torch.max's first index).
// Pass 2 walks the distinct routed rows; each is recomputed one output channel per lane and
// back-propagated with the weights staged in LDS.  Every wave accumulates its parameter gradients
// in registers across its centres (lane c owns row c of each dW) and writes them once; a second
// kernel sums the wave partials in a fixed order in fp64, so parameter gradients are
// deterministic.  The feature scatter uses float atomics.
#include "common.h"

#include <algorithm>

namespace dvcp {

constexpr int kSbWaves = 4;
constexpr int kSbThreads = kSbWaves * kWave;
constexpr int kSbMaxGrid = 1024;

template <typename FT>
struct SbFeat {
  const FT* p;
  int64_t fb, fd, fn;
  __device__ __forceinline__ float at(int b, int d, int64_t n) const {
    return static_cast<float>(p[b * fb + d * fd + n * fn]);
  }
};

// y = relu((W x + b) * scale + shift), weights as wave-uniform scalar loads (the forward kernel's
// arithmetic: sa_mlp.hip sa_layer); also returns the pre-activation a (for the relu mask).
template <int CIN, int COUT>
__device__ __forceinline__ void sb_layer_rows(const float (&x)[CIN], float (&y)[COUT], const float* __restrict__ p) {
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    float acc = 0.0f;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc = __fmaf_rn(p[co * CIN + ci], x[ci], acc);
    const float v = (acc + p[CIN * COUT + co]) * p[CIN * COUT + COUT + co] + p[CIN * COUT + 2 * COUT + co];
    y[co] = v > 0.0f ? v : 0.0f;
  }
}

// Sizes of a table: C0 = 3 + D inputs, C1, C2 and C3 (0 for two layers).
template <int D, int C1, int C2, int C3>
struct SbTable {
  static constexpr int C0 = 3 + D;
  static constexpr int L = C3 > 0 ? 3 : 2;
  static constexpr int CL = C3 > 0 ? C3 : C2;
  static constexpr int CMAX = C1 > C2 ? (C1 > C3 ? C1 : C3) : (C2 > C3 ? C2 : C3);
  static constexpr int P1 = C0 * C1 + 3 * C1;  // packed gradient sizes: W, b, gamma, beta
  static constexpr int P2 = C1 * C2 + 3 * C2;
  static constexpr int P3 = C3 > 0 ? C2 * C3 + 3 * C3 : 0;
  static constexpr int P = P1 + P2 + P3;
  // LDS weights: W_l as [cout][cin + 1] (row padding against bank conflicts)
  static constexpr int LW1 = C1 * (C0 + 1), LW2 = C2 * (C1 + 1), LW3 = C3 > 0 ? C3 * (C2 + 1) : 0;
};

// Lane-per-output-channel helpers over LDS-staged weights (row stride CIN + 1).
// z[lane] = W[lane] . v + b   (v broadcast from LDS)
template <int CIN>
__device__ __forceinline__ float sb_dot_row(const float* __restrict__ W, const float* __restrict__ v, int row) {
  float acc = 0.0f;
#pragma unroll 8
  for (int k = 0; k < CIN; ++k) acc = __fmaf_rn(W[row * (CIN + 1) + k], v[k], acc);
  return acc;
}
// g[lane] = sum_c W[c][lane] gz[c]
template <int CIN, int COUT>
__device__ __forceinline__ float sb_dot_col(const float* __restrict__ W, const float* __restrict__ gz, int col) {
  float acc = 0.0f;
#pragma unroll 8
  for (int c = 0; c < COUT; ++c) acc = __fmaf_rn(W[c * (CIN + 1) + col], gz[c], acc);
  return acc;
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
__global__ __launch_bounds__(kSbThreads) void sa_bwd_kernel(
    PointsView<T> pts, PointsView<T> ctr, int S, int B, SbFeat<FT> feat, const int32_t* __restrict__ count,
    const int32_t* __restrict__ list, int nsample, const float* __restrict__ params, const float* __restrict__ bnst,
    const float* __restrict__ gout, float* __restrict__ gfeat, int64_t gfb, float* __restrict__ partial) {
  using Tb = SbTable<D, C1, C2, C3>;
  constexpr int C0 = Tb::C0, CL = Tb::CL;
  __shared__ float sW1[Tb::LW1], sW2[Tb::LW2], sW3[Tb::LW3 > 0 ? Tb::LW3 : 1];
  __shared__ float tile[kSbWaves][kWave][CL + 1];    // pass 1: last-layer rows
  __shared__ float vx[kSbWaves][C0 + 1];             // pass 2: the routed row's input
  __shared__ float vh[kSbWaves][2][Tb::CMAX];        // h1, h2 of the routed row
  __shared__ float vg[kSbWaves][Tb::CMAX];           // g_z of the layer above

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // folded parameters (forward): per layer W, b, scale, shift; bn statistics: per layer rm, istd
  const float* p1 = params;
  const float* p2 = p1 + C0 * C1 + 3 * C1;
  const float* p3 = p2 + C1 * C2 + 3 * C2;
  for (int i = tid; i < C1 * C0; i += kSbThreads) sW1[(i / C0) * (C0 + 1) + i % C0] = p1[i];
  for (int i = tid; i < C2 * C1; i += kSbThreads) sW2[(i / C1) * (C1 + 1) + i % C1] = p2[i];
  if constexpr (C3 > 0)
    for (int i = tid; i < C3 * C2; i += kSbThreads) sW3[(i / C2) * (C2 + 1) + i % C2] = p3[i];
  __syncthreads();

  // per-lane channel constants of each layer (lane = output channel)
  const int c1 = lane < C1 ? lane : 0, c2 = lane < C2 ? lane : 0, c3 = lane < (C3 > 0 ? C3 : 1) ? lane : 0;
  const float b1 = p1[C0 * C1 + c1], sc1 = p1[C0 * C1 + C1 + c1], sh1 = p1[C0 * C1 + 2 * C1 + c1];
  const float b2 = p2[C1 * C2 + c2], sc2 = p2[C1 * C2 + C2 + c2], sh2 = p2[C1 * C2 + 2 * C2 + c2];
  float b3 = 0.f, sc3 = 0.f, sh3 = 0.f;
  if constexpr (C3 > 0) {
    b3 = p3[C2 * C3 + c3];
    sc3 = p3[C2 * C3 + C3 + c3];
    sh3 = p3[C2 * C3 + 2 * C3 + c3];
  }
  const float* s1 = bnst;
  const float* s2 = s1 + 2 * C1;
  const float* s3 = s2 + 2 * C2;
  const float rm1 = s1[c1], is1 = s1[C1 + c1], rm2 = s2[c2], is2 = s2[C2 + c2];
  float rm3 = 0.f, is3 = 0.f;
  if constexpr (C3 > 0) {
    rm3 = s3[c3];
    is3 = s3[C3 + c3];
  }

  // gradient accumulators: lane c owns row c of each layer's dW and its b / gamma / beta terms
  float dW1[C0], dW2[C1], dW3[C3 > 0 ? C2 : 1];
  float db1 = 0.f, dg1 = 0.f, dbe1 = 0.f, db2 = 0.f, dg2 = 0.f, dbe2 = 0.f, db3 = 0.f, dg3 = 0.f, dbe3 = 0.f;
#pragma unroll
  for (int k = 0; k < C0; ++k) dW1[k] = 0.f;
#pragma unroll
  for (int k = 0; k < C1; ++k) dW2[k] = 0.f;
#pragma unroll
  for (int k = 0; k < (C3 > 0 ? C2 : 1); ++k) dW3[k] = 0.f;

  float(*tl)[CL + 1] = tile[wave];
  float* x_s = vx[wave];
  float* h1_s = vh[wave][0];
  float* h2_s = vh[wave][1];
  float* g_s = vg[wave];
  const int64_t total = static_cast<int64_t>(B) * S;
  for (int64_t cs = static_cast<int64_t>(blockIdx.x) * kSbWaves + wave; cs < total;
       cs += static_cast<int64_t>(gridDim.x) * kSbWaves) {
    const int b = static_cast<int>(cs / S), s = static_cast<int>(cs - static_cast<int64_t>(b) * S);
    const float g_c = lane < CL ? gout[cs * CL + lane] : 0.0f;
    if (!__ballot(g_c != 0.0f)) continue;
    int cnt = count[cs];
    cnt = cnt < 1 ? 1 : (cnt > nsample ? nsample : cnt);
    const int32_t* lst = list + cs * nsample;
    const T cx = ctr.at(b, 0, s), cy = ctr.at(b, 1, s), cz = ctr.at(b, 2, s);

    // ---- pass 1: each channel's arg-max row (lane = row, then lane = channel over the tile) ----
    float best = -1.0f;  // outputs are >= 0
    int arg = 0;
    for (int r0 = 0; r0 < cnt; r0 += kWave) {
      const int r = r0 + lane;
      if (r < cnt) {
        const int n = lst[r];
        float x[C0];
        x[0] = static_cast<float>(pts.at(b, 0, n) - cx);
        x[1] = static_cast<float>(pts.at(b, 1, n) - cy);
        x[2] = static_cast<float>(pts.at(b, 2, n) - cz);
#pragma unroll
        for (int d = 0; d < D; ++d) x[3 + d] = feat.at(b, d, n);
        float y1[C1], y2[C2];
        sb_layer_rows<C0, C1>(x, y1, p1);
        sb_layer_rows<C1, C2>(y1, y2, p2);
        if constexpr (C3 > 0) {
          float y3[C3];
          sb_layer_rows<C2, C3>(y2, y3, p3);
#pragma unroll
          for (int c = 0; c < C3; ++c) tl[lane][c] = y3[c];
        } else {
#pragma unroll
          for (int c = 0; c < C2; ++c) tl[lane][c] = y2[c];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (lane < CL) {
        const int rn = min(kWave, cnt - r0);
        for (int j = 0; j < rn; ++j) {
          const float v = tl[j][lane];
          if (v > best) {  // strict: the first row among equal maxima
            best = v;
            arg = r0 + j;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    // ---- pass 2: the distinct routed rows (channels whose maximum is > 0) ----------------------
    uint64_t pending = __ballot(lane < CL && best > 0.0f && g_c != 0.0f);
    while (pending) {
      const int lead = __ffsll(static_cast<long long>(pending)) - 1;
      const int r = __builtin_amdgcn_readlane(arg, lead);
      const bool mine = ((pending >> lane) & 1ull) && arg == r;
      pending &= ~__ballot(mine);
      const float gh = mine ? g_c : 0.0f;  // g of the last layer's output on this row
      const int n = lst[r];
      // the row's input (uniform: every lane reads the same point)
      if (lane < C0) {
        float v;
        if (lane == 0) v = static_cast<float>(pts.at(b, 0, n) - cx);
        else if (lane == 1) v = static_cast<float>(pts.at(b, 1, n) - cy);
        else if (lane == 2) v = static_cast<float>(pts.at(b, 2, n) - cz);
        else v = feat.at(b, lane - 3, n);
        x_s[lane] = v;
      }
      if constexpr (C0 > kWave) {
        if (lane + kWave < C0) x_s[lane + kWave] = feat.at(b, lane + kWave - 3, n);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      // forward, one output channel per lane
      const float z1 = sb_dot_row<C0>(sW1, x_s, c1) + b1;
      const float a1 = z1 * sc1 + sh1;
      if (lane < C1) h1_s[lane] = a1 > 0.0f ? a1 : 0.0f;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const float z2 = sb_dot_row<C1>(sW2, h1_s, c2) + b2;
      const float a2 = z2 * sc2 + sh2;
      float gz2;
      if constexpr (C3 > 0) {
        if (lane < C2) h2_s[lane] = a2 > 0.0f ? a2 : 0.0f;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const float z3 = sb_dot_row<C2>(sW3, h2_s, c3) + b3;
        const float a3 = z3 * sc3 + sh3;
        const float ga3 = (lane < C3 && a3 > 0.0f) ? gh : 0.0f;
        const float gz3 = ga3 * sc3;
        db3 += gz3;
        dbe3 += ga3;
        dg3 += ga3 * ((z3 - rm3) * is3);
#pragma unroll
        for (int k = 0; k < C2; ++k) dW3[k] = __fmaf_rn(gz3, h2_s[k], dW3[k]);
        __builtin_amdgcn_wave_barrier();
        if (lane < C3) g_s[lane] = gz3;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const float gh2 = sb_dot_col<C2, C3>(sW3, g_s, c2);
        const float ga2 = (lane < C2 && a2 > 0.0f) ? gh2 : 0.0f;
        gz2 = ga2 * sc2;
        dbe2 += ga2;
        dg2 += ga2 * ((z2 - rm2) * is2);
      } else {
        const float ga2 = (lane < C2 && a2 > 0.0f) ? gh : 0.0f;
        gz2 = ga2 * sc2;
        dbe2 += ga2;
        dg2 += ga2 * ((z2 - rm2) * is2);
      }
      db2 += gz2;
#pragma unroll
      for (int k = 0; k < C1; ++k) dW2[k] = __fmaf_rn(gz2, h1_s[k], dW2[k]);
      __builtin_amdgcn_wave_barrier();
      if (lane < C2) g_s[lane] = gz2;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const float gh1 = sb_dot_col<C1, C2>(sW2, g_s, c1);
      const float ga1 = (lane < C1 && a1 > 0.0f) ? gh1 : 0.0f;
      const float gz1 = ga1 * sc1;
      db1 += gz1;
      dbe1 += ga1;
      dg1 += ga1 * ((z1 - rm1) * is1);
#pragma unroll
      for (int k = 0; k < C0; ++k) dW1[k] = __fmaf_rn(gz1, x_s[k], dW1[k]);
      if constexpr (D > 0) {
        if (gfeat) {  // the gather's backward: g_f_n += (W1^T g_z1)[3:]
          __builtin_amdgcn_wave_barrier();
          if (lane < C1) g_s[lane] = gz1;
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
          float* gf = gfeat + b * gfb + static_cast<int64_t>(n) * D;
          for (int d = lane; d < D; d += kWave) {
            const float gx = sb_dot_col<C0, C1>(sW1, g_s, 3 + d);
            if (gx != 0.0f) atomicAdd(gf + d, gx);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  // ---- this wave's partial gradients, in the packed layout (per layer: W, b, gamma, beta) --------
  float* o = partial + (static_cast<int64_t>(blockIdx.x) * kSbWaves + wave) * Tb::P;
  if (lane < C1) {
#pragma unroll
    for (int k = 0; k < C0; ++k) o[lane * C0 + k] = dW1[k];
    o[C0 * C1 + lane] = db1;
    o[C0 * C1 + C1 + lane] = dg1;
    o[C0 * C1 + 2 * C1 + lane] = dbe1;
  }
  float* o2 = o + Tb::P1;
  if (lane < C2) {
#pragma unroll
    for (int k = 0; k < C1; ++k) o2[lane * C1 + k] = dW2[k];
    o2[C1 * C2 + lane] = db2;
    o2[C1 * C2 + C2 + lane] = dg2;
    o2[C1 * C2 + 2 * C2 + lane] = dbe2;
  }
  if constexpr (C3 > 0) {
    float* o3 = o2 + Tb::P2;
    if (lane < C3) {
#pragma unroll
      for (int k = 0; k < C2; ++k) o3[lane * C2 + k] = dW3[k];
      o3[C2 * C3 + lane] = db3;
      o3[C2 * C3 + C3 + lane] = dg3;
      o3[C2 * C3 + 2 * C3 + lane] = dbe3;
    }
  }
}

// out[e] = sum over the nw partial rows of part[k][e] in fp64, in a fixed order (deterministic):
// 64 parameters x 16 row slices per workgroup, the slices combined in order.
__global__ __launch_bounds__(1024) void sb_sum_kernel(const float* __restrict__ part, int nw, int P,
                                                      float* __restrict__ out) {
  __shared__ double sl[16][64];
  const int tid = threadIdx.x, c = tid & 63, slice = tid >> 6;
  const int e = blockIdx.x * 64 + c;
  double acc = 0.0;
  if (e < P)
    for (int k = slice; k < nw; k += 16) acc += static_cast<double>(part[static_cast<int64_t>(k) * P + e]);
  sl[slice][c] = acc;
  __syncthreads();
  if (tid < 64 && e < P) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += sl[k][c];
    out[e] = static_cast<float>(t);
  }
}

// fc backward (deep_feat_extraction.py:15, y = W x + b, W 32 x 64): gx = W^T g per row, and the
// wave partials of dW = sum_rows g x^T, db = sum_rows g (lane f < 32 owns row f of dW).
constexpr int kFcIn = 64, kFcOut = 32;
__global__ __launch_bounds__(256) void fc_bwd_kernel(const float* __restrict__ x, int P, const float* __restrict__ params,
                                                     const float* __restrict__ g, float* __restrict__ gx,
                                                     float* __restrict__ partial) {
  __shared__ float sW[kFcOut][kFcIn + 1];
  __shared__ float rows_x[4][kFcIn];
  __shared__ float rows_g[4][kFcOut];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < kFcOut * kFcIn; i += 256) sW[i / kFcIn][i % kFcIn] = params[i];
  __syncthreads();
  float dW[kFcIn];
#pragma unroll
  for (int k = 0; k < kFcIn; ++k) dW[k] = 0.f;
  float db = 0.f;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + wave; r < P; r += static_cast<int64_t>(gridDim.x) * 4) {
    rows_x[wave][lane] = x[r * kFcIn + lane];
    if (lane < kFcOut) rows_g[wave][lane] = g[r * kFcOut + lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (gx) {  // lane = input channel
      float acc = 0.f;
#pragma unroll 8
      for (int f = 0; f < kFcOut; ++f) acc = __fmaf_rn(sW[f][lane], rows_g[wave][f], acc);
      gx[r * kFcIn + lane] = acc;
    }
    const float gf = lane < kFcOut ? rows_g[wave][lane] : 0.f;
    db += gf;
#pragma unroll
    for (int k = 0; k < kFcIn; ++k) dW[k] = __fmaf_rn(gf, rows_x[wave][k], dW[k]);
    __builtin_amdgcn_wave_barrier();
  }
  float* o = partial + (static_cast<int64_t>(blockIdx.x) * 4 + wave) * (kFcOut * kFcIn + kFcOut);
  if (lane < kFcOut) {
#pragma unroll
    for (int k = 0; k < kFcIn; ++k) o[lane * kFcIn + k] = dW[k];
    o[kFcOut * kFcIn + lane] = db;
  }
}

static int sb_grid(int64_t total) {
  const int64_t need = (total + kSbWaves - 1) / kSbWaves;
  return static_cast<int>(need < kSbMaxGrid ? (need > 0 ? need : 1) : kSbMaxGrid);
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
static int launch_sa_bwd(const void* xyz, int64_t sb, int64_t sc, int64_t sn, const void* c, int64_t cb, int64_t cc,
                         int64_t cn, int S, int B, const void* feat, int64_t fb, int64_t fd, int64_t fn,
                         const int32_t* count, const int32_t* list, int nsample, const float* params, const float* bnst,
                         const float* gout, float* gfeat, int64_t gfb, float* ws, float* gparams, hipStream_t st) {
  using Tb = SbTable<D, C1, C2, C3>;
  const int grid = sb_grid(static_cast<int64_t>(B) * S);
  PointsView<T> pv{static_cast<const T*>(xyz), sb, sc, sn};
  PointsView<T> cv{static_cast<const T*>(c), cb, cc, cn};
  SbFeat<FT> fv{static_cast<const FT*>(feat), fb, fd, fn};
  hipLaunchKernelGGL((sa_bwd_kernel<T, FT, D, C1, C2, C3>), dim3(grid), dim3(kSbThreads), 0, st, pv, cv, S, B, fv,
                     count, list, nsample, params, bnst, gout, gfeat, gfb, ws);
  if (int e = launch_status("dvcp_sa_group_mlp_backward")) return e;
  hipLaunchKernelGGL(sb_sum_kernel, dim3(ceil_div(Tb::P, 64)), dim3(1024), 0, st, ws, grid * kSbWaves, Tb::P, gparams);
  return launch_status("dvcp_sa_group_mlp_backward(sum)");
}

}  // namespace dvcp

// Workspace (fp32 wave partials) of dvcp_sa_group_mlp_backward.
extern "C" int64_t dvcp_sa_group_mlp_backward_workspace_bytes(int B, int S, int nlayer, const int* chans) {
  if (B < 0 || S < 0 || !chans || (nlayer != 2 && nlayer != 3)) return -1;
  int64_t P = 0;
  for (int l = 0; l < nlayer; ++l) P += static_cast<int64_t>(chans[l]) * chans[l + 1] + 3 * chans[l + 1];
  return static_cast<int64_t>(dvcp::sb_grid(static_cast<int64_t>(B) * S)) * dvcp::kSbWaves * P * 4;
}

extern "C" int dvcp_sa_group_mlp_backward(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                          const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B,
                                          int feat_dtype, const void* feat, int64_t fb, int64_t fd, int64_t fn, int D,
                                          const int32_t* count, const int32_t* list, int nsample, int nlayer,
                                          const int* chans, const float* params, const float* bnstat,
                                          const float* grad_out, float* grad_feat, void* workspace,
                                          float* grad_params, void* stream) {
  DVCP_REQUIRE(xyz && ctr && count && list && chans && params && bnstat && grad_out && workspace && grad_params,
               "dvcp_sa_group_mlp_backward: null pointer");
  DVCP_REQUIRE(D == 0 || feat, "dvcp_sa_group_mlp_backward: D=%d but feat is NULL", D);
  DVCP_REQUIRE(chans[0] == 3 + D, "dvcp_sa_group_mlp_backward: chans[0]=%d != 3+D", chans[0]);
  DVCP_REQUIRE(N > 0 && S >= 0 && B >= 0 && B <= 65535 && nsample > 0, "dvcp_sa_group_mlp_backward: bad sizes");
  DVCP_REQUIRE(dtype == DVCP_F32 || dtype == DVCP_F64, "dvcp_sa_group_mlp_backward: bad dtype %d", dtype);
  DVCP_REQUIRE(feat_dtype == DVCP_F32 || (D == 0 || feat_dtype == DVCP_F64), "dvcp_sa_group_mlp_backward: bad feat dtype");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0 || S == 0) {
    int64_t P = 0;
    for (int l = 0; l < nlayer; ++l) P += static_cast<int64_t>(chans[l]) * chans[l + 1] + 3 * chans[l + 1];
    if (hipMemsetAsync(grad_params, 0, P * 4, st) != hipSuccess)
      return dvcp::launch_status("dvcp_sa_group_mlp_backward(empty)");
    return DVCP_OK;
  }
  const bool f64 = dtype == DVCP_F64, ff64 = feat_dtype == DVCP_F64;
  const int64_t gfb = static_cast<int64_t>(N) * D;  // grad_feat: (B, N, D) fp32 rows
  float* ws = static_cast<float*>(workspace);
#define DVCP_SB(DD, A, Bc, Cc)                                                                                    \
  if (D == DD && chans[1] == A && chans[2] == Bc && (nlayer == 2 ? 0 : chans[3]) == Cc) {                      \
    if (f64)                                                                                                      \
      return ff64 ? dvcp::launch_sa_bwd<double, double, DD, A, Bc, Cc>(xyz, sb, sc, sn, ctr, cb, cc, cn, S, B,  \
                                                                         feat, fb, fd, fn, count, list, nsample, \
                                                                         params, bnstat, grad_out, grad_feat, gfb,  \
                                                                         ws, grad_params, st)                     \
                  : dvcp::launch_sa_bwd<double, float, DD, A, Bc, Cc>(xyz, sb, sc, sn, ctr, cb, cc, cn, S, B,    \
                                                                        feat, fb, fd, fn, count, list, nsample,  \
                                                                        params, bnstat, grad_out, grad_feat, gfb,   \
                                                                        ws, grad_params, st);                     \
    return ff64 ? dvcp::launch_sa_bwd<float, double, DD, A, Bc, Cc>(xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat,  \
                                                                      fb, fd, fn, count, list, nsample, params,      \
                                                                      bnstat, grad_out, grad_feat, gfb, ws,          \
                                                                      grad_params, st)                               \
                : dvcp::launch_sa_bwd<float, float, DD, A, Bc, Cc>(xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, \
                                                                     fd, fn, count, list, nsample, params, bnstat,   \
                                                                     grad_out, grad_feat, gfb, ws, grad_params, st); \
  }
  // the REF-R tables (deep_feat_extraction.py:10-13 + R1): sa1 without / with normals, sa2, sa3
  DVCP_SB(0, 16, 16, 32)
  DVCP_SB(3, 16, 16, 32)
  DVCP_SB(32, 32, 64, 0)
  DVCP_SB(64, 64, 64, 0)
#undef DVCP_SB
  dvcp::set_error("dvcp_sa_group_mlp_backward: unsupported table D=%d chans=%d,%d%s", D, chans[1], chans[2],
                  nlayer == 3 ? ",..." : "");
  return DVCP_EINVAL;
}

extern "C" int64_t dvcp_fe_head_backward_workspace_bytes(int P) {
  if (P < 0) return -1;
  const int64_t grid = P <= 0 ? 1 : std::min<int64_t>(1024, (static_cast<int64_t>(P) + 3) / 4);
  return grid * 4 * (dvcp::kFcOut * dvcp::kFcIn + dvcp::kFcOut) * 4;
}

// fc backward: x (P x 64) fp32 rows (the sa3 output), params fc.W (32 x 64) | fc.b (32), grad (P x 32);
// grad_x (P x 64, optional), grad_params (32 x 64 + 32).
extern "C" int dvcp_fe_head_backward(const float* x, int P, const float* params, const float* grad, float* grad_x,
                                     void* workspace, float* grad_params, void* stream) {
  DVCP_REQUIRE(x && params && grad && workspace && grad_params, "dvcp_fe_head_backward: null pointer");
  DVCP_REQUIRE(P >= 0, "dvcp_fe_head_backward: bad size");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int grid = static_cast<int>(P <= 0 ? 1 : std::min<int64_t>(1024, (static_cast<int64_t>(P) + 3) / 4));
  float* ws = static_cast<float*>(workspace);
  hipLaunchKernelGGL(dvcp::fc_bwd_kernel, dim3(grid), dim3(256), 0, st, x, P, params, grad, grad_x, ws);
  if (int e = dvcp::launch_status("dvcp_fe_head_backward")) return e;
  const int PP = dvcp::kFcOut * dvcp::kFcIn + dvcp::kFcOut;
  hipLaunchKernelGGL(dvcp::sb_sum_kernel, dim3(dvcp::ceil_div(PP, 64)), dim3(1024), 0, st, ws, grid * 4, PP,
                     grad_params);
  return dvcp::launch_status("dvcp_fe_head_backward(sum)");
}
