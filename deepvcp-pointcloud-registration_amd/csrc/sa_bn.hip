// sa_bn.hip -- the grouped set-abstraction MLP with BatchNorm in TRAINING mode (batch statistics):
// the statistics passes of the forward and the dense backward (pointnet2_utils.py:195-200 with the
// module in train(), driven by train.py:105-125 with the whole model trainable).
//
// Forward per grouped entry e = (centre s, slot j), j < nsample (padding slots repeat the first hit
// and are entries of the batch like any other, so they count in the statistics):
//   z_l = W_l h_{l-1} + b_l,  xh_l = (z_l - mu_l) * istd_l,  y_l = gamma_l xh_l + beta_l,
//   h_l = relu(y_l),  out[s][c] = max_j h_L[e][c]
// with mu_l, var_l the biased mean / variance of z_l over all M = B * S * nsample entries (BN2d
// over (B, H, W)), istd_l = 1 / sqrt(var_l + eps).  y is evaluated as z * scale + shift with
// scale = gamma * istd, shift = beta - mu * scale: the forward kernel's (sa_mlp*.hip) arithmetic.
//
// dvcp_sa_bn_stats(layer l): sum z_l and sum z_l^2 per channel in fp64, layers below l
// normalised with their (already known) batch statistics.  One wave per centre; lane = slot; the
// centre's z_l rows go through an LDS tile and lanes (channel, slot group) sum its columns.
//
// dvcp_sa_bn_backward: torch's batch-norm backward,
//   gy_l = gh_l [y_l > 0],  A_l = sum_e gy_l (= dbeta),  B_l = sum_e gy_l xh_l (= dgamma),
//   gz_l = scale_l (gy_l - A_l / M - xh_l B_l / M),  gh_{l-1} = W_l^T gz_l,
//   dW_l = sum_e gz_l h_{l-1}^T,  db_l = sum_e gz_l,  g_f += (W_1^T gz_1)[3:]  (the :59 gather)
// gz_l is dense (every entry carries the mean terms), so layer l's sums need A, B of the layers
// above it.  mode = L: A_L, B_L over the routed (arg-max) rows only (gy_L is zero elsewhere);
// mode = k < L: one dense recompute pass over every entry gives A_k, B_k; mode = 0: the dense pass
// with every A, B known accumulates dW, db and scatters the feature gradient.  The nsample - cnt
// padding entries of a centre are one virtual row of weight nsample - cnt (identical rows, never
// routed: torch.max takes the first of equal maxima).  Per-wave partials are summed in a fixed
// order in fp64, so all parameter gradients are deterministic; the feature scatter uses atomics.
#include "common.h"

#include <algorithm>

namespace dvcp {

constexpr int kBnWaves = 4;
constexpr int kBnThreads = kBnWaves * kWave;
constexpr int kBnMaxGrid = 1024;

template <typename FT>
struct BnFeat {
  const FT* p;
  int64_t fb, fd, fn;
  __device__ __forceinline__ float at(int b, int d, int64_t n) const {
    return static_cast<float>(p[b * fb + d * fd + n * fn]);
  }
};

// Layer pack (per layer, Cin -> Cout): W[Cout][Cin] | bias | scale | shift | mean | istd | ga | gb,
// ga = A / M and gb = B / M of the layer (zero until known).
__host__ __device__ constexpr int bn_layer_size(int cin, int cout) { return cout * cin + 7 * cout; }

template <int D, int C1, int C2, int C3>
struct BnTable {
  static constexpr int C0 = 3 + D;
  static constexpr int L = C3 > 0 ? 3 : 2;
  static constexpr int CL = C3 > 0 ? C3 : C2;
  static constexpr int CMAX = C1 > C2 ? (C1 > C3 ? C1 : C3) : (C2 > C3 ? C2 : C3);
  static constexpr int O1 = 0;
  static constexpr int O2 = bn_layer_size(C0, C1);
  static constexpr int O3 = O2 + bn_layer_size(C1, C2);
  // packed parameter gradient (dvcp_sa_group_mlp_backward's layout): per layer W, b, gamma, beta
  static constexpr int P1 = C0 * C1 + 3 * C1;
  static constexpr int P2 = C1 * C2 + 3 * C2;
  static constexpr int P3 = C3 > 0 ? C2 * C3 + 3 * C3 : 0;
  static constexpr int P = P1 + P2 + P3;
  static constexpr int LW1 = C1 * (C0 + 1), LW2 = C2 * (C1 + 1), LW3 = C3 > 0 ? C3 * (C2 + 1) : 0;
};

// lane = slot: h = relu((W x + b) * scale + shift), weights as wave-uniform scalar loads
template <int CIN, int COUT>
__device__ __forceinline__ void bn_rows(const float (&x)[CIN], float (&h)[COUT], const float* __restrict__ p) {
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    float acc = 0.0f;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc = __fmaf_rn(p[co * CIN + ci], x[ci], acc);
    const float v = (acc + p[CIN * COUT + co]) * p[CIN * COUT + COUT + co] + p[CIN * COUT + 2 * COUT + co];
    h[co] = v > 0.0f ? v : 0.0f;
  }
}
// lane = slot: z = W x + b (the layer whose statistics are being taken)
template <int CIN, int COUT>
__device__ __forceinline__ void bn_rows_raw(const float (&x)[CIN], float (&z)[COUT], const float* __restrict__ p) {
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    float acc = 0.0f;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc = __fmaf_rn(p[co * CIN + ci], x[ci], acc);
    z[co] = acc + p[CIN * COUT + co];
  }
}

template <typename T, typename FT, int D>
__device__ __forceinline__ void bn_load_x(float (&x)[3 + D], PointsView<T> pts, BnFeat<FT> feat, int b, int n, T cx,
                                          T cy, T cz) {
  x[0] = static_cast<float>(pts.at(b, 0, n) - cx);
  x[1] = static_cast<float>(pts.at(b, 1, n) - cy);
  x[2] = static_cast<float>(pts.at(b, 2, n) - cz);
#pragma unroll
  for (int d = 0; d < D; ++d) x[3 + d] = feat.at(b, d, n);
}

// ---- statistics pass ----------------------------------------------------------------------------
template <typename T, typename FT, int D, int C1, int C2, int C3, int LAYER>
__global__ __launch_bounds__(kBnThreads) void sa_bn_stats_kernel(PointsView<T> pts, PointsView<T> ctr, int S, int B,
                                                                 BnFeat<FT> feat, const int32_t* __restrict__ count,
                                                                 const int32_t* __restrict__ list, int nsample,
                                                                 const float* __restrict__ pack,
                                                                 double* __restrict__ partial) {
  using Tb = BnTable<D, C1, C2, C3>;
  constexpr int C0 = Tb::C0;
  constexpr int CZ = LAYER == 1 ? C1 : (LAYER == 2 ? C2 : C3);
  constexpr int G = kWave / CZ;  // slot groups (CZ divides 64)
  __shared__ float tile[kBnWaves][kWave][CZ + 1];
  __shared__ double red[kBnWaves][2][kWave];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane % CZ, grp = lane / CZ;
  const float* p1 = pack + Tb::O1;
  const float* p2 = pack + Tb::O2;
  const float* p3 = pack + Tb::O3;
  double s1 = 0.0, s2 = 0.0;
  float(*tl)[CZ + 1] = tile[wave];
  const int64_t total = static_cast<int64_t>(B) * S;
  for (int64_t cs = static_cast<int64_t>(blockIdx.x) * kBnWaves + wave; cs < total;
       cs += static_cast<int64_t>(gridDim.x) * kBnWaves) {
    const int b = static_cast<int>(cs / S), s = static_cast<int>(cs - static_cast<int64_t>(b) * S);
    int cnt = count[cs];
    cnt = cnt < 1 ? 1 : (cnt > nsample ? nsample : cnt);
    const int32_t* lst = list + cs * nsample;
    const T cx = ctr.at(b, 0, s), cy = ctr.at(b, 1, s), cz = ctr.at(b, 2, s);
    for (int r0 = 0; r0 < nsample; r0 += kWave) {
      const int r = r0 + lane;
      if (r < nsample) {
        const int n = lst[r < cnt ? r : 0];
        float x[C0];
        bn_load_x<T, FT, D>(x, pts, feat, b, n, cx, cy, cz);
        float z[CZ];
        if constexpr (LAYER == 1) {
          bn_rows_raw<C0, C1>(x, z, p1);
        } else {
          float h1[C1];
          bn_rows<C0, C1>(x, h1, p1);
          if constexpr (LAYER == 2) {
            bn_rows_raw<C1, C2>(h1, z, p2);
          } else {
            float h2[C2];
            bn_rows<C1, C2>(h1, h2, p2);
            bn_rows_raw<C2, C3>(h2, z, p3);
          }
        }
#pragma unroll
        for (int k = 0; k < CZ; ++k) tl[lane][k] = z[k];
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const int rn = min(kWave, nsample - r0);
      for (int j = grp; j < rn; j += G) {
        const double v = static_cast<double>(tl[j][c]);
        s1 += v;
        s2 += v * v;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
  // this wave's per-channel sums, the slot groups combined in a fixed order
  red[wave][0][lane] = s1;
  red[wave][1][lane] = s2;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (lane < CZ) {
    double a = 0.0, q = 0.0;
    for (int g = 0; g < G; ++g) {
      a += red[wave][0][g * CZ + lane];
      q += red[wave][1][g * CZ + lane];
    }
    double* o = partial + (static_cast<int64_t>(blockIdx.x) * kBnWaves + wave) * (2 * CZ);
    o[lane] = a;
    o[CZ + lane] = q;
  }
}

// ---- dense backward pass ------------------------------------------------------------------------
// Lane-per-output-channel helpers over LDS-staged weights (row stride CIN + 1).
template <int CIN>
__device__ __forceinline__ float bn_dot_row(const float* __restrict__ W, const float* __restrict__ v, int row) {
  float acc = 0.0f;
#pragma unroll 8
  for (int k = 0; k < CIN; ++k) acc = __fmaf_rn(W[row * (CIN + 1) + k], v[k], acc);
  return acc;
}
template <int CIN, int COUT>
__device__ __forceinline__ float bn_dot_col(const float* __restrict__ W, const float* __restrict__ gz, int col) {
  float acc = 0.0f;
#pragma unroll 8
  for (int c = 0; c < COUT; ++c) acc = __fmaf_rn(W[c * (CIN + 1) + col], gz[c], acc);
  return acc;
}

// Per-lane constants of one layer (lane = output channel).
struct BnLane {
  float bias, scale, shift, mean, istd, ga, gb;
  __device__ __forceinline__ void load(const float* p, int cin, int cout, int c) {
    const float* v = p + cout * cin;
    bias = v[c];
    scale = v[cout + c];
    shift = v[2 * cout + c];
    mean = v[3 * cout + c];
    istd = v[4 * cout + c];
    ga = v[5 * cout + c];
    gb = v[6 * cout + c];
  }
  // gz = scale (gy - w (A/M + xh B/M)): w entries of this row (padding rows folded)
  __device__ __forceinline__ float gz(float gy, float xh, float w) const {
    return scale * (gy - w * (ga + xh * gb));
  }
};

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// MODE: 0 = parameter / feature gradients; k in 1..L = the sums A_k, B_k.
template <typename T, typename FT, int D, int C1, int C2, int C3, int MODE>
__global__ __launch_bounds__(kBnThreads) void sa_bn_bwd_kernel(
    PointsView<T> pts, PointsView<T> ctr, int S, int B, BnFeat<FT> feat, const int32_t* __restrict__ count,
    const int32_t* __restrict__ list, int nsample, const float* __restrict__ pack, const float* __restrict__ gout,
    float* __restrict__ gfeat, int64_t gfb, float* __restrict__ partial, double* __restrict__ dpartial) {
  using Tb = BnTable<D, C1, C2, C3>;
  constexpr int C0 = Tb::C0, CL = Tb::CL, L = Tb::L;
  constexpr bool FINAL = MODE == 0;
  __shared__ float sW1[Tb::LW1], sW2[Tb::LW2], sW3[Tb::LW3 > 0 ? Tb::LW3 : 1];
  __shared__ float tile[kBnWaves][kWave][CL + 1];  // pass 1: last-layer rows
  __shared__ float vx[kBnWaves][C0 + 1];           // pass 2: the row's input
  __shared__ float vh[kBnWaves][2][Tb::CMAX];      // h1, h2 of the row
  __shared__ float vg[kBnWaves][Tb::CMAX];         // gz of the layer above

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* p1 = pack + Tb::O1;
  const float* p2 = pack + Tb::O2;
  const float* p3 = pack + Tb::O3;
  for (int i = tid; i < C1 * C0; i += kBnThreads) sW1[(i / C0) * (C0 + 1) + i % C0] = p1[i];
  for (int i = tid; i < C2 * C1; i += kBnThreads) sW2[(i / C1) * (C1 + 1) + i % C1] = p2[i];
  if constexpr (C3 > 0)
    for (int i = tid; i < C3 * C2; i += kBnThreads) sW3[(i / C2) * (C2 + 1) + i % C2] = p3[i];
  __syncthreads();

  const int c1 = lane < C1 ? lane : 0, c2 = lane < C2 ? lane : 0, c3 = lane < (C3 > 0 ? C3 : 1) ? lane : 0;
  BnLane q1, q2, q3;
  q1.load(p1, C0, C1, c1);
  q2.load(p2, C1, C2, c2);
  if constexpr (C3 > 0) q3.load(p3, C2, C3, c3);

  // accumulators: FINAL -- lane c owns row c of each dW and db_l[c]; sums -- A, B of layer MODE
  constexpr int NW1 = FINAL ? C0 : 1, NW2 = FINAL ? C1 : 1, NW3 = (FINAL && C3 > 0) ? C2 : 1;
  float dW1[NW1], dW2[NW2], dW3[NW3];
  float db1 = 0.f, db2 = 0.f, db3 = 0.f;
#pragma unroll
  for (int k = 0; k < NW1; ++k) dW1[k] = 0.f;
#pragma unroll
  for (int k = 0; k < NW2; ++k) dW2[k] = 0.f;
#pragma unroll
  for (int k = 0; k < NW3; ++k) dW3[k] = 0.f;
  double accA = 0.0, accB = 0.0;

  float(*tl)[CL + 1] = tile[wave];
  float* x_s = vx[wave];
  float* h1_s = vh[wave][0];
  float* h2_s = vh[wave][1];
  float* g_s = vg[wave];
  const int64_t total = static_cast<int64_t>(B) * S;
  for (int64_t cs = static_cast<int64_t>(blockIdx.x) * kBnWaves + wave; cs < total;
       cs += static_cast<int64_t>(gridDim.x) * kBnWaves) {
    const int b = static_cast<int>(cs / S), s = static_cast<int>(cs - static_cast<int64_t>(b) * S);
    const float g_c = lane < CL ? gout[cs * CL + lane] : 0.0f;
    if constexpr (MODE == L) {
      if (!__ballot(g_c != 0.0f)) continue;  // only routed rows carry gy_L
    }
    int cnt = count[cs];
    cnt = cnt < 1 ? 1 : (cnt > nsample ? nsample : cnt);
    const int32_t* lst = list + cs * nsample;
    const T cx = ctr.at(b, 0, s), cy = ctr.at(b, 1, s), cz = ctr.at(b, 2, s);

    // ---- pass 1: each channel's arg-max row among the distinct slots (lane = slot) -------------
    float best = -1.0f;  // outputs are >= 0
    int arg = 0;
    for (int r0 = 0; r0 < cnt; r0 += kWave) {
      const int r = r0 + lane;
      if (r < cnt) {
        float x[C0];
        bn_load_x<T, FT, D>(x, pts, feat, b, lst[r], cx, cy, cz);
        float h1[C1], h2[C2];
        bn_rows<C0, C1>(x, h1, p1);
        bn_rows<C1, C2>(h1, h2, p2);
        if constexpr (C3 > 0) {
          float h3[C3];
          bn_rows<C2, C3>(h2, h3, p3);
#pragma unroll
          for (int k = 0; k < C3; ++k) tl[lane][k] = h3[k];
        } else {
#pragma unroll
          for (int k = 0; k < C2; ++k) tl[lane][k] = h2[k];
        }
      }
      wave_sync_lds();
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
      wave_sync_lds();
    }
    // lane c < CL: the routed gradient of channel c goes to row `arg` (nothing if the max is 0)
    const float rg = (lane < CL && best > 0.0f) ? g_c : 0.0f;
    const int rarg = (lane < CL && best > 0.0f && g_c != 0.0f) ? arg : -1;

    // ---- pass 2: the rows (lane = output channel) -----------------------------------------------
    // MODE == L: the distinct routed rows; otherwise every distinct row plus one virtual row for
    // the nsample - cnt padding slots.
    uint64_t pending = MODE == L ? __ballot(rarg >= 0) : 0ull;
    const int nv = MODE == L ? 0 : cnt + (cnt < nsample ? 1 : 0);
    for (int v = 0;; ++v) {
      int r;
      float w = 1.0f;
      if constexpr (MODE == L) {
        if (!pending) break;
        const int lead = __ffsll(static_cast<long long>(pending)) - 1;
        r = __builtin_amdgcn_readlane(rarg, lead);
        pending &= ~__ballot(rarg == r);
      } else {
        if (v >= nv) break;
        if (v < cnt) {
          r = v;
        } else {
          r = 0;
          w = static_cast<float>(nsample - cnt);
        }
      }
      const bool routed_row = v < cnt || MODE == L;  // the padding row is never routed
      const int n = lst[r];
      if (lane < C0) {
        float xv;
        if (lane == 0) xv = static_cast<float>(pts.at(b, 0, n) - cx);
        else if (lane == 1) xv = static_cast<float>(pts.at(b, 1, n) - cy);
        else if (lane == 2) xv = static_cast<float>(pts.at(b, 2, n) - cz);
        else xv = feat.at(b, lane - 3, n);
        x_s[lane] = xv;
      }
      if constexpr (C0 > kWave) {
        if (lane + kWave < C0) x_s[lane + kWave] = feat.at(b, lane + kWave - 3, n);
      }
      wave_sync_lds();
      // forward, one output channel per lane
      const float z1 = bn_dot_row<C0>(sW1, x_s, c1) + q1.bias;
      const float y1 = z1 * q1.scale + q1.shift;
      const float xh1 = (z1 - q1.mean) * q1.istd;
      if (lane < C1) h1_s[lane] = y1 > 0.0f ? y1 : 0.0f;
      wave_sync_lds();
      const float z2 = bn_dot_row<C1>(sW2, h1_s, c2) + q2.bias;
      const float y2 = z2 * q2.scale + q2.shift;
      const float xh2 = (z2 - q2.mean) * q2.istd;
      float gy2;
      if constexpr (C3 > 0) {
        if (lane < C2) h2_s[lane] = y2 > 0.0f ? y2 : 0.0f;
        wave_sync_lds();
        const float z3 = bn_dot_row<C2>(sW3, h2_s, c3) + q3.bias;
        const float y3 = z3 * q3.scale + q3.shift;
        const float xh3 = (z3 - q3.mean) * q3.istd;
        const float gh3 = (routed_row && rarg == r) ? rg : 0.0f;
        const float gy3 = (lane < C3 && y3 > 0.0f) ? gh3 : 0.0f;
        if constexpr (MODE == 3) {
          accA += static_cast<double>(gy3);
          accB += static_cast<double>(gy3) * static_cast<double>(xh3);
          wave_sync_lds();
          continue;
        }
        const float gz3 = lane < C3 ? q3.gz(gy3, xh3, w) : 0.0f;
        if constexpr (FINAL) {
          db3 += gz3;
#pragma unroll
          for (int k = 0; k < NW3; ++k) dW3[k] = __fmaf_rn(gz3, h2_s[k], dW3[k]);
        }
        wave_sync_lds();
        if (lane < C3) g_s[lane] = gz3;
        wave_sync_lds();
        const float gh2 = bn_dot_col<C2, C3>(sW3, g_s, c2);
        gy2 = (lane < C2 && y2 > 0.0f) ? gh2 : 0.0f;
      } else {
        const float gh2 = (routed_row && rarg == r) ? rg : 0.0f;
        gy2 = (lane < C2 && y2 > 0.0f) ? gh2 : 0.0f;
      }
      if constexpr (MODE == 2) {
        accA += static_cast<double>(gy2);
        accB += static_cast<double>(gy2) * static_cast<double>(xh2);
        wave_sync_lds();
        continue;
      }
      const float gz2 = lane < C2 ? q2.gz(gy2, xh2, w) : 0.0f;
      if constexpr (FINAL) {
        db2 += gz2;
#pragma unroll
        for (int k = 0; k < NW2; ++k) dW2[k] = __fmaf_rn(gz2, h1_s[k], dW2[k]);
      }
      wave_sync_lds();
      if (lane < C2) g_s[lane] = gz2;
      wave_sync_lds();
      const float gh1 = bn_dot_col<C1, C2>(sW2, g_s, c1);
      const float gy1 = (lane < C1 && y1 > 0.0f) ? gh1 : 0.0f;
      if constexpr (MODE == 1) {
        accA += static_cast<double>(gy1);
        accB += static_cast<double>(gy1) * static_cast<double>(xh1);
        wave_sync_lds();
        continue;
      }
      if constexpr (FINAL) {
        const float gz1 = lane < C1 ? q1.gz(gy1, xh1, w) : 0.0f;
        db1 += gz1;
#pragma unroll
        for (int k = 0; k < NW1; ++k) dW1[k] = __fmaf_rn(gz1, x_s[k], dW1[k]);
        if constexpr (D > 0) {
          if (gfeat) {  // the gather's backward: g_f_n += (W1^T gz1)[3:] (w folded into gz1)
            wave_sync_lds();
            if (lane < C1) g_s[lane] = gz1;
            wave_sync_lds();
            float* gf = gfeat + b * gfb + static_cast<int64_t>(n) * D;
            for (int d = lane; d < D; d += kWave) {
              const float gx = bn_dot_col<C0, C1>(sW1, g_s, 3 + d);
              if (gx != 0.0f) atomicAdd(gf + d, gx);
            }
          }
        }
      }
      wave_sync_lds();
    }
  }
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * kBnWaves + wave;
  if constexpr (FINAL) {
    // this wave's partial gradients in the packed layout (gamma / beta slots: zero, the host fills
    // them from the sums passes)
    float* o = partial + gw * Tb::P;
    if (lane < C1) {
#pragma unroll
      for (int k = 0; k < C0; ++k) o[lane * C0 + k] = dW1[k];
      o[C0 * C1 + lane] = db1;
      o[C0 * C1 + C1 + lane] = 0.f;
      o[C0 * C1 + 2 * C1 + lane] = 0.f;
    }
    float* o2 = o + Tb::P1;
    if (lane < C2) {
#pragma unroll
      for (int k = 0; k < C1; ++k) o2[lane * C1 + k] = dW2[k];
      o2[C1 * C2 + lane] = db2;
      o2[C1 * C2 + C2 + lane] = 0.f;
      o2[C1 * C2 + 2 * C2 + lane] = 0.f;
    }
    if constexpr (C3 > 0) {
      float* o3 = o2 + Tb::P2;
      if (lane < C3) {
#pragma unroll
        for (int k = 0; k < C2; ++k) o3[lane * C2 + k] = dW3[k];
        o3[C2 * C3 + lane] = db3;
        o3[C2 * C3 + C3 + lane] = 0.f;
        o3[C2 * C3 + 2 * C3 + lane] = 0.f;
      }
    }
  } else {
    constexpr int CM = MODE == 1 ? C1 : (MODE == 2 ? C2 : C3);
    if (lane < CM) {
      double* o = dpartial + gw * (2 * CM);
      o[lane] = accA;
      o[CM + lane] = accB;
    }
  }
}

// out[e] = sum over the nw partial rows of part[k][e] in fp64, in a fixed order (deterministic).
template <typename PT, typename OT>
__global__ __launch_bounds__(1024) void bn_sum_kernel(const PT* __restrict__ part, int nw, int P, OT* __restrict__ out) {
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
    out[e] = static_cast<OT>(t);
  }
}

static int bn_grid(int64_t total) {
  const int64_t need = (total + kBnWaves - 1) / kBnWaves;
  return static_cast<int>(need < kBnMaxGrid ? (need > 0 ? need : 1) : kBnMaxGrid);
}

struct BnArgs {
  const void* xyz;
  int64_t sb, sc, sn;
  const void* ctr;
  int64_t cb, cc, cn;
  int S, B;
  const void* feat;
  int64_t fb, fd, fn;
  const int32_t* count;
  const int32_t* list;
  int nsample;
  const float* pack;
  hipStream_t st;
};

template <typename T, typename FT, int D, int C1, int C2, int C3, int LAYER>
static int launch_stats(const BnArgs& a, void* ws, double* sums) {
  constexpr int CZ = LAYER == 1 ? C1 : (LAYER == 2 ? C2 : C3);
  const int grid = bn_grid(static_cast<int64_t>(a.B) * a.S);
  PointsView<T> pv{static_cast<const T*>(a.xyz), a.sb, a.sc, a.sn};
  PointsView<T> cv{static_cast<const T*>(a.ctr), a.cb, a.cc, a.cn};
  BnFeat<FT> fv{static_cast<const FT*>(a.feat), a.fb, a.fd, a.fn};
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL((sa_bn_stats_kernel<T, FT, D, C1, C2, C3, LAYER>), dim3(grid), dim3(kBnThreads), 0, a.st, pv,
                     cv, a.S, a.B, fv, a.count, a.list, a.nsample, a.pack, part);
  if (int e = launch_status("dvcp_sa_bn_stats")) return e;
  hipLaunchKernelGGL((bn_sum_kernel<double, double>), dim3(ceil_div(2 * CZ, 64)), dim3(1024), 0, a.st, part,
                     grid * kBnWaves, 2 * CZ, sums);
  return launch_status("dvcp_sa_bn_stats(sum)");
}

template <typename T, typename FT, int D, int C1, int C2, int C3, int MODE>
static int launch_bwd(const BnArgs& a, const float* gout, float* gfeat, int64_t gfb, void* ws, double* sums,
                      float* gparams) {
  using Tb = BnTable<D, C1, C2, C3>;
  const int grid = bn_grid(static_cast<int64_t>(a.B) * a.S);
  PointsView<T> pv{static_cast<const T*>(a.xyz), a.sb, a.sc, a.sn};
  PointsView<T> cv{static_cast<const T*>(a.ctr), a.cb, a.cc, a.cn};
  BnFeat<FT> fv{static_cast<const FT*>(a.feat), a.fb, a.fd, a.fn};
  hipLaunchKernelGGL((sa_bn_bwd_kernel<T, FT, D, C1, C2, C3, MODE>), dim3(grid), dim3(kBnThreads), 0, a.st, pv, cv,
                     a.S, a.B, fv, a.count, a.list, a.nsample, a.pack, gout, gfeat, gfb, static_cast<float*>(ws),
                     static_cast<double*>(ws));
  if (int e = launch_status("dvcp_sa_bn_backward")) return e;
  if constexpr (MODE == 0) {
    hipLaunchKernelGGL((bn_sum_kernel<float, float>), dim3(ceil_div(Tb::P, 64)), dim3(1024), 0, a.st,
                       static_cast<const float*>(ws), grid * kBnWaves, Tb::P, gparams);
  } else {
    constexpr int CM = MODE == 1 ? C1 : (MODE == 2 ? C2 : C3);
    hipLaunchKernelGGL((bn_sum_kernel<double, double>), dim3(ceil_div(2 * CM, 64)), dim3(1024), 0, a.st,
                       static_cast<const double*>(ws), grid * kBnWaves, 2 * CM, sums);
  }
  return launch_status("dvcp_sa_bn_backward(sum)");
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
static int dispatch_stats(const BnArgs& a, int layer, void* ws, double* sums) {
  if (layer == 1) return launch_stats<T, FT, D, C1, C2, C3, 1>(a, ws, sums);
  if (layer == 2) return launch_stats<T, FT, D, C1, C2, C3, 2>(a, ws, sums);
  if constexpr (C3 > 0)
    if (layer == 3) return launch_stats<T, FT, D, C1, C2, C3, 3>(a, ws, sums);
  set_error("dvcp_sa_bn_stats: layer %d out of range", layer);
  return DVCP_EINVAL;
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
static int dispatch_bwd(const BnArgs& a, int mode, const float* gout, float* gfeat, int64_t gfb, void* ws,
                        double* sums, float* gparams) {
  if (mode == 0) return launch_bwd<T, FT, D, C1, C2, C3, 0>(a, gout, gfeat, gfb, ws, sums, gparams);
  if (mode == 1) return launch_bwd<T, FT, D, C1, C2, C3, 1>(a, gout, gfeat, gfb, ws, sums, gparams);
  if (mode == 2) return launch_bwd<T, FT, D, C1, C2, C3, 2>(a, gout, gfeat, gfb, ws, sums, gparams);
  if constexpr (C3 > 0)
    if (mode == 3) return launch_bwd<T, FT, D, C1, C2, C3, 3>(a, gout, gfeat, gfb, ws, sums, gparams);
  set_error("dvcp_sa_bn_backward: mode %d out of range", mode);
  return DVCP_EINVAL;
}

static int64_t bn_pack_floats(int nlayer, const int* chans) {
  int64_t n = 0;
  for (int l = 0; l < nlayer; ++l) n += bn_layer_size(chans[l], chans[l + 1]);
  return n;
}

}  // namespace dvcp

// The REF-R tables (deep_feat_extraction.py:10-13 + R1): sa1 without / with normals, sa2, sa3.
#define DVCP_BN_TABLES(X) \
  X(0, 16, 16, 32)        \
  X(3, 16, 16, 32)        \
  X(32, 32, 64, 0)        \
  X(64, 64, 64, 0)

extern "C" int64_t dvcp_sa_bn_workspace_bytes(int B, int S, int nlayer, const int* chans) {
  if (B < 0 || S < 0 || !chans || (nlayer != 2 && nlayer != 3)) return -1;
  int64_t P = 0, cmax = 0;
  for (int l = 0; l < nlayer; ++l) {
    P += static_cast<int64_t>(chans[l]) * chans[l + 1] + 3 * chans[l + 1];
    cmax = std::max<int64_t>(cmax, chans[l + 1]);
  }
  const int64_t nw = static_cast<int64_t>(dvcp::bn_grid(static_cast<int64_t>(B) * S)) * dvcp::kBnWaves;
  return std::max(nw * P * 4, nw * 2 * cmax * 8);
}

extern "C" int64_t dvcp_sa_bn_pack_floats(int nlayer, const int* chans) {
  if (!chans || (nlayer != 2 && nlayer != 3)) return -1;
  return dvcp::bn_pack_floats(nlayer, chans);
}

static int bn_check(const char* who, int dtype, const void* xyz, const void* ctr, int N, int S, int B, int feat_dtype,
                    const void* feat, int D, const int32_t* count, const int32_t* list, int nsample, int nlayer,
                    const int* chans, const float* pack, const void* workspace) {
  DVCP_REQUIRE(xyz && ctr && count && list && chans && pack && workspace, "%s: null pointer", who);
  DVCP_REQUIRE(nlayer == 2 || nlayer == 3, "%s: nlayer=%d", who, nlayer);
  DVCP_REQUIRE(D == 0 || feat, "%s: D=%d but feat is NULL", who, D);
  DVCP_REQUIRE(chans[0] == 3 + D, "%s: chans[0]=%d != 3+D", who, chans[0]);
  DVCP_REQUIRE(N > 0 && S >= 0 && B >= 0 && B <= 65535 && nsample > 0, "%s: bad sizes", who);
  DVCP_REQUIRE(dtype == DVCP_F32 || dtype == DVCP_F64, "%s: bad dtype %d", who, dtype);
  DVCP_REQUIRE(feat_dtype == DVCP_F32 || (D == 0 || feat_dtype == DVCP_F64), "%s: bad feat dtype", who);
  return DVCP_OK;
}

extern "C" int dvcp_sa_bn_stats(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const void* ctr,
                                int64_t cb, int64_t cc, int64_t cn, int S, int B, int feat_dtype, const void* feat,
                                int64_t fb, int64_t fd, int64_t fn, int D, const int32_t* count, const int32_t* list,
                                int nsample, int nlayer, const int* chans, const float* pack, int layer,
                                void* workspace, double* sums, void* stream) {
  if (int e = bn_check("dvcp_sa_bn_stats", dtype, xyz, ctr, N, S, B, feat_dtype, feat, D, count, list, nsample, nlayer,
                       chans, pack, workspace))
    return e;
  DVCP_REQUIRE(sums, "dvcp_sa_bn_stats: null sums");
  DVCP_REQUIRE(layer >= 1 && layer <= nlayer, "dvcp_sa_bn_stats: layer %d of %d", layer, nlayer);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0 || S == 0) {
    if (hipMemsetAsync(sums, 0, 2 * chans[layer] * sizeof(double), st) != hipSuccess)
      return dvcp::launch_status("dvcp_sa_bn_stats(empty)");
    return DVCP_OK;
  }
  const dvcp::BnArgs a{xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, fd, fn, count, list, nsample, pack, st};
  const bool f64 = dtype == DVCP_F64, ff64 = feat_dtype == DVCP_F64;
#define DVCP_BN_S(DD, A1, A2, A3)                                                                           \
  if (D == DD && chans[1] == A1 && chans[2] == A2 && (nlayer == 2 ? 0 : chans[3]) == A3) {                 \
    if (f64)                                                                                                \
      return ff64 ? dvcp::dispatch_stats<double, double, DD, A1, A2, A3>(a, layer, workspace, sums)         \
                  : dvcp::dispatch_stats<double, float, DD, A1, A2, A3>(a, layer, workspace, sums);         \
    return ff64 ? dvcp::dispatch_stats<float, double, DD, A1, A2, A3>(a, layer, workspace, sums)            \
                : dvcp::dispatch_stats<float, float, DD, A1, A2, A3>(a, layer, workspace, sums);            \
  }
  DVCP_BN_TABLES(DVCP_BN_S)
#undef DVCP_BN_S
  dvcp::set_error("dvcp_sa_bn_stats: unsupported table D=%d chans=%d,%d", D, chans[1], chans[2]);
  return DVCP_EINVAL;
}

extern "C" int dvcp_sa_bn_backward(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                   const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B, int feat_dtype,
                                   const void* feat, int64_t fb, int64_t fd, int64_t fn, int D, const int32_t* count,
                                   const int32_t* list, int nsample, int nlayer, const int* chans, const float* pack,
                                   int mode, const float* grad_out, float* grad_feat, void* workspace, double* sums,
                                   float* grad_params, void* stream) {
  if (int e = bn_check("dvcp_sa_bn_backward", dtype, xyz, ctr, N, S, B, feat_dtype, feat, D, count, list, nsample,
                       nlayer, chans, pack, workspace))
    return e;
  DVCP_REQUIRE(grad_out, "dvcp_sa_bn_backward: null grad_out");
  DVCP_REQUIRE(mode >= 0 && mode <= nlayer, "dvcp_sa_bn_backward: mode %d of %d", mode, nlayer);
  DVCP_REQUIRE(mode == 0 ? grad_params != nullptr : sums != nullptr, "dvcp_sa_bn_backward: null output");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0 || S == 0) {
    int64_t P = 0;
    for (int l = 0; l < nlayer; ++l) P += static_cast<int64_t>(chans[l]) * chans[l + 1] + 3 * chans[l + 1];
    const hipError_t e = mode == 0 ? hipMemsetAsync(grad_params, 0, P * 4, st)
                                   : hipMemsetAsync(sums, 0, 2 * chans[mode] * sizeof(double), st);
    if (e != hipSuccess) return dvcp::launch_status("dvcp_sa_bn_backward(empty)");
    return DVCP_OK;
  }
  const dvcp::BnArgs a{xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, fd, fn, count, list, nsample, pack, st};
  const bool f64 = dtype == DVCP_F64, ff64 = feat_dtype == DVCP_F64;
  const int64_t gfb = static_cast<int64_t>(N) * D;  // grad_feat: (B, N, D) fp32 rows
#define DVCP_BN_B(DD, A1, A2, A3)                                                                                   \
  if (D == DD && chans[1] == A1 && chans[2] == A2 && (nlayer == 2 ? 0 : chans[3]) == A3) {                         \
    if (f64)                                                                                                        \
      return ff64 ? dvcp::dispatch_bwd<double, double, DD, A1, A2, A3>(a, mode, grad_out, grad_feat, gfb,          \
                                                                        workspace, sums, grad_params)               \
                  : dvcp::dispatch_bwd<double, float, DD, A1, A2, A3>(a, mode, grad_out, grad_feat, gfb,           \
                                                                       workspace, sums, grad_params);               \
    return ff64 ? dvcp::dispatch_bwd<float, double, DD, A1, A2, A3>(a, mode, grad_out, grad_feat, gfb, workspace,   \
                                                                     sums, grad_params)                             \
                : dvcp::dispatch_bwd<float, float, DD, A1, A2, A3>(a, mode, grad_out, grad_feat, gfb, workspace,    \
                                                                    sums, grad_params);                             \
  }
  DVCP_BN_TABLES(DVCP_BN_B)
#undef DVCP_BN_B
  dvcp::set_error("dvcp_sa_bn_backward: unsupported table D=%d chans=%d,%d", D, chans[1], chans[2]);
  return DVCP_EINVAL;
}
