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
// with every A, B known writes each entry's gz_l and layer input (channel-major rows: dW_l, db_l
// are then plain GEMMs over the entries, done by the host) and scatters the feature gradient.
// The padding slots are evaluated as the copies of the first hit they are (never routed:
// torch.max takes the first of equal maxima).  The sums are per-wave fp64 partials summed in a
// fixed order (deterministic); the feature scatter uses float atomics.
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
};

// An opaque zero ordered after a value of the previous output channel's arithmetic: added to a
// weight-row offset, it keeps one row's scalar loads from being scheduled (or hoisted out of the
// centre loop) ahead of the previous row's use -- a layer's up-to-64 x 67 weights held at once
// spilled to VGPR lanes.  (The pointer keeps the kernel argument's provenance: loads stay scalar.)
__device__ __forceinline__ int bn_zero_after(float dep) {
  int z = 0;
  asm volatile("" : "+s"(z) : "v"(dep));
  return z;
}

// acc = W x (fp32, input channels in ascending order per output), one weight row at a time;
// epi(co, acc, q) finishes output co with q = p offset by the same opaque zero (its per-channel
// vector loads ordered likewise).
template <int CIN, int COUT, typename Epi>
__device__ __forceinline__ void bn_matvec(const float (&x)[CIN], const float* __restrict__ p, Epi epi) {
  float prev = 0.0f;
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    const float* q = p + bn_zero_after(prev);
    const float* w = q + co * CIN;
    float a = 0.0f;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) a = __fmaf_rn(w[ci], x[ci], a);
    epi(co, a, q);
    prev = a;
  }
}

// lane = slot: h = relu((W x + b) * scale + shift)
template <int CIN, int COUT>
__device__ __forceinline__ void bn_rows(const float (&x)[CIN], float (&h)[COUT], const float* __restrict__ p) {
  bn_matvec<CIN, COUT>(x, p, [&](int co, float acc, const float* q) {
    const float v = (acc + q[CIN * COUT + co]) * q[CIN * COUT + COUT + co] + q[CIN * COUT + 2 * COUT + co];
    h[co] = v > 0.0f ? v : 0.0f;
  });
}
// lane = slot: z = W x + b (the layer whose statistics are being taken)
template <int CIN, int COUT>
__device__ __forceinline__ void bn_rows_raw(const float (&x)[CIN], float (&z)[COUT], const float* __restrict__ p) {
  bn_matvec<CIN, COUT>(x, p, [&](int co, float acc, const float* q) { z[co] = acc + q[CIN * COUT + co]; });
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

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// Row layout of the z / gradient / input rows: 64-entry blocks, channel-major inside a block --
// element (entry e, channel c) of a C-channel table at (e / 64) * C * 64 + c * 64 + e % 64 -- so a
// wave's 64 consecutive entries of one channel are one 256-byte run and its whole chunk one
// contiguous C x 256-byte region (tables are padded to a multiple of 64 entries).
template <typename P>
__device__ __forceinline__ P* bn_at(P* base, int C, int64_t e) {
  return base + (e >> 6) * (static_cast<int64_t>(C) * 64) + (e & 63);
}

// The mode-0 gradient / input rows (the host's weight-gradient GEMM operands): 65536-entry
// chunks, channel-major inside a chunk -- (e / 65536) * C * 65536 + c * 65536 + e % 65536 -- so
// each chunk of a table is one (C x 65536) row-major GEMM operand (no layout copy on the host);
// tables are padded to a multiple of 65536 entries.
constexpr int kBnRowChunkLog = 16;
constexpr int64_t kBnRowChunk = int64_t(1) << kBnRowChunkLog;
__device__ __forceinline__ float* bn_at_rows(float* base, int C, int64_t e) {
  return base + (e >> kBnRowChunkLog) * (static_cast<int64_t>(C) * kBnRowChunk) + (e & (kBnRowChunk - 1));
}

// z = W x + b stored to its row (channel-major), h = relu(z * scale + shift), channel by channel
template <int CIN, int COUT>
__device__ __forceinline__ void bn_layer_store(const float (&x)[CIN], float (&h)[COUT], const float* __restrict__ p,
                                               float* __restrict__ zr, int64_t M, int64_t e) {
  bn_matvec<CIN, COUT>(x, p, [&](int co, float acc, const float* q) {
    const float z = acc + q[CIN * COUT + co];
    bn_at(zr, COUT, e)[co * 64] = z;
    const float y = z * q[CIN * COUT + COUT + co] + q[CIN * COUT + 2 * COUT + co];
    h[co] = y > 0.0f ? y : 0.0f;
  });
}

// ---- statistics pass ----------------------------------------------------------------------------
template <typename T, typename FT, int D, int C1, int C2, int C3, int LAYER>
__global__ __launch_bounds__(kBnThreads) void sa_bn_stats_kernel(PointsView<T> pts, PointsView<T> ctr, int S, int B,
                                                                 BnFeat<FT> feat, const int32_t* __restrict__ count,
                                                                 const int32_t* __restrict__ list, int nsample,
                                                                 const float* __restrict__ pack,
                                                                 double* __restrict__ partial,
                                                                 float* __restrict__ zrows) {
  using Tb = BnTable<D, C1, C2, C3>;
  constexpr int C0 = Tb::C0;
  constexpr int CZ = LAYER == 1 ? C1 : (LAYER == 2 ? C2 : C3);
  // the last layer's pass (every lower layer's batch statistics final) can also write every
  // entry's z rows for the backward (zrows != null): the z-row pass of dvcp_sa_bn_zrows, fused
  constexpr bool kLast = LAYER == (C3 > 0 ? 3 : 2);
  const int64_t Mz = (static_cast<int64_t>(B) * S * nsample + 63) & ~static_cast<int64_t>(63);
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
        const int64_t e = cs * nsample + r;
        bool done = false;
        if constexpr (kLast) {
          if (zrows) {
          done = true;
          float h1[C1];
          bn_layer_store<C0, C1>(x, h1, p1, zrows, Mz, e);
          if constexpr (C3 > 0) {
            float h2[C2];
            bn_layer_store<C1, C2>(h1, h2, p2, zrows + C1 * Mz, Mz, e);
            bn_rows_raw<C2, C3>(h2, z, p3);
          } else {
            bn_rows_raw<C1, C2>(h1, z, p2);
          }
          float* zl = zrows + (C3 > 0 ? (C1 + C2) : C1) * Mz;
#pragma unroll
          for (int k = 0; k < CZ; ++k) bn_at(zl, CZ, e)[k * 64] = z[k];
          }
        }
        if (done) {
        } else if constexpr (LAYER == 1) {
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

// ---- forward rows -------------------------------------------------------------------------------
// Every entry's conv outputs z_l of every layer (batch statistics final), channel-major
// (C_l x M per layer, e = centre * nsample + slot): the backward passes read them instead of
// recomputing the MLP.  lane = slot.
template <typename T, typename FT, int D, int C1, int C2, int C3>
__global__ __launch_bounds__(kBnThreads) void sa_bn_zrows_kernel(PointsView<T> pts, PointsView<T> ctr, int S, int B,
                                                                 BnFeat<FT> feat, const int32_t* __restrict__ count,
                                                                 const int32_t* __restrict__ list, int nsample,
                                                                 const float* __restrict__ pack,
                                                                 float* __restrict__ zrows) {
  using Tb = BnTable<D, C1, C2, C3>;
  constexpr int C0 = Tb::C0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* p1 = pack + Tb::O1;
  const float* p2 = pack + Tb::O2;
  const float* p3 = pack + Tb::O3;
  const int64_t M = (static_cast<int64_t>(B) * S * nsample + 63) & ~static_cast<int64_t>(63);  // padded
  float* z1r = zrows;
  float* z2r = z1r + C1 * M;
  float* z3r = z2r + C2 * M;
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
      if (r >= nsample) continue;
      const int64_t e = cs * nsample + r;
      float x[C0];
      bn_load_x<T, FT, D>(x, pts, feat, b, lst[r < cnt ? r : 0], cx, cy, cz);
      float h1[C1], h2[C2];
      bn_layer_store<C0, C1>(x, h1, p1, z1r, M, e);
      bn_layer_store<C1, C2>(h1, h2, p2, z2r, M, e);
      if constexpr (C3 > 0) {
        float h3[C3];
        bn_layer_store<C2, C3>(h2, h3, p3, z3r, M, e);
      }
    }
  }
}

// ---- backward (lane = grouped entry) ------------------------------------------------------------
// Per centre (one wave).  Pass 1 finds each last-layer channel's arg-max slot among the distinct
// hits from the z rows (first of equal maxima) and keeps that row's z; mode L takes A_L, B_L from
// those rows directly.  Otherwise pass 2 walks the centre's nsample slots in chunks of 64 (lane =
// slot; padding slots are the copies of the first hit they are, never routed) and runs the
// batch-norm backward top-down, channel by channel, streaming each layer's z rows (coalesced:
// consecutive lanes, consecutive entries) with the weights as wave-uniform scalar loads.  Mode k
// stops at layer k and sums gy_k and gy_k xhat_k through an LDS tile (fp64 column sums); mode 0
// writes each entry's gz_l and layer input h_{l-1} (plus a ones row, for the bias) as
// channel-major rows for the host's weight-gradient GEMMs, and scatters W_1^T gz_1 to the input
// features (float atomics).

template <int C>
__device__ __forceinline__ void bn_put(float* __restrict__ base, int64_t M, int64_t e, const float (&v)[C], bool ones) {
  float* o = bn_at_rows(base, ones ? C + 1 : C, e);
#pragma unroll
  for (int k = 0; k < C; ++k) o[k * kBnRowChunk] = v[k];
  if (ones) o[C * kBnRowChunk] = 1.0f;
}

template <int COUT>
struct BnVec {  // one layer's per-channel vectors (wave-uniform)
  const float* v;
  __device__ __forceinline__ float y(int c, float z) const { return z * v[COUT + c] + v[2 * COUT + c]; }
  __device__ __forceinline__ float xh(int c, float z) const { return (z - v[3 * COUT + c]) * v[4 * COUT + c]; }
  // gz = scale (gy - (A/M + xhat B/M))
  __device__ __forceinline__ float gz(int c, float z, float gy) const {
    return v[COUT + c] * (gy - (v[5 * COUT + c] + xh(c, z) * v[6 * COUT + c]));
  }
};

// The last layer: gy from the centre's route table (slot r; routable = a distinct hit), gz written
// (mode 0) and propagated: gprev = W^T gz.
template <int CIN, int COUT, bool FINAL>
__device__ __forceinline__ void bn_bwd_top(const float* __restrict__ zr, int64_t M, int64_t e, bool act,
                                           const float* __restrict__ p, const float* sv, const int* sarg, const float* srg, int r,
                                           bool routable, float (&gprev)[CIN], float* __restrict__ gzr) {
  const BnVec<COUT> q{sv};
#pragma unroll
  for (int k = 0; k < CIN; ++k) gprev[k] = 0.0f;
#pragma unroll 1
  for (int c = 0; c < COUT; ++c) {
    const float z = act ? bn_at(zr, COUT, e)[c * 64] : 0.0f;
    const float gy = (routable && sarg[c] == r && q.y(c, z) > 0.0f) ? srg[c] : 0.0f;
    const float gz = q.gz(c, z, gy);
    if constexpr (FINAL) {
      if (act) bn_at_rows(gzr, COUT, e)[c * kBnRowChunk] = gz;
    }
#pragma unroll
    for (int k = 0; k < CIN; ++k) gprev[k] = __fmaf_rn(p[c * CIN + k], gz, gprev[k]);
  }
}

// A lower layer: g = dL/dh on entry, gy = [y > 0] g, gz written (mode 0), gprev = W^T gz.
template <int CIN, int COUT, bool FINAL>
__device__ __forceinline__ void bn_bwd_mid(const float* __restrict__ zr, int64_t M, int64_t e, bool act,
                                           const float* __restrict__ p, const float* sv, const float (&g)[COUT], float (&gprev)[CIN],
                                           float* __restrict__ gzr) {
  const BnVec<COUT> q{sv};
#pragma unroll
  for (int k = 0; k < CIN; ++k) gprev[k] = 0.0f;
#pragma unroll 1
  for (int c = 0; c < COUT; ++c) {
    const float z = act ? bn_at(zr, COUT, e)[c * 64] : 0.0f;
    const float gz = q.gz(c, z, q.y(c, z) > 0.0f ? g[c] : 0.0f);
    if constexpr (FINAL) {
      if (act) bn_at_rows(gzr, COUT, e)[c * kBnRowChunk] = gz;
    }
#pragma unroll
    for (int k = 0; k < CIN; ++k) gprev[k] = __fmaf_rn(p[c * CIN + k], gz, gprev[k]);
  }
}

// Mode 0: the input rows of layer l+1, h_l = relu(y_l), and a ones row.
template <int CIN, int COUT>
__device__ __forceinline__ void bn_put_h(const float* __restrict__ zr, int64_t M, int64_t e, const float* sv,
                                         float* __restrict__ har) {
  const BnVec<COUT> q{sv};
#pragma unroll
  for (int c = 0; c < COUT; ++c) {
    const float y = q.y(c, bn_at(zr, COUT, e)[c * 64]);
    bn_at_rows(har, COUT + 1, e)[c * kBnRowChunk] = y > 0.0f ? y : 0.0f;
  }
  bn_at_rows(har, COUT + 1, e)[COUT * kBnRowChunk] = 1.0f;
}

// The sums of one layer over the chunk: A += sum gy, B += sum gy xhat (gy = [y > 0] g), through
// the wave's LDS tile (two phases, z re-read); lanes = (channel lane % COUT, slot group lane / COUT).
template <int CIN, int COUT, int TW>
__device__ __forceinline__ void bn_bwd_sums(const float* __restrict__ zr, int64_t M, int64_t e, bool act,
                                            const float* sv, const float (&g)[COUT], float (*tl)[TW + 1],
                                            int lane, int rn, double& s1, double& s2) {
  constexpr int G = kWave / COUT;
  const BnVec<COUT> q{sv};
  const int c = lane % COUT, grp = lane / COUT;
#pragma unroll
  for (int k = 0; k < COUT; ++k) {
    const float z = act ? bn_at(zr, COUT, e)[k * 64] : 0.0f;
    tl[lane][k] = (act && q.y(k, z) > 0.0f) ? g[k] : 0.0f;
  }
  wave_sync_lds();
  for (int j = grp; j < rn; j += G) s1 += static_cast<double>(tl[j][c]);
  wave_sync_lds();
#pragma unroll
  for (int k = 0; k < COUT; ++k) {
    const float z = act ? bn_at(zr, COUT, e)[k * 64] : 0.0f;
    tl[lane][k] = (act && q.y(k, z) > 0.0f) ? g[k] * q.xh(k, z) : 0.0f;
  }
  wave_sync_lds();
  for (int j = grp; j < rn; j += G) s2 += static_cast<double>(tl[j][c]);
  wave_sync_lds();
}

// Layer 1 in mode 0: gz_1 written (g becomes gz_1).
template <int CIN, int COUT>
__device__ __forceinline__ void bn_bwd_first(const float* __restrict__ zr, int64_t e, bool act,
                                             const float* sv, float (&g)[COUT], float* __restrict__ gzr) {
  const BnVec<COUT> q{sv};
#pragma unroll
  for (int c = 0; c < COUT; ++c) {
    const float z = act ? bn_at(zr, COUT, e)[c * 64] : 0.0f;
    g[c] = q.gz(c, z, q.y(c, z) > 0.0f ? g[c] : 0.0f);
    if (act) bn_at_rows(gzr, COUT, e)[c * kBnRowChunk] = g[c];
  }
}

// The feature gradient of the chunk, W_1^T gz_1 (input columns 3..), scattered to the points:
// the chunk's gz_1 rows go through the LDS tile, then row by row lane d < D adds its channel
// (one coalesced atomic per row instead of D scattered ones per lane).
template <int D, int C0, int C1, int TW>
__device__ __forceinline__ void bn_scatter_feat(const float (&g)[C1], float (*tl)[TW + 1], const float* __restrict__ p1,
                                                int lane, int rn, int n, bool act, float* __restrict__ gfb) {
#pragma unroll
  for (int k = 0; k < C1; ++k) tl[lane][k] = act ? g[k] : 0.0f;
  wave_sync_lds();
  const int d = lane < D ? lane : 0;
  float w[C1];
#pragma unroll
  for (int c = 0; c < C1; ++c) w[c] = p1[c * C0 + 3 + d];
  for (int j = 0; j < rn; ++j) {
    const int nj = __builtin_amdgcn_readlane(n, j);
    float acc = 0.0f;
#pragma unroll
    for (int c = 0; c < C1; ++c) acc = __fmaf_rn(w[c], tl[j][c], acc);
    if (lane < D && acc != 0.0f) atomicAdd(gfb + static_cast<int64_t>(nj) * D + lane, acc);
  }
  wave_sync_lds();
}

// D = 32 / 64 (C1 = D): the entry's dL/dz_1 row, row-major (C1 floats), for the feature gradient
//   dL/df_n = W_1f^T sum_{e: n(e) = n} gz_1[e]
// -- segment_sum adds each point's rows in entry order (deterministic, no float atomics), then
// bn_feat_grad_kernel applies W_1f^T once per point instead of once per grouped entry.
template <int C>
__device__ __forceinline__ void bn_put_rowmajor(float* __restrict__ o, const float (&g)[C]) {
#pragma unroll
  for (int k = 0; k < C; k += 4) *reinterpret_cast<float4*>(o + k) = make_float4(g[k], g[k + 1], g[k + 2], g[k + 3]);
}

// gfeat[b][n][d] = sum_c G[b * N + n][c] W_1[c][3 + d] (fp32, c ascending): one thread per (point, d).
template <int D, int C0, int C1>
__global__ __launch_bounds__(256) void bn_feat_grad_kernel(const float* __restrict__ G, const float* __restrict__ p1,
                                                           int64_t rows, float* __restrict__ gfeat) {
  __shared__ float w[C1][D];
  for (int i = threadIdx.x; i < C1 * D; i += 256) w[i / D][i % D] = p1[(i / D) * C0 + 3 + i % D];
  __syncthreads();
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= rows * D) return;
  const int64_t r = t / D;
  const int d = static_cast<int>(t % D);
  const float* g = G + r * C1;
  float acc = 0.0f;
#pragma unroll 8
  for (int c = 0; c < C1; ++c) acc = __fmaf_rn(g[c], w[c][d], acc);
  gfeat[t] = acc;
}

// MODE: 0 = per-entry gradient rows + feature gradient; k in 1..L = the sums A_k, B_k.
template <typename T, typename FT, int D, int C1, int C2, int C3, int MODE>
__global__ __launch_bounds__(kBnThreads) __attribute__((amdgpu_waves_per_eu(2))) void sa_bn_bwd_kernel(
    PointsView<T> pts, PointsView<T> ctr, int S, int B, BnFeat<FT> feat, const int32_t* __restrict__ count,
    const int32_t* __restrict__ list, int nsample, const float* __restrict__ pack, const float* __restrict__ zrows,
    const float* __restrict__ gout, float* __restrict__ gfeat, int64_t gfb, double* __restrict__ dpartial,
    float* __restrict__ rows, float* __restrict__ frows, uint32_t* __restrict__ fkeys, int nfeat) {
  using Tb = BnTable<D, C1, C2, C3>;
  constexpr int C0 = Tb::C0, CL = Tb::CL, L = Tb::L;
  constexpr bool FINAL = MODE == 0;
  constexpr int CM = MODE == 1 ? C1 : (MODE == 2 ? C2 : (MODE == 3 ? C3 : 1));
  constexpr int TW = CL > CM ? (CL > C1 ? CL : C1) : (CM > C1 ? CM : C1);
  constexpr int CINL = C3 > 0 ? C2 : C1;
  __shared__ float tile[kBnWaves][kWave][TW + 1];
  __shared__ int s_arg[kBnWaves][CL];
  __shared__ float s_rg[kBnWaves][CL];
  __shared__ double red[kBnWaves][2][kWave];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* p1 = pack + Tb::O1;
  const float* p2 = pack + Tb::O2;
  const float* p3 = pack + Tb::O3;
  const float* pL = C3 > 0 ? p3 : p2;
  const float* vL = pL + CL * CINL;
  // the layers' per-channel vectors (bias | scale | shift | mean | istd | A/M | B/M) in LDS: read
  // as wave-uniform LDS loads, not hoisted into (spilled) SGPRs
  __shared__ float svec[7 * (C1 + C2 + (C3 > 0 ? C3 : 1))];
  float* sv1 = svec;
  float* sv2 = sv1 + 7 * C1;
  float* sv3 = sv2 + 7 * C2;
  for (int i = tid; i < 7 * C1; i += kBnThreads) sv1[i] = p1[C1 * C0 + i];
  for (int i = tid; i < 7 * C2; i += kBnThreads) sv2[i] = p2[C2 * C1 + i];
  if constexpr (C3 > 0)
    for (int i = tid; i < 7 * C3; i += kBnThreads) sv3[i] = p3[C3 * C2 + i];
  __syncthreads();
  const int cL = lane < CL ? lane : 0;
  const float scL = vL[CL + cL], shL = vL[2 * CL + cL], muL = vL[3 * CL + cL], isL = vL[4 * CL + cL];
  const int64_t M = (static_cast<int64_t>(B) * S * nsample + 63) & ~static_cast<int64_t>(63);  // padded
  const float* z1r = zrows;
  const float* z2r = z1r + C1 * M;
  const float* z3r = z2r + C2 * M;
  const float* zLr = C3 > 0 ? z3r : z2r;
  // mode 0 rows, per layer l: gz_l (C_l x M) | its input h_{l-1} and a ones row (C_{l-1} + 1 x M)
  float *gz1r = nullptr, *ha1r = nullptr, *gz2r = nullptr, *ha2r = nullptr, *gz3r = nullptr, *ha3r = nullptr;
  if constexpr (FINAL) {
    const int64_t Mk = (M + kBnRowChunk - 1) / kBnRowChunk * kBnRowChunk;
    gz1r = rows;
    ha1r = gz1r + C1 * Mk;
    gz2r = ha1r + (C0 + 1) * Mk;
    ha2r = gz2r + C2 * Mk;
    gz3r = ha2r + (C1 + 1) * Mk;
    ha3r = gz3r + C3 * Mk;
  }
  double s1 = 0.0, s2 = 0.0;
  float(*tl)[TW + 1] = tile[wave];
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

    // ---- pass 1: each channel's arg-max slot among the distinct hits, and its z ------------------
    float best = -1.0f, zbest = 0.0f;  // outputs are >= 0
    int arg = 0;
    for (int r0 = 0; r0 < cnt; r0 += kWave) {
      const int r = r0 + lane;
      if (r < cnt) {
#pragma unroll
        for (int k = 0; k < CL; ++k) tl[lane][k] = bn_at(zLr, CL, cs * nsample + r)[k * 64];
      }
      wave_sync_lds();
      if (lane < CL) {
        const int rn = min(kWave, cnt - r0);
        for (int j = 0; j < rn; ++j) {
          const float z = tl[j][lane];
          const float y = z * scL + shL;
          const float h = y > 0.0f ? y : 0.0f;
          if (h > best) {  // strict: the first row among equal maxima
            best = h;
            zbest = z;
            arg = r0 + j;
          }
        }
      }
      wave_sync_lds();
    }
    const bool routed = lane < CL && best > 0.0f && g_c != 0.0f;
    if constexpr (MODE == L) {
      if (routed) {
        s1 += static_cast<double>(g_c);
        s2 += static_cast<double>(g_c) * static_cast<double>((zbest - muL) * isL);
      }
      continue;
    }
    if (lane < CL) {
      s_arg[wave][lane] = routed ? arg : -1;
      s_rg[wave][lane] = g_c;
    }
    wave_sync_lds();

    // ---- pass 2: every slot (lane = slot) --------------------------------------------------------
    const T cx = ctr.at(b, 0, s), cy = ctr.at(b, 1, s), cz = ctr.at(b, 2, s);
    for (int r0 = 0; r0 < nsample; r0 += kWave) {
      const int r = r0 + lane;
      const bool act = r < nsample;
      const int rn = min(kWave, nsample - r0);
      const int64_t e = cs * nsample + (act ? r : 0);
      const int n = lst[(act && r < cnt) ? r : 0];
      if constexpr (FINAL) {
        if (act) {
          float x[C0];
          bn_load_x<T, FT, D>(x, pts, feat, b, n, cx, cy, cz);
          bn_put<C0>(ha1r, M, e, x, true);
        }
      }
      if constexpr (C3 > 0) {
        float g2[C2], g1[C1];
        bn_bwd_top<C2, C3, FINAL>(z3r, M, e, act, p3, sv3, s_arg[wave], s_rg[wave], r, r < cnt, g2, gz3r);
        if constexpr (MODE == 2) {
          bn_bwd_sums<C1, C2, TW>(z2r, M, e, act, sv2, g2, tl, lane, rn, s1, s2);
          continue;
        }
        if constexpr (FINAL) {
          if (act) bn_put_h<C1, C2>(z2r, M, e, sv2, ha3r);
        }
        bn_bwd_mid<C1, C2, FINAL>(z2r, M, e, act, p2, sv2, g2, g1, gz2r);
        if constexpr (MODE == 1) {
          bn_bwd_sums<C0, C1, TW>(z1r, M, e, act, sv1, g1, tl, lane, rn, s1, s2);
          continue;
        }
        if constexpr (FINAL) {
          if (act) bn_put_h<C0, C1>(z1r, M, e, sv1, ha2r);
          bn_bwd_first<C0, C1>(z1r, e, act, sv1, g1, gz1r);
          if constexpr (D == 32 || D == 64) {
            if (frows) {
              if (act) fkeys[e] = static_cast<uint32_t>(static_cast<int64_t>(b) * nfeat + n);
              if (act) bn_put_rowmajor<C1>(frows + e * C1, g1);
            }
          } else if constexpr (D > 0) {
            if (gfeat) bn_scatter_feat<D, C0, C1, TW>(g1, tl, p1, lane, rn, n, act, gfeat + b * gfb);
          }
        }
      } else {
        float g1[C1];
        bn_bwd_top<C1, C2, FINAL>(z2r, M, e, act, p2, sv2, s_arg[wave], s_rg[wave], r, r < cnt, g1, gz2r);
        if constexpr (MODE == 1) {
          bn_bwd_sums<C0, C1, TW>(z1r, M, e, act, sv1, g1, tl, lane, rn, s1, s2);
          continue;
        }
        if constexpr (FINAL) {
          if (act) bn_put_h<C0, C1>(z1r, M, e, sv1, ha2r);
          bn_bwd_first<C0, C1>(z1r, e, act, sv1, g1, gz1r);
          if constexpr (D == 32 || D == 64) {
            if (frows) {
              if (act) fkeys[e] = static_cast<uint32_t>(static_cast<int64_t>(b) * nfeat + n);
              if (act) bn_put_rowmajor<C1>(frows + e * C1, g1);
            }
          } else if constexpr (D > 0) {
            if (gfeat) bn_scatter_feat<D, C0, C1, TW>(g1, tl, p1, lane, rn, n, act, gfeat + b * gfb);
          }
        }
      }
    }
    wave_sync_lds();  // s_arg / s_rg are rewritten by the next centre
  }
  if constexpr (!FINAL) {
    // this wave's per-channel sums, the slot groups combined in a fixed order
    constexpr int G = kWave / CM;
    red[wave][0][lane] = s1;
    red[wave][1][lane] = s2;
    wave_sync_lds();
    if (lane < CM) {
      double a = 0.0, q = 0.0;
      for (int g = 0; g < G; ++g) {
        a += red[wave][0][g * CM + lane];
        q += red[wave][1][g * CM + lane];
      }
      double* o = dpartial + (static_cast<int64_t>(blockIdx.x) * kBnWaves + wave) * (2 * CM);
      o[lane] = a;
      o[CM + lane] = q;
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

// segsum.hip
int64_t segment_sum_workspace_bytes(int64_t E, int64_t nrows);
int segment_sum(const uint32_t* keys, const float* contrib, int64_t E, int64_t nrows, int ncol, float* out, void* ws,
                hipStream_t st);

// Mode-0 feature-gradient workspace: keys (E u32) | rows (E x D fp32) | segment_sum's own.
inline int64_t bn_align(int64_t x) { return (x + 255) / 256 * 256; }
static void bn_feat_ws_layout(void* ws, int64_t E, int64_t npts, int C, uint32_t** keys, float** rows, float** G,
                              void** seg) {
  char* p = static_cast<char*>(ws);
  *keys = reinterpret_cast<uint32_t*>(p);
  *rows = reinterpret_cast<float*>(p + bn_align(E * 4));
  *G = reinterpret_cast<float*>(p + bn_align(E * 4) + bn_align(E * C * 4));
  *seg = p + bn_align(E * 4) + bn_align(E * C * 4) + bn_align(npts * C * 4);
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
static int launch_stats(const BnArgs& a, void* ws, double* sums, float* zrows) {
  constexpr int CZ = LAYER == 1 ? C1 : (LAYER == 2 ? C2 : C3);
  const int grid = bn_grid(static_cast<int64_t>(a.B) * a.S);
  PointsView<T> pv{static_cast<const T*>(a.xyz), a.sb, a.sc, a.sn};
  PointsView<T> cv{static_cast<const T*>(a.ctr), a.cb, a.cc, a.cn};
  BnFeat<FT> fv{static_cast<const FT*>(a.feat), a.fb, a.fd, a.fn};
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL((sa_bn_stats_kernel<T, FT, D, C1, C2, C3, LAYER>), dim3(grid), dim3(kBnThreads), 0, a.st, pv,
                     cv, a.S, a.B, fv, a.count, a.list, a.nsample, a.pack, part, zrows);
  if (int e = launch_status("dvcp_sa_bn_stats")) return e;
  hipLaunchKernelGGL((bn_sum_kernel<double, double>), dim3(ceil_div(2 * CZ, 64)), dim3(1024), 0, a.st, part,
                     grid * kBnWaves, 2 * CZ, sums);
  return launch_status("dvcp_sa_bn_stats(sum)");
}

template <typename T, typename FT, int D, int C1, int C2, int C3, int MODE>
static int launch_bwd(const BnArgs& a, const float* zrows, const float* gout, float* gfeat, int64_t gfb, void* ws,
                      double* sums, float* rows) {
  const int grid = bn_grid(static_cast<int64_t>(a.B) * a.S);
  PointsView<T> pv{static_cast<const T*>(a.xyz), a.sb, a.sc, a.sn};
  PointsView<T> cv{static_cast<const T*>(a.ctr), a.cb, a.cc, a.cn};
  BnFeat<FT> fv{static_cast<const FT*>(a.feat), a.fb, a.fd, a.fn};
  // mode 0, D = C1 = 32 / 64 with a feature gradient: per-entry gz_1 rows + keys in the workspace,
  // the deterministic per-point segment sums, then W_1f^T per point (bn_feat_ws_layout)
  constexpr bool kSeg = MODE == 0 && (D == 32 || D == 64) && C1 == D;
  const int nfeat = D > 0 ? static_cast<int>(gfb / D) : 0;
  const int64_t E = static_cast<int64_t>(a.B) * a.S * a.nsample;
  uint32_t* fkeys = nullptr;
  float* frows = nullptr;
  void* segws = nullptr;
  float* G = nullptr;
  const int64_t npts = static_cast<int64_t>(a.B) * nfeat;
  if (kSeg && gfeat) bn_feat_ws_layout(ws, E, npts, C1, &fkeys, &frows, &G, &segws);
  hipLaunchKernelGGL((sa_bn_bwd_kernel<T, FT, D, C1, C2, C3, MODE>), dim3(grid), dim3(kBnThreads), 0, a.st, pv, cv,
                     a.S, a.B, fv, a.count, a.list, a.nsample, a.pack, zrows, gout, gfeat, gfb,
                     static_cast<double*>(ws), rows, frows, fkeys, nfeat);
  if (int e = launch_status("dvcp_sa_bn_backward")) return e;
  if constexpr (kSeg) {
    if (gfeat) {
      if (int e = segment_sum(fkeys, frows, E, npts, C1, G, segws, a.st)) return e;
      hipLaunchKernelGGL((bn_feat_grad_kernel<D, 3 + D, C1>), dim3(ceil_div(npts * D, 256)), dim3(256), 0, a.st, G,
                         a.pack, npts, gfeat);
      return launch_status("dvcp_sa_bn_backward(feat)");
    }
  }
  if constexpr (MODE != 0) {
    constexpr int CM = MODE == 1 ? C1 : (MODE == 2 ? C2 : C3);
    hipLaunchKernelGGL((bn_sum_kernel<double, double>), dim3(ceil_div(2 * CM, 64)), dim3(1024), 0, a.st,
                       static_cast<const double*>(ws), grid * kBnWaves, 2 * CM, sums);
    return launch_status("dvcp_sa_bn_backward(sum)");
  }
  return DVCP_OK;
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
static int dispatch_stats(const BnArgs& a, int layer, void* ws, double* sums, float* zrows) {
  if (layer == 1) return launch_stats<T, FT, D, C1, C2, C3, 1>(a, ws, sums, zrows);
  if (layer == 2) return launch_stats<T, FT, D, C1, C2, C3, 2>(a, ws, sums, zrows);
  if constexpr (C3 > 0)
    if (layer == 3) return launch_stats<T, FT, D, C1, C2, C3, 3>(a, ws, sums, zrows);
  set_error("dvcp_sa_bn_stats: layer %d out of range", layer);
  return DVCP_EINVAL;
}

template <typename T, typename FT, int D, int C1, int C2, int C3>
static int dispatch_bwd(const BnArgs& a, int mode, const float* zrows, const float* gout, float* gfeat, int64_t gfb,
                        void* ws, double* sums, float* rows) {
  if (mode == -1) {  // the z rows (forward)
    const int grid = bn_grid(static_cast<int64_t>(a.B) * a.S);
    PointsView<T> pv{static_cast<const T*>(a.xyz), a.sb, a.sc, a.sn};
    PointsView<T> cv{static_cast<const T*>(a.ctr), a.cb, a.cc, a.cn};
    BnFeat<FT> fv{static_cast<const FT*>(a.feat), a.fb, a.fd, a.fn};
    hipLaunchKernelGGL((sa_bn_zrows_kernel<T, FT, D, C1, C2, C3>), dim3(grid), dim3(kBnThreads), 0, a.st, pv, cv, a.S,
                       a.B, fv, a.count, a.list, a.nsample, a.pack, rows);
    return launch_status("dvcp_sa_bn_zrows");
  }
  if (mode == 0) return launch_bwd<T, FT, D, C1, C2, C3, 0>(a, zrows, gout, gfeat, gfb, ws, sums, rows);
  if (mode == 1) return launch_bwd<T, FT, D, C1, C2, C3, 1>(a, zrows, gout, gfeat, gfb, ws, sums, rows);
  if (mode == 2) return launch_bwd<T, FT, D, C1, C2, C3, 2>(a, zrows, gout, gfeat, gfb, ws, sums, rows);
  if constexpr (C3 > 0)
    if (mode == 3) return launch_bwd<T, FT, D, C1, C2, C3, 3>(a, zrows, gout, gfeat, gfb, ws, sums, rows);
  set_error("dvcp_sa_bn_backward: mode %d out of range", mode);
  return DVCP_EINVAL;
}

// Feature dtypes: fp64 only for the 3-channel normals table (ModelNet's double clouds); the
// 32 / 64-channel tables read the previous layer's fp32 outputs.
template <typename T, int DD, int A1, int A2, int A3>
static int stats_ft(const BnArgs& a, bool ff64, int layer, void* ws, double* sums, float* zrows) {
  if constexpr (DD == 3) {
    if (ff64) return dispatch_stats<T, double, DD, A1, A2, A3>(a, layer, ws, sums, zrows);
  } else if (DD > 0 && ff64) {
    set_error("dvcp_sa_bn_stats: fp64 features are taken for the 3-channel table only (D=%d)", DD);
    return DVCP_EINVAL;
  }
  return dispatch_stats<T, float, DD, A1, A2, A3>(a, layer, ws, sums, zrows);
}

template <typename T, int DD, int A1, int A2, int A3>
static int bwd_ft(const BnArgs& a, bool ff64, int mode, const float* zrows, const float* gout, float* gfeat,
                  int64_t gfb, void* ws, double* sums, float* rows) {
  if constexpr (DD == 3) {
    if (ff64) return dispatch_bwd<T, double, DD, A1, A2, A3>(a, mode, zrows, gout, gfeat, gfb, ws, sums, rows);
  } else if (DD > 0 && ff64) {
    set_error("dvcp_sa_bn_backward: fp64 features are taken for the 3-channel table only (D=%d)", DD);
    return DVCP_EINVAL;
  }
  return dispatch_bwd<T, float, DD, A1, A2, A3>(a, mode, zrows, gout, gfeat, gfb, ws, sums, rows);
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
  int64_t cmax = 0;
  for (int l = 0; l < nlayer; ++l) cmax = std::max<int64_t>(cmax, chans[l + 1]);
  const int64_t nw = static_cast<int64_t>(dvcp::bn_grid(static_cast<int64_t>(B) * S)) * dvcp::kBnWaves;
  return nw * 2 * cmax * 8;
}

extern "C" int64_t dvcp_sa_bn_feat_workspace_bytes(int B, int S, int nsample, int N, int D) {
  if (B < 0 || S < 0 || nsample < 0 || N < 0 || D < 0) return -1;
  if (D != 32 && D != 64) return 0;  // other tables scatter with atomics (no workspace)
  const int64_t E = static_cast<int64_t>(B) * S * nsample, npts = static_cast<int64_t>(B) * N;
  const int64_t seg = dvcp::segment_sum_workspace_bytes(E, npts);  // (C1 = D for these tables)
  return seg < 0 ? -1 : dvcp::bn_align(E * 4) + dvcp::bn_align(E * D * 4) + dvcp::bn_align(npts * D * 4) + seg;
}

extern "C" int64_t dvcp_sa_bn_rows_floats(int B, int S, int nsample, int nlayer, const int* chans) {
  if (B < 0 || S < 0 || nsample < 0 || !chans || (nlayer != 2 && nlayer != 3)) return -1;
  int64_t per = 0;
  for (int l = 0; l < nlayer; ++l) per += chans[l + 1] + chans[l] + 1;
  const int64_t K = dvcp::kBnRowChunk;
  return per * ((static_cast<int64_t>(B) * S * nsample + K - 1) / K * K);
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
                                void* workspace, double* sums, float* zrows, void* stream) {
  if (int e = bn_check("dvcp_sa_bn_stats", dtype, xyz, ctr, N, S, B, feat_dtype, feat, D, count, list, nsample, nlayer,
                       chans, pack, workspace))
    return e;
  DVCP_REQUIRE(sums, "dvcp_sa_bn_stats: null sums");
  DVCP_REQUIRE(layer >= 1 && layer <= nlayer, "dvcp_sa_bn_stats: layer %d of %d", layer, nlayer);
  DVCP_REQUIRE(!zrows || layer == nlayer, "dvcp_sa_bn_stats: z rows are written by the last layer's pass only");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0 || S == 0) {
    if (hipMemsetAsync(sums, 0, 2 * chans[layer] * sizeof(double), st) != hipSuccess)
      return dvcp::launch_status("dvcp_sa_bn_stats(empty)");
    return DVCP_OK;
  }
  const dvcp::BnArgs a{xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, fd, fn, count, list, nsample, pack, st};
  const bool f64 = dtype == DVCP_F64, ff64 = feat_dtype == DVCP_F64;
#define DVCP_BN_S(DD, A1, A2, A3)                                                                           \
  if (D == DD && chans[1] == A1 && chans[2] == A2 && (nlayer == 2 ? 0 : chans[3]) == A3)                   \
    return f64 ? dvcp::stats_ft<double, DD, A1, A2, A3>(a, ff64, layer, workspace, sums, zrows)             \
               : dvcp::stats_ft<float, DD, A1, A2, A3>(a, ff64, layer, workspace, sums, zrows);
  DVCP_BN_TABLES(DVCP_BN_S)
#undef DVCP_BN_S
  dvcp::set_error("dvcp_sa_bn_stats: unsupported table D=%d chans=%d,%d", D, chans[1], chans[2]);
  return DVCP_EINVAL;
}

extern "C" int dvcp_sa_bn_backward(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N,
                                   const void* ctr, int64_t cb, int64_t cc, int64_t cn, int S, int B, int feat_dtype,
                                   const void* feat, int64_t fb, int64_t fd, int64_t fn, int D, const int32_t* count,
                                   const int32_t* list, int nsample, int nlayer, const int* chans, const float* pack,
                                   const float* zrows, int mode, const float* grad_out, float* grad_feat,
                                   void* workspace, double* sums, float* rows, void* stream) {
  if (int e = bn_check("dvcp_sa_bn_backward", dtype, xyz, ctr, N, S, B, feat_dtype, feat, D, count, list, nsample,
                       nlayer, chans, pack, workspace))
    return e;
  DVCP_REQUIRE(grad_out && zrows, "dvcp_sa_bn_backward: null grad_out / zrows");
  DVCP_REQUIRE(mode >= 0 && mode <= nlayer, "dvcp_sa_bn_backward: mode %d of %d", mode, nlayer);
  DVCP_REQUIRE(mode == 0 ? rows != nullptr : sums != nullptr, "dvcp_sa_bn_backward: null output");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0 || S == 0) {
    if (mode != 0 && hipMemsetAsync(sums, 0, 2 * chans[mode] * sizeof(double), st) != hipSuccess)
      return dvcp::launch_status("dvcp_sa_bn_backward(empty)");
    return DVCP_OK;
  }
  const dvcp::BnArgs a{xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, fd, fn, count, list, nsample, pack, st};
  const bool f64 = dtype == DVCP_F64, ff64 = feat_dtype == DVCP_F64;
  const int64_t gfb = static_cast<int64_t>(N) * D;  // grad_feat: (B, N, D) fp32 rows
#define DVCP_BN_B(DD, A1, A2, A3)                                                                           \
  if (D == DD && chans[1] == A1 && chans[2] == A2 && (nlayer == 2 ? 0 : chans[3]) == A3)                   \
    return f64 ? dvcp::bwd_ft<double, DD, A1, A2, A3>(a, ff64, mode, zrows, grad_out, grad_feat, gfb,       \
                                                       workspace, sums, rows)                               \
               : dvcp::bwd_ft<float, DD, A1, A2, A3>(a, ff64, mode, zrows, grad_out, grad_feat, gfb,        \
                                                      workspace, sums, rows);
  DVCP_BN_TABLES(DVCP_BN_B)
#undef DVCP_BN_B
  dvcp::set_error("dvcp_sa_bn_backward: unsupported table D=%d chans=%d,%d", D, chans[1], chans[2]);
  return DVCP_EINVAL;
}

extern "C" int64_t dvcp_sa_bn_zrows_floats(int B, int S, int nsample, int nlayer, const int* chans) {
  if (B < 0 || S < 0 || nsample < 0 || !chans || (nlayer != 2 && nlayer != 3)) return -1;
  int64_t per = 0;
  for (int l = 0; l < nlayer; ++l) per += chans[l + 1];
  return per * ((static_cast<int64_t>(B) * S * nsample + 63) / 64 * 64);
}

extern "C" int dvcp_sa_bn_zrows(int dtype, const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const void* ctr,
                                int64_t cb, int64_t cc, int64_t cn, int S, int B, int feat_dtype, const void* feat,
                                int64_t fb, int64_t fd, int64_t fn, int D, const int32_t* count, const int32_t* list,
                                int nsample, int nlayer, const int* chans, const float* pack, float* zrows,
                                void* stream) {
  const int dummy_ws = 0;
  if (int e = bn_check("dvcp_sa_bn_zrows", dtype, xyz, ctr, N, S, B, feat_dtype, feat, D, count, list, nsample, nlayer,
                       chans, pack, &dummy_ws))
    return e;
  DVCP_REQUIRE(zrows, "dvcp_sa_bn_zrows: null zrows");
  if (B == 0 || S == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dvcp::BnArgs a{xyz, sb, sc, sn, ctr, cb, cc, cn, S, B, feat, fb, fd, fn, count, list, nsample, pack, st};
  const bool f64 = dtype == DVCP_F64, ff64 = feat_dtype == DVCP_F64;
#define DVCP_BN_Z(DD, A1, A2, A3)                                                                           \
  if (D == DD && chans[1] == A1 && chans[2] == A2 && (nlayer == 2 ? 0 : chans[3]) == A3)                   \
    return f64 ? dvcp::bwd_ft<double, DD, A1, A2, A3>(a, ff64, -1, nullptr, nullptr, nullptr, 0, nullptr,  \
                                                       nullptr, zrows)                                      \
               : dvcp::bwd_ft<float, DD, A1, A2, A3>(a, ff64, -1, nullptr, nullptr, nullptr, 0, nullptr,   \
                                                      nullptr, zrows);
  DVCP_BN_TABLES(DVCP_BN_Z)
#undef DVCP_BN_Z
  dvcp::set_error("dvcp_sa_bn_zrows: unsupported table D=%d chans=%d,%d", D, chans[1], chans[2]);
  return DVCP_EINVAL;
}
