// sa_bn_mfma.hip -- batch-statistics BatchNorm training of the REF-R set-abstraction tables
// (sa1 3[+3]-16-16-32, sa2 35-32-64, sa3 67-64-64; pointnet2_utils.py:195-200 with the module in
// train(), driven by train.py:105-125) on the matrix cores (sa1: sa_bnm3_kernel, passes 1-3 / 10 /
// 21 / 22 / 30; sa2 / sa3: sa_bnm_kernel).  The lane-per-entry VALU passes of sa_bn.hip remain only
// for fp64 inputs and channel-first two-layer feature tables (and as batchnorm.USE_MFMA = False).
//
// Per grouped entry e = (centre, slot), x = [p - c, f_n]:
//   z1 = W1 x + b1, h1 = relu(z1 s1 + t1), z2 = W2 h1 + b2, h2 = relu(z2 s2 + t2), out = max_slot h2
// with s_l = gamma_l istd_l, t_l = beta_l - mu_l s_l from the batch statistics over all
// M = B S nsample entries (padding slots repeat the first hit and count in every sum).
// Backward (torch's batch-norm backward; a_l = A_l / M, b_l = B_l / M):
//   gz_l = s_l gy_l - s_l b_l istd_l (z_l - mu_l) - s_l a_l,  gh1 = W2^T gz2,  gy1 = [y1 > 0] gh1,
//   dW2 = sum_e gz2 h1^T, dW1 = sum_e gz1 x^T, db_l = sum_e gz_l, dL/df_n = W1f^T sum_{e -> n} gz1
//
// Nothing per entry is stored: every pass recomputes the MLP (a 32-entry tile of a centre is a
// few dozen MFMAs), so the passes stream only the ball-query lists, the points and a per-point
// table U[n] = W1f f_n + b1 (the feature half of layer 1, once per call).  One wave per centre;
// its distinct hits go through in 32-entry tiles; the nsample - count padding slots, which equal
// the first hit except that they are never routed by the max, are one extra "ghost" entry of the
// last tile weighted nsample - count.
//
// Two register layouts of a tile (v_mfma_f32_32x32x*, D[i][j] in lane j + 32 (i / 4 % 2),
// register 4 (i / 8) + i % 4):
//   T ("channels in registers"): D = W . X^T, lane = entry, register = channel;
//   N ("entries in registers"):  D = X . W^T, lane = channel, register = entry.
// A T-layout tile is directly the k-operand of a product over channels, an N-layout tile that of
// a product over entries (the weight gradients).  So z1 is formed in both (two fp32 MFMA k-steps
// from U each); z2 in N for the statistics, the forward max and dW2, in T for the backward chain
// gz2 -> gh1 = gz2 W2 (N) -> gz1 (N) -> dW1 = gz1^T [x].  Products over 16+ channels run as the
// three-way bf16 split of sa_mlp_mfma.hip (six v_mfma_f32_32x32x16_bf16, fp32-accurate).
//
// Statistics are summed per entry in fp64 (z^2 exact): the variance is E[z^2] - E[z]^2, a
// difference of nearly equal sums wherever |mean| >> std (sa1's first layer sees local
// coordinates of a few centimetres), and fp32 tile partials cost 5e-4 of the running variance there.
// Passes: S1 / S2 = the statistics of layer 1 / 2 (fp64 per-wave partials), FWD = the output max
// with its arg-max entry and that entry's z2 (what routes the backward), B1 = A1, B1 (layer 2's
// sums come from the routed rows alone, host side), B0A = dW2, db2, B0B = dW1, db1 and the
// per-entry gz1 rows of the feature gradient (segment sums, segsum.hip).  Weight-gradient
// partials are per wave (fp32 MFMA accumulators), summed in fp64 in a fixed order: deterministic.
#include "common.h"

#include <algorithm>

namespace dvcp {

// segsum.hip
int64_t segment_sum_workspace_bytes(int64_t E, int64_t nrows);
int segment_sum(const uint32_t* keys, const float* contrib, int64_t E, int64_t nrows, int ncol, float* out, void* ws,
                hipStream_t st);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBnmWaves = 4;
constexpr int kBnmThreads = kBnmWaves * kWave;
constexpr int kBnmMaxGrid = 1024;

enum : int { kS1 = 1, kS2 = 2, kS3 = 8, kFwd = 3, kB1 = 4, kB0A = 5, kB0B = 6 };

// x = p0 + p1 + p2 exactly (bf16 pieces of eight fp32 values)
struct Pieces {
  bf16x8 p0, p1, p2;
};
__device__ __forceinline__ Pieces bnm_split(const float (&x)[8]) {
  Pieces s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 b0 = static_cast<__bf16>(x[j]);
    const float r1 = x[j] - static_cast<float>(b0);
    const __bf16 b1 = static_cast<__bf16>(r1);
    s.p0[j] = b0;
    s.p1[j] = b1;
    s.p2[j] = static_cast<__bf16>(r1 - static_cast<float>(b1));
  }
  return s;
}
// acc += a . b over one 16-deep k-step: the six significant piece products, smallest first
__device__ __forceinline__ f32x16 bnm_mfma6(const Pieces& a, const Pieces& b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p2, b.p0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b.p1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b.p2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b.p0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b.p1, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b.p0, acc, 0, 0, 0);
}
// row of accumulator register r in lane half h (32x32 D map)
__device__ __forceinline__ int arow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int D, int C1, int C2>
struct BnmShape {
  static constexpr int C0 = 3 + D;
  static constexpr int MT = C1 / 32, CT = C2 / 32, DT = D / 32;
  static constexpr int KB1 = C1 / 16, KB2 = C2 / 16;  // 16-deep k-steps over layer-1 / layer-2 channels
  static_assert(D % 32 == 0 && C1 % 32 == 0 && C2 % 32 == 0 && C2 <= 64, "tiling");
};

template <int D, int C1, int C2>
struct BnmLds {
  using S = BnmShape<D, C1, C2>;
  float wx[S::MT][2][64];               // W1 xyz columns: k-steps (x | y), (z | 0), lane = channel
  bf16x8 w2s[S::CT][S::KB1][3][64];     // W2 rows (lane = c2), k = c1 in T register order
  bf16x8 w2t[S::MT][S::KB2][3][64];     // W2 columns (lane = c1), k = c2 in T register order
  float s1T[S::MT][2][16], t1T[S::MT][2][16];  // layer-1 BN scale / shift by T register
  float b2T[S::CT][2][16];              // layer-2 bias by T register
  float4 q2T[S::CT][2][16];             // layer-2 backward constants {s2, k2, mu2, ka2} by T register
  int2 route[kBnmWaves][C2];            // the wave's centre: per c2 {arg-max entry, routed gradient}
  float4 dtab[kBnmWaves][32];           // the tile's entries: (dx, dy, dz, weight)
  int ntab[kBnmWaves][32];              // the tile's entries: point index
};

struct BnmArgs {
  const float* xyz;
  int64_t sb, sc, sn;
  const float* ctr;
  int64_t cb, cc, cn;
  int S, B, N, nsample;
  const float* feat;  // feat[b fb + d fd + n fn] (the two-layer tables: fd = 1, 16-byte aligned rows)
  int64_t fb, fd, fn;
  const int32_t* count;
  const int32_t* list;
  const float* pack;  // per layer W | bias | scale | shift | mean | istd | A/M | B/M
  const float* U;     // (B, N, C1) = W1f f + b1
  const float* gout;  // (B S, C2)
  int32_t* arg;       // (B S, C2)
  float* out;         // (B S, C2)
  float* zbest;       // (B S, C2)
  void* part;         // per-wave partials
  float* frows;       // (E, C1) gz1 rows (B0B, feature gradient)
  uint32_t* fkeys;    // (E) their point rows b N + n; sentinel B N: none
};

template <int D, int C1, int C2, int PASS>
__global__ __launch_bounds__(kBnmThreads) __attribute__((amdgpu_waves_per_eu(PASS >= kB1 ? 1 : 2))) void sa_bnm_kernel(
    BnmArgs a) {
  using Sh = BnmShape<D, C1, C2>;
  constexpr int C0 = Sh::C0, MT = Sh::MT, CT = Sh::CT, KB1 = Sh::KB1, KB2 = Sh::KB2;
  constexpr bool kZ2N = PASS == kS2 || PASS == kFwd || PASS == kB0A;
  constexpr bool kZ2T = PASS == kB1 || PASS == kB0B;
  constexpr bool kRoute = PASS == kB1 || PASS == kB0A || PASS == kB0B;
  __shared__ BnmLds<D, C1, C2> L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;

  // ---- weights and per-channel constants -----------------------------------------------------
  const float* W1 = a.pack;
  const float* v1 = W1 + C1 * C0;  // bias | scale | shift | mean | istd | A/M | B/M
  const float* W2 = v1 + 7 * C1;
  const float* v2 = W2 + C2 * C1;
  for (int i = tid; i < MT * 2 * 64; i += kBnmThreads) {
    const int l = i % 64, s = (i / 64) % 2, mt = i / 128;
    const int ch = s == 0 ? (l >> 5) : ((l >> 5) == 0 ? 2 : -1);
    L.wx[mt][s][l] = ch < 0 ? 0.0f : W1[(32 * mt + (l & 31)) * C0 + ch];
  }
  if constexpr (kZ2N || kZ2T)
    for (int i = tid; i < CT * KB1 * 64; i += kBnmThreads) {
      const int l = i % 64, s = (i / 64) % KB1, ct = i / (64 * KB1);
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = W2[(32 * ct + (l & 31)) * C1 + 32 * (s / 2) + arow(8 * (s % 2) + j, l >> 5)];
      const Pieces p = bnm_split(w);
      L.w2s[ct][s][0][l] = p.p0;
      L.w2s[ct][s][1][l] = p.p1;
      L.w2s[ct][s][2][l] = p.p2;
    }
  if constexpr (kZ2T)
    for (int i = tid; i < MT * KB2 * 64; i += kBnmThreads) {
      const int l = i % 64, s = (i / 64) % KB2, mt = i / (64 * KB2);
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = W2[(32 * (s / 2) + arow(8 * (s % 2) + j, l >> 5)) * C1 + 32 * mt + (l & 31)];
      const Pieces p = bnm_split(w);
      L.w2t[mt][s][0][l] = p.p0;
      L.w2t[mt][s][1][l] = p.p1;
      L.w2t[mt][s][2][l] = p.p2;
    }
  for (int i = tid; i < MT * 32; i += kBnmThreads) {
    const int r = i % 16, hh = (i / 16) % 2, mt = i / 32;
    const int c = 32 * mt + arow(r, hh);
    L.s1T[mt][hh][r] = v1[C1 + c];
    L.t1T[mt][hh][r] = v1[2 * C1 + c];
  }
  if constexpr (kZ2T)
    for (int i = tid; i < CT * 32; i += kBnmThreads) {
      const int r = i % 16, hh = (i / 16) % 2, ct = i / 32;
      const int c = 32 * ct + arow(r, hh);
      const double s2 = v2[C2 + c], is2 = v2[4 * C2 + c];
      L.b2T[ct][hh][r] = v2[c];
      L.q2T[ct][hh][r] = make_float4(v2[C2 + c], static_cast<float>(-(s2 * v2[6 * C2 + c] * is2)), v2[3 * C2 + c],
                                     static_cast<float>(s2 * v2[5 * C2 + c]));
    }
  // N-layout constants: lane = channel
  float s1n[MT], t1n[MT], mu1n[MT], is1n[MT], k1n[MT], ka1n[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int c = 32 * mt + r32;
    s1n[mt] = v1[C1 + c];
    t1n[mt] = v1[2 * C1 + c];
    mu1n[mt] = v1[3 * C1 + c];
    is1n[mt] = v1[4 * C1 + c];
    k1n[mt] = static_cast<float>(-(static_cast<double>(s1n[mt]) * v1[6 * C1 + c] * is1n[mt]));
    ka1n[mt] = static_cast<float>(static_cast<double>(s1n[mt]) * v1[5 * C1 + c]);
  }
  float b2n[CT], s2n[CT], t2n[CT], mu2n[CT], k2n[CT], ka2n[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int c = 32 * ct + r32;
    b2n[ct] = v2[c];
    s2n[ct] = v2[C2 + c];
    t2n[ct] = v2[2 * C2 + c];
    mu2n[ct] = v2[3 * C2 + c];
    k2n[ct] = static_cast<float>(-(static_cast<double>(s2n[ct]) * v2[6 * C2 + c] * v2[4 * C2 + c]));
    ka2n[ct] = static_cast<float>(static_cast<double>(s2n[ct]) * v2[5 * C2 + c]);
  }
  __syncthreads();

  // ---- accumulators over the wave's centres ---------------------------------------------------
  constexpr int CS = PASS == kS2 ? CT : MT;  // statistics channel tiles (S1, S2, B1)
  double st1[CS], st2[CS];
#pragma unroll
  for (int i = 0; i < CS; ++i) st1[i] = st2[i] = 0.0;
  f32x16 dw2[CT][MT];
  float db2[CT], dx1[MT][4];  // B0A: db2; B0B: the xyz columns of dW1 and db1
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    db2[ct] = 0.0f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) dw2[ct][mt][r] = 0.0f;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int k = 0; k < 4; ++k) dx1[mt][k] = 0.0f;

  const int ns = a.nsample;
  const uint32_t sentinel = static_cast<uint32_t>(a.B) * static_cast<uint32_t>(a.N);
  const int64_t total = static_cast<int64_t>(a.B) * a.S;
  for (int64_t fc = static_cast<int64_t>(blockIdx.x) * kBnmWaves + wave; fc < total;
       fc += static_cast<int64_t>(gridDim.x) * kBnmWaves) {
    const int b = static_cast<int>(fc / a.S), s = static_cast<int>(fc - static_cast<int64_t>(b) * a.S);
    int rows = a.count[fc];
    rows = rows < 1 ? 1 : (rows > ns ? ns : rows);
    const int ghost = rows < ns ? 1 : 0;
    const float gw = static_cast<float>(ns - rows);  // the ghost entry's weight
    const float cx = a.ctr[b * a.cb + s * a.cn], cy = a.ctr[b * a.cb + a.cc + s * a.cn],
                cz = a.ctr[b * a.cb + 2 * a.cc + s * a.cn];
    const int32_t* lst = a.list + fc * ns;
    const float* Ub = a.U + static_cast<int64_t>(b) * a.N * C1;
    int argN[CT];
    float gN[CT];
    if constexpr (kRoute) {
      // the routed gradient: g where the forward max is positive (gy2 = [y2 > 0] g at the arg-max)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int64_t o = fc * C2 + 32 * ct + r32;
        const float g = a.gout[o];
        argN[ct] = a.arg[o];
        gN[ct] = a.out[o] > 0.0f ? g : 0.0f;
        if (h == 0) L.route[wave][32 * ct + r32] = make_int2(argN[ct], __float_as_int(gN[ct]));
      }
    }
    float best[CT], bz[CT];
    int barg[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      best[ct] = -1.0f;  // outputs are >= 0
      bz[ct] = 0.0f;
      barg[ct] = 0;
    }
    const int ntiles = (rows + ghost + 31) / 32;
    for (int t = 0; t < ntiles; ++t) {
      __builtin_amdgcn_wave_barrier();  // (the previous tile's reads of ntab / dtab come first)
      // An opaque zero added to the LDS indices of the weight fragments and per-channel tables:
      // they are re-read per tile (one ds_read per use) instead of being hoisted out of the loops
      // into a few hundred registers.
      int zo = 0;
      asm volatile("" : "+v"(zo));
      const int n0 = 32 * t;
      // T layout: this lane's entry
      const int p = n0 + r32;
      const bool valid = p < rows, isg = ghost && p == rows;
      const int n = lst[valid ? p : 0];
      const float dx = a.xyz[b * a.sb + n * a.sn] - cx;
      const float dy = a.xyz[b * a.sb + a.sc + n * a.sn] - cy;
      const float dz = a.xyz[b * a.sb + 2 * a.sc + n * a.sn] - cz;
      const float x0 = h == 0 ? dx : dy, x1 = h == 0 ? dz : 0.0f;
      if (h == 0) {
        L.ntab[wave][r32] = n;
        L.dtab[wave][r32] = make_float4(dx, dy, dz, 0.0f);
      }
      if constexpr (PASS == kB0B) {
        if (a.fkeys && h == 0 && p < ns)
          a.fkeys[fc * ns + p] = (valid || isg) ? static_cast<uint32_t>(b) * a.N + n : sentinel;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      // N layout: register r holds entry arow(r, h) of the tile, of weight wt(r)
      auto wt = [&](int r) {
        const int pa = n0 + arow(r, h);
        return pa < rows ? 1.0f : ((ghost && pa == rows) ? gw : 0.0f);
      };
      // z1 in N layout: the U rows of the N entries + the xyz k-steps.  The gathers are ordered
      // after `dep` (the last result of the chain before them), so they do not hold registers
      // across it.
      auto z1_n = [&](f32x16(&z)[MT], float dep) {
        int q[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          q[r] = L.ntab[wave][arow(r, h)];
          asm volatile("" : "+v"(q[r]) : "v"(dep));
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
          for (int r = 0; r < 16; ++r) z[mt][r] = Ub[static_cast<int64_t>(q[r]) * C1 + 32 * mt + r32];
          z[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, L.wx[mt][0][lane + zo], z[mt], 0, 0, 0);
          z[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, L.wx[mt][1][lane + zo], z[mt], 0, 0, 0);
        }
      };

      if constexpr (PASS == kS1) {
        f32x16 z1N[MT];
        z1_n(z1N, 0.0f);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          double a1 = 0.0, a2 = 0.0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float z = z1N[mt][r], w = wt(r);
            a1 += static_cast<double>(w) * z;
            a2 += static_cast<double>(w) * (static_cast<double>(z) * z);
          }
          st1[mt] += a1;
          st2[mt] += a2;
        }
        continue;
      }

      // ---- z1, T layout: U rows + the xyz k-steps; h1 -----------------------------------------------
      f32x16 h1T[MT];
      {
        const float4* ur = reinterpret_cast<const float4*>(Ub + static_cast<int64_t>(n) * C1 + 4 * h);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 u = ur[8 * mt + 2 * i];
            h1T[mt][4 * i] = u.x;
            h1T[mt][4 * i + 1] = u.y;
            h1T[mt][4 * i + 2] = u.z;
            h1T[mt][4 * i + 3] = u.w;
          }
          h1T[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[mt][0][lane + zo], x0, h1T[mt], 0, 0, 0);
          h1T[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[mt][1][lane + zo], x1, h1T[mt], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float y = h1T[mt][r] * L.s1T[mt][h][r + zo] + L.t1T[mt][h][r + zo];
            h1T[mt][r] = y > 0.0f ? y : 0.0f;
          }
        }
      }

      // ---- z2, N layout: statistics, forward max, dW2 -------------------------------------------------
      if constexpr (kZ2N) {
        f32x16 z2N[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) z2N[ct][r] = b2n[ct];
#pragma unroll
        for (int k = 0; k < KB1; ++k) {
          float x[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = h1T[k / 2][8 * (k % 2) + j];
          const Pieces pa = bnm_split(x);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const Pieces pb{L.w2s[ct][k][0][lane + zo], L.w2s[ct][k][1][lane + zo], L.w2s[ct][k][2][lane + zo]};
            z2N[ct] = bnm_mfma6(pa, pb, z2N[ct]);
          }
        }
        if constexpr (PASS == kS2) {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            double a1 = 0.0, a2 = 0.0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float z = z2N[ct][r], w = wt(r);
              a1 += static_cast<double>(w) * z;
              a2 += static_cast<double>(w) * (static_cast<double>(z) * z);
            }
            st1[ct] += a1;
            st2[ct] += a2;
          }
        } else if constexpr (PASS == kFwd) {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int pa = n0 + arow(r, h);
              const float y = z2N[ct][r] * s2n[ct] + t2n[ct];
              const float hv = y > 0.0f ? y : 0.0f;
              if (pa < rows && hv > best[ct]) {  // strict: the first of equal maxima (entries ascend)
                best[ct] = hv;
                barg[ct] = pa;
                bz[ct] = z2N[ct][r];
              }
            }
        } else {  // kB0A: weighted gz2 in place, then h1 in N layout, dW2 += gz2^T h1 over the entries
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int pa = n0 + arow(r, h);
              const float z = z2N[ct][r];
              const float gy = pa == argN[ct] ? gN[ct] : 0.0f;
              z2N[ct][r] = wt(r) * ((s2n[ct] * gy + k2n[ct] * (z - mu2n[ct])) - ka2n[ct]);
              db2[ct] += z2N[ct][r];
            }
          f32x16 h1N[MT];
          z1_n(h1N, z2N[CT - 1][15]);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float y = h1N[mt][r] * s1n[mt] + t1n[mt];
              h1N[mt][r] = y > 0.0f ? y : 0.0f;
            }
#pragma unroll
          for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              float y[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) y[j] = h1N[mt][8 * k + j];
              const Pieces ph = bnm_split(y);
#pragma unroll
              for (int ct = 0; ct < CT; ++ct) {
                float x[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = z2N[ct][8 * k + j];
                dw2[ct][mt] = bnm_mfma6(bnm_split(x), ph, dw2[ct][mt]);
              }
            }
        }
      }

      // ---- z2, T layout -> gz2 -> gh1 (N) -> gz1: A1, B1 or dW1's xyz columns, db1, the gz1 rows ----
      if constexpr (kZ2T) {
        f32x16 g2T[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) g2T[ct][r] = L.b2T[ct][h][r + zo];
#pragma unroll
        for (int k = 0; k < KB1; ++k) {
          float x[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = h1T[k / 2][8 * (k % 2) + j];
          const Pieces pb = bnm_split(x);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const Pieces pw{L.w2s[ct][k][0][lane + zo], L.w2s[ct][k][1][lane + zo], L.w2s[ct][k][2][lane + zo]};
            g2T[ct] = bnm_mfma6(pw, pb, g2T[ct]);
          }
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c = 32 * ct + arow(r, h);
            const int2 rt = L.route[wave][c + zo];
            const float4 q = L.q2T[ct][h][r + zo];
            const float gy = p == rt.x ? __int_as_float(rt.y) : 0.0f;
            g2T[ct][r] = (q.x * gy + q.y * (g2T[ct][r] - q.z)) - q.w;  // gz2 (unweighted)
          }
        f32x16 gh1[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 16; ++r) gh1[mt][r] = 0.0f;
#pragma unroll
        for (int k = 0; k < KB2; ++k) {
          float x[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = g2T[k / 2][8 * (k % 2) + j];
          const Pieces pa = bnm_split(x);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const Pieces pw{L.w2t[mt][k][0][lane + zo], L.w2t[mt][k][1][lane + zo], L.w2t[mt][k][2][lane + zo]};
            gh1[mt] = bnm_mfma6(pa, pw, gh1[mt]);
          }
        }
        f32x16 z1N[MT];
        z1_n(z1N, gh1[MT - 1][15]);
        if constexpr (PASS == kB1) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            double a1 = 0.0, a2 = 0.0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float z = z1N[mt][r], w = wt(r);
              const float gy = z * s1n[mt] + t1n[mt] > 0.0f ? gh1[mt][r] : 0.0f;
              a1 += static_cast<double>(w) * gy;
              a2 += static_cast<double>(w) * (gy * ((z - mu1n[mt]) * is1n[mt]));
            }
            st1[mt] += a1;
            st2[mt] += a2;
          }
        } else {  // kB0B
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float4 dq = L.dtab[wave][arow(r, h)];
            const float w = wt(r);
            const int64_t e = fc * ns + n0 + arow(r, h);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              const float z = z1N[mt][r];
              const float gy = z * s1n[mt] + t1n[mt] > 0.0f ? gh1[mt][r] : 0.0f;
              const float gz = w * ((s1n[mt] * gy + k1n[mt] * (z - mu1n[mt])) - ka1n[mt]);  // weighted gz1
              dx1[mt][0] += gz * dq.x;
              dx1[mt][1] += gz * dq.y;
              dx1[mt][2] += gz * dq.z;
              dx1[mt][3] += gz;
              if (a.frows && w != 0.0f) a.frows[e * C1 + 32 * mt + r32] = gz;
            }
          }
        }
      }
    }
    if constexpr (PASS == kB0B) {
      if (a.fkeys)
        for (int r = ntiles * 32 + lane; r < ns; r += kWave) a.fkeys[fc * ns + r] = sentinel;
    }
    if constexpr (PASS == kFwd) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const float ob = __shfl_xor(best[ct], 32, kWave), oz = __shfl_xor(bz[ct], 32, kWave);
        const int oa = __shfl_xor(barg[ct], 32, kWave);
        if (ob > best[ct] || (ob == best[ct] && oa < barg[ct])) {
          best[ct] = ob;
          barg[ct] = oa;
          bz[ct] = oz;
        }
        if (h == 0) {
          const int64_t o = fc * C2 + 32 * ct + r32;
          a.out[o] = best[ct];
          a.arg[o] = barg[ct];
          a.zbest[o] = bz[ct];
        }
      }
    }
    if constexpr (kRoute) {
      __builtin_amdgcn_wave_barrier();  // (the next centre rewrites route)
    }
  }

  // ---- per-wave partials ------------------------------------------------------------------------
  const int64_t wg = static_cast<int64_t>(blockIdx.x) * kBnmWaves + wave;
  if constexpr (PASS == kS1 || PASS == kS2 || PASS == kB1) {
    constexpr int C = PASS == kS2 ? C2 : C1;
    double* o = static_cast<double*>(a.part) + (wg * 2 + h) * (2 * C);  // one row per lane half
#pragma unroll
    for (int i = 0; i < CS; ++i) {
      o[32 * i + r32] = st1[i];
      o[C + 32 * i + r32] = st2[i];
    }
  } else if constexpr (PASS == kB0A) {
    constexpr int P = C2 * C1 + C2;
    float* o = static_cast<float*>(a.part) + wg * P;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[(32 * ct + arow(r, h)) * C1 + 32 * mt + r32] = dw2[ct][mt][r];
      const float d = db2[ct] + __shfl_xor(db2[ct], 32, kWave);
      if (h == 0) o[C2 * C1 + 32 * ct + r32] = d;
    }
  } else if constexpr (PASS == kB0B) {
    float* o = static_cast<float*>(a.part) + wg * (4 * C1);  // [c][x, y, z, bias]
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float d[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k] = dx1[mt][k] + __shfl_xor(dx1[mt][k], 32, kWave);
      if (h == 0) *reinterpret_cast<float4*>(o + 4 * (32 * mt + r32)) = make_float4(d[0], d[1], d[2], d[3]);
    }
  }
}

// ---- sa1: 3 [+3 normals] - 16 - 16 - 32 --------------------------------------------------------
// The same scheme for the three-layer table.  The 16-channel layers fill half of a 32-row tile (the
// other rows have zero weights and constants, so they stay zero), and a product over 16 channels
// is one 16-deep k-step: in T register order k-step 0 (registers 0..7) holds channels 0..15 in
// both lane halves.  Layer 1 (k = 3 or 6) is fp32 MFMA k-steps from the bias; there is no
// per-point table.  Passes: S1..S3, FWD, B2 = A2, B2 (needs A3, B3 from the host), B1 = A1, B1,
// B0 = every weight gradient (dW3 = gz3^T h2, dW2 = gz2^T h1 on the matrix cores, dW1 on VALU).
// No feature gradient: the layer's input features are the data (normals) or absent.
struct Bnm3Lds {
  float wx[4][64];       // W1: k-steps (x | y), (z | 0), (nx | ny), (nz | 0); lane = c1 row
  bf16x8 w2[3][64];      // W2: lane = c2 row, k = c1 (T order)
  bf16x8 w2t[3][64];     // W2^T: lane = c1 row, k = c2
  bf16x8 w3[3][64];      // W3: lane = c3 row, k = c2
  bf16x8 w3t[2][3][64];  // W3^T: lane = c2 row, k = c3 (two k-steps)
  float b1T[2][16], s1T[2][16], t1T[2][16];
  float b2T[2][16], s2T[2][16], t2T[2][16];
  float4 q2T[2][16];     // {s2, k2, mu2, ka2}
  float b3T[2][16];
  float4 q3T[2][16];     // {s3, k3, mu3, ka3}
  int2 route[kBnmWaves][32];
  float4 dtab[kBnmWaves][32];  // the tile's entries: (dx, dy, dz, -)
  float4 ntab[kBnmWaves][32];  // the tile's entries: normals
};

// One layer's per-channel constants for channel c (zero beyond C): bias, BN scale / shift, mean,
// istd, and the backward's k = -s b istd, ka = s a (a = A/M, b = B/M).
struct BnmLayerC {
  float b, s, t, mu, is, k, ka;
};
__device__ __forceinline__ BnmLayerC bnm_layer_c(const float* v, int C, int c) {
  BnmLayerC q{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    q.b = v[c];
    q.s = v[C + c];
    q.t = v[2 * C + c];
    q.mu = v[3 * C + c];
    q.is = v[4 * C + c];
    q.k = static_cast<float>(-(static_cast<double>(q.s) * v[6 * C + c] * q.is));
    q.ka = static_cast<float>(static_cast<double>(q.s) * v[5 * C + c]);
  }
  return q;
}

enum : int { kB2 = 7 };  // three-layer backward sums of layer 2

template <int D, int PASS>
__global__ __launch_bounds__(kBnmThreads) __attribute__((amdgpu_waves_per_eu(PASS == kB0A ? 1 : 2))) void sa_bnm3_kernel(
    BnmArgs a) {
  constexpr int C0 = 3 + D, C1 = 16, C2 = 16, C3 = 32;
  constexpr bool kRoute = PASS == kB2 || PASS == kB1 || PASS == kB0A;  // kB0A: every weight gradient
  __shared__ Bnm3Lds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const float* W1 = a.pack;
  const float* v1 = W1 + C1 * C0;
  const float* W2 = v1 + 7 * C1;
  const float* v2 = W2 + C2 * C1;
  const float* W3 = v2 + 7 * C2;
  const float* v3 = W3 + C3 * C2;
  for (int i = tid; i < 4 * 64; i += kBnmThreads) {
    const int l = i % 64, st = i / 64, c1 = l & 31, hh = l >> 5;
    int ch = st == 0 ? hh : (st == 1 ? (hh == 0 ? 2 : -1) : (st == 2 ? 3 + hh : (hh == 0 ? 5 : -1)));
    if (ch >= C0) ch = -1;
    L.wx[st][l] = (ch < 0 || c1 >= C1) ? 0.0f : W1[c1 * C0 + ch];
  }
  for (int l = tid; l < 64; l += kBnmThreads) {
    const int row = l & 31, hh = l >> 5;
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = row < C2 ? W2[row * C1 + arow(j, hh)] : 0.0f;
    Pieces p = bnm_split(w);
    L.w2[0][l] = p.p0, L.w2[1][l] = p.p1, L.w2[2][l] = p.p2;
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = row < C1 ? W2[arow(j, hh) * C1 + row] : 0.0f;
    p = bnm_split(w);
    L.w2t[0][l] = p.p0, L.w2t[1][l] = p.p1, L.w2t[2][l] = p.p2;
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = W3[row * C2 + arow(j, hh)];
    p = bnm_split(w);
    L.w3[0][l] = p.p0, L.w3[1][l] = p.p1, L.w3[2][l] = p.p2;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = row < C2 ? W3[arow(8 * k + j, hh) * C2 + row] : 0.0f;
      p = bnm_split(w);
      L.w3t[k][0][l] = p.p0, L.w3t[k][1][l] = p.p1, L.w3t[k][2][l] = p.p2;
    }
  }
  for (int i = tid; i < 32; i += kBnmThreads) {
    const int r = i % 16, hh = i / 16, c = arow(r, hh);
    const BnmLayerC q1 = bnm_layer_c(v1, C1, c), q2 = bnm_layer_c(v2, C2, c), q3 = bnm_layer_c(v3, C3, c);
    L.b1T[hh][r] = q1.b, L.s1T[hh][r] = q1.s, L.t1T[hh][r] = q1.t;
    L.b2T[hh][r] = q2.b, L.s2T[hh][r] = q2.s, L.t2T[hh][r] = q2.t;
    L.q2T[hh][r] = make_float4(q2.s, q2.k, q2.mu, q2.ka);
    L.b3T[hh][r] = q3.b;
    L.q3T[hh][r] = make_float4(q3.s, q3.k, q3.mu, q3.ka);
  }
  const BnmLayerC n1 = bnm_layer_c(v1, C1, r32), n2 = bnm_layer_c(v2, C2, r32), n3 = bnm_layer_c(v3, C3, r32);
  __syncthreads();

  constexpr int CS = PASS == kS3 ? C3 : 16;
  double st1 = 0.0, st2 = 0.0;
  f32x16 dw3, dw2;
#pragma unroll
  for (int r = 0; r < 16; ++r) dw3[r] = dw2[r] = 0.0f;
  float db2 = 0.0f, db3 = 0.0f, dw1[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) dw1[k] = 0.0f;

  const int ns = a.nsample;
  const int64_t total = static_cast<int64_t>(a.B) * a.S;
  for (int64_t fc = static_cast<int64_t>(blockIdx.x) * kBnmWaves + wave; fc < total;
       fc += static_cast<int64_t>(gridDim.x) * kBnmWaves) {
    const int b = static_cast<int>(fc / a.S), s = static_cast<int>(fc - static_cast<int64_t>(b) * a.S);
    int rows = a.count[fc];
    rows = rows < 1 ? 1 : (rows > ns ? ns : rows);
    const int ghost = rows < ns ? 1 : 0;
    const float gw = static_cast<float>(ns - rows);
    const float cx = a.ctr[b * a.cb + s * a.cn], cy = a.ctr[b * a.cb + a.cc + s * a.cn],
                cz = a.ctr[b * a.cb + 2 * a.cc + s * a.cn];
    const int32_t* lst = a.list + fc * ns;
    int argN = 0;
    float gN = 0.0f;
    if constexpr (kRoute) {
      const int64_t o = fc * C3 + r32;
      argN = a.arg[o];
      gN = a.out[o] > 0.0f ? a.gout[o] : 0.0f;
      if (h == 0) L.route[wave][r32] = make_int2(argN, __float_as_int(gN));
    }
    float best = -1.0f, bz = 0.0f;
    int barg = 0;
    const int ntiles = (rows + ghost + 31) / 32;
    for (int t = 0; t < ntiles; ++t) {
      __builtin_amdgcn_wave_barrier();
      int zo = 0;
      asm volatile("" : "+v"(zo));
      const int n0 = 32 * t;
      const int p = n0 + r32;
      const int n = lst[p < rows ? p : 0];
      const float dx = a.xyz[b * a.sb + n * a.sn] - cx;
      const float dy = a.xyz[b * a.sb + a.sc + n * a.sn] - cy;
      const float dz = a.xyz[b * a.sb + 2 * a.sc + n * a.sn] - cz;
      float nx = 0.0f, ny = 0.0f, nz = 0.0f;
      if constexpr (D == 3) {
        const float* fr = a.feat + b * a.fb + static_cast<int64_t>(n) * a.fn;
        nx = fr[0];
        ny = fr[a.fd];
        nz = fr[2 * a.fd];
      }
      const float x0 = h == 0 ? dx : dy, x1 = h == 0 ? dz : 0.0f;
      const float x2 = h == 0 ? nx : ny, x3 = h == 0 ? nz : 0.0f;
      if (h == 0) {
        L.dtab[wave][r32] = make_float4(dx, dy, dz, 0.0f);
        L.ntab[wave][r32] = make_float4(nx, ny, nz, 0.0f);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      auto wt = [&](int r) {
        const int pa = n0 + arow(r, h);
        return pa < rows ? 1.0f : ((ghost && pa == rows) ? gw : 0.0f);
      };
      auto frag = [&](const bf16x8(&f)[3][64]) { return Pieces{f[0][lane + zo], f[1][lane + zo], f[2][lane + zo]}; };
      auto piece = [&](const f32x16& v, int k) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = v[8 * k + j];
        return bnm_split(x);
      };
      auto z1_t = [&]() {
        f32x16 z;
#pragma unroll
        for (int r = 0; r < 16; ++r) z[r] = L.b1T[h][r + zo];
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[0][lane + zo], x0, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[1][lane + zo], x1, z, 0, 0, 0);
        if constexpr (D == 3) {
          z = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[2][lane + zo], x2, z, 0, 0, 0);
          z = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[3][lane + zo], x3, z, 0, 0, 0);
        }
        return z;
      };
      auto z1_n = [&]() {
        f32x16 z;
#pragma unroll
        for (int r = 0; r < 16; ++r) z[r] = n1.b;
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, L.wx[0][lane + zo], z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, L.wx[1][lane + zo], z, 0, 0, 0);
        if constexpr (D == 3) {
          z = __builtin_amdgcn_mfma_f32_32x32x2f32(x2, L.wx[2][lane + zo], z, 0, 0, 0);
          z = __builtin_amdgcn_mfma_f32_32x32x2f32(x3, L.wx[3][lane + zo], z, 0, 0, 0);
        }
        return z;
      };
      auto sums = [&](const f32x16& z) {
        double a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float w = wt(r);
          a1 += static_cast<double>(w) * z[r];
          a2 += static_cast<double>(w) * (static_cast<double>(z[r]) * z[r]);
        }
        st1 += a1;
        st2 += a2;
      };
      if constexpr (PASS == kS1) {
        sums(z1_n());
        continue;
      }
      // h1 (T)
      f32x16 h1T = z1_t();
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float y = h1T[r] * L.s1T[h][r + zo] + L.t1T[h][r + zo];
        h1T[r] = y > 0.0f ? y : 0.0f;
      }
      const Pieces ph1 = piece(h1T, 0);
      auto z2_n = [&]() {
        f32x16 z;
#pragma unroll
        for (int r = 0; r < 16; ++r) z[r] = n2.b;
        return bnm_mfma6(ph1, frag(L.w2), z);
      };
      if constexpr (PASS == kS2) {
        sums(z2_n());
        continue;
      }
      f32x16 z2T;
#pragma unroll
      for (int r = 0; r < 16; ++r) z2T[r] = L.b2T[h][r + zo];
      z2T = bnm_mfma6(frag(L.w2), ph1, z2T);
      f32x16 z2N;
      if constexpr (PASS == kB2 || PASS == kB0A) z2N = z2_n();
      f32x16 h2T;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float y = z2T[r] * L.s2T[h][r + zo] + L.t2T[h][r + zo];
        h2T[r] = y > 0.0f ? y : 0.0f;
      }
      const Pieces ph2 = piece(h2T, 0);
      if constexpr (PASS == kS3 || PASS == kFwd) {
        f32x16 z3N;
#pragma unroll
        for (int r = 0; r < 16; ++r) z3N[r] = n3.b;
        z3N = bnm_mfma6(ph2, frag(L.w3), z3N);
        if constexpr (PASS == kS3) {
          sums(z3N);
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int pa = n0 + arow(r, h);
            const float y = z3N[r] * n3.s + n3.t;
            const float hv = y > 0.0f ? y : 0.0f;
            if (pa < rows && hv > best) {
              best = hv;
              barg = pa;
              bz = z3N[r];
            }
          }
        }
        continue;
      }
      // ---- backward chain: gz3 (T) -> gh2 ----------------------------------------------------------
      f32x16 g3T;
#pragma unroll
      for (int r = 0; r < 16; ++r) g3T[r] = L.b3T[h][r + zo];
      g3T = bnm_mfma6(frag(L.w3), ph2, g3T);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int2 rt = L.route[wave][arow(r, h) + zo];
        const float4 q = L.q3T[h][r + zo];
        const float gy = p == rt.x ? __int_as_float(rt.y) : 0.0f;
        g3T[r] = (q.x * gy + q.y * (g3T[r] - q.z)) - q.w;  // gz3 (unweighted)
      }
      const Pieces pg0 = piece(g3T, 0), pg1 = piece(g3T, 1);
      if constexpr (PASS == kB2) {
        f32x16 gh2N;
#pragma unroll
        for (int r = 0; r < 16; ++r) gh2N[r] = 0.0f;
        gh2N = bnm_mfma6(pg0, frag(L.w3t[0]), gh2N);
        gh2N = bnm_mfma6(pg1, frag(L.w3t[1]), gh2N);
        double a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float z = z2N[r], w = wt(r);
          const float gy = z * n2.s + n2.t > 0.0f ? gh2N[r] : 0.0f;
          a1 += static_cast<double>(w) * gy;
          a2 += static_cast<double>(w) * (gy * ((z - n2.mu) * n2.is));
        }
        st1 += a1;
        st2 += a2;
        continue;
      }
      // gh2 (T) -> gz2 (T) -> gh1 (N)
      f32x16 gz2T;
#pragma unroll
      for (int r = 0; r < 16; ++r) gz2T[r] = 0.0f;
      gz2T = bnm_mfma6(frag(L.w3t[0]), pg0, gz2T);
      gz2T = bnm_mfma6(frag(L.w3t[1]), pg1, gz2T);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float4 q = L.q2T[h][r + zo];
        const float z = z2T[r];
        const float gy = z * L.s2T[h][r + zo] + L.t2T[h][r + zo] > 0.0f ? gz2T[r] : 0.0f;
        gz2T[r] = (q.x * gy + q.y * (z - q.z)) - q.w;
      }
      f32x16 gh1N;
#pragma unroll
      for (int r = 0; r < 16; ++r) gh1N[r] = 0.0f;
      gh1N = bnm_mfma6(piece(gz2T, 0), frag(L.w2t), gh1N);
      const f32x16 z1N = z1_n();
      if constexpr (PASS == kB1) {
        double a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float z = z1N[r], w = wt(r);
          const float gy = z * n1.s + n1.t > 0.0f ? gh1N[r] : 0.0f;
          a1 += static_cast<double>(w) * gy;
          a2 += static_cast<double>(w) * (gy * ((z - n1.mu) * n1.is));
        }
        st1 += a1;
        st2 += a2;
        continue;
      }
      // ---- every weight gradient (N layouts) -------------------------------------------------------
      // dW3 += gz3^T h2
      f32x16 g3N;
#pragma unroll
      for (int r = 0; r < 16; ++r) g3N[r] = n3.b;
      g3N = bnm_mfma6(ph2, frag(L.w3), g3N);
      f32x16 h2N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pa = n0 + arow(r, h);
        const float gy = pa == argN ? gN : 0.0f;
        g3N[r] = wt(r) * ((n3.s * gy + n3.k * (g3N[r] - n3.mu)) - n3.ka);
        db3 += g3N[r];
        const float y = z2N[r] * n2.s + n2.t;
        h2N[r] = y > 0.0f ? y : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) dw3 = bnm_mfma6(piece(g3N, k), piece(h2N, k), dw3);
      // dW2 += gz2^T h1 (gh2 in N layout)
      f32x16 g2N;
#pragma unroll
      for (int r = 0; r < 16; ++r) g2N[r] = 0.0f;
      g2N = bnm_mfma6(pg0, frag(L.w3t[0]), g2N);
      g2N = bnm_mfma6(pg1, frag(L.w3t[1]), g2N);
      f32x16 h1N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float z = z2N[r];
        const float gy = z * n2.s + n2.t > 0.0f ? g2N[r] : 0.0f;
        g2N[r] = wt(r) * ((n2.s * gy + n2.k * (z - n2.mu)) - n2.ka);
        db2 += g2N[r];
        const float y = z1N[r] * n1.s + n1.t;
        h1N[r] = y > 0.0f ? y : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) dw2 = bnm_mfma6(piece(g2N, k), piece(h1N, k), dw2);
      // dW1, db1 (VALU; lane = c1)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float z = z1N[r];
        const float gy = z * n1.s + n1.t > 0.0f ? gh1N[r] : 0.0f;
        const float gz = wt(r) * ((n1.s * gy + n1.k * (z - n1.mu)) - n1.ka);
        const float4 dq = L.dtab[wave][arow(r, h)];
        dw1[0] += gz * dq.x;
        dw1[1] += gz * dq.y;
        dw1[2] += gz * dq.z;
        if constexpr (D == 3) {
          const float4 nq = L.ntab[wave][arow(r, h)];
          dw1[3] += gz * nq.x;
          dw1[4] += gz * nq.y;
          dw1[5] += gz * nq.z;
        }
        dw1[6] += gz;
      }
    }
    if constexpr (PASS == kFwd) {
      const float ob = __shfl_xor(best, 32, kWave), oz = __shfl_xor(bz, 32, kWave);
      const int oa = __shfl_xor(barg, 32, kWave);
      if (ob > best || (ob == best && oa < barg)) {
        best = ob;
        barg = oa;
        bz = oz;
      }
      if (h == 0) {
        const int64_t o = fc * C3 + r32;
        a.out[o] = best;
        a.arg[o] = barg;
        a.zbest[o] = bz;
      }
    }
    if constexpr (kRoute) {
      __builtin_amdgcn_wave_barrier();
    }
  }

  const int64_t wg = static_cast<int64_t>(blockIdx.x) * kBnmWaves + wave;
  if constexpr (PASS == kS1 || PASS == kS2 || PASS == kS3 || PASS == kB1 || PASS == kB2) {
    double* o = static_cast<double*>(a.part) + (wg * 2 + h) * (2 * CS);
    if (r32 < CS) {
      o[r32] = st1;
      o[CS + r32] = st2;
    }
  } else if constexpr (PASS == kB0A) {
    constexpr int P1 = C1 * C0 + C1, P2 = C2 * C1 + C2, P3 = C3 * C2 + C3;
    float* o = static_cast<float*>(a.part) + wg * (P1 + P2 + P3);
    float d[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) d[k] = dw1[k] + __shfl_xor(dw1[k], 32, kWave);
    const float e2 = db2 + __shfl_xor(db2, 32, kWave), e3 = db3 + __shfl_xor(db3, 32, kWave);
    if (h == 0) {
      if (r32 < C1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) o[r32 * C0 + k] = d[k];
#pragma unroll
        for (int k = 0; k < D; ++k) o[r32 * C0 + 3 + k] = d[3 + k];
        o[C1 * C0 + r32] = d[6];
        o[P1 + C2 * C1 + r32] = e2;
      }
      o[P1 + P2 + C3 * C2 + r32] = e3;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = arow(r, h);
      if (row < C2 && r32 < C1) o[P1 + row * C1 + r32] = dw2[r];
      if (r32 < C2) o[P1 + P2 + row * C2 + r32] = dw3[r];
    }
  }
}

// U[b][n] = W1f f_n + b1 (fp32, features in ascending order from the bias): thread (point,
// 4-channel group), the weights as [k][c] float4 rows in LDS.
template <int D, int C1>
__global__ __launch_bounds__(256) void bnm_pre_kernel(const float* __restrict__ feat, int64_t fb, int64_t fn, int N,
                                                      int B, const float* __restrict__ pack, float* __restrict__ U) {
  constexpr int C0 = 3 + D, CG = C1 / 4, PPB = 256 / CG;
  __shared__ float4 w[D][CG];
  __shared__ float4 bias[CG];
  for (int i = threadIdx.x; i < D * C1; i += 256) {
    const int k = i / C1, c = i % C1;
    reinterpret_cast<float*>(&w[k][0])[c] = pack[c * C0 + 3 + k];
  }
  for (int c = threadIdx.x; c < C1; c += 256) reinterpret_cast<float*>(&bias[0])[c] = pack[C1 * C0 + c];
  __syncthreads();
  const int g = threadIdx.x % CG;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * PPB + threadIdx.x / CG;
  if (i >= static_cast<int64_t>(B) * N) return;
  const int b = static_cast<int>(i / N), n = static_cast<int>(i % N);
  const float4* fr = reinterpret_cast<const float4*>(feat + b * fb + static_cast<int64_t>(n) * fn);
  float4 acc = bias[g];
#pragma unroll 4
  for (int v = 0; v < D / 4; ++v) {
    const float4 q = fr[v];
    const float fq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float4 wk = w[4 * v + e][g];
      acc.x = __fmaf_rn(wk.x, fq[e], acc.x);
      acc.y = __fmaf_rn(wk.y, fq[e], acc.y);
      acc.z = __fmaf_rn(wk.z, fq[e], acc.z);
      acc.w = __fmaf_rn(wk.w, fq[e], acc.w);
    }
  }
  reinterpret_cast<float4*>(U + i * C1)[g] = acc;
}

// out[e] = sum over the nw partial rows of part[k][e] in fp64, in a fixed order.
template <typename PT, typename OT>
__global__ __launch_bounds__(1024) void bnm_sum_kernel(const PT* __restrict__ part, int nw, int P, OT* __restrict__ out) {
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

// Slice sums of the partial rows: block (column group, slice s) sums rows [s per, (s + 1) per) in
// a fixed order into tmp[s] (fp64); bnm_sum_kernel then adds the slices in order.  (One workgroup
// per 64 columns over thousands of rows was latency-bound: 0.13 ms for a 128-column statistic.)
template <typename PT>
__global__ __launch_bounds__(1024) void bnm_slice_kernel(const PT* __restrict__ part, int nrows, int P, int per,
                                                         double* __restrict__ tmp) {
  __shared__ double sl[16][64];
  const int tid = threadIdx.x, c = tid & 63, lane16 = tid >> 6;
  const int e = blockIdx.x * 64 + c;
  const int r0 = blockIdx.y * per, r1 = min(nrows, r0 + per);
  double acc = 0.0;
  if (e < P)
    for (int k = r0 + lane16; k < r1; k += 16) acc += static_cast<double>(part[static_cast<int64_t>(k) * P + e]);
  sl[lane16][c] = acc;
  __syncthreads();
  if (tid < 64 && e < P) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += sl[k][c];
    tmp[static_cast<int64_t>(blockIdx.y) * P + e] = t;
  }
}

// The feature columns of dW1 through the per-point sums: sum_e gz1[e] f[n(e)]^T = sum_n G[n] f[n]^T
// (G = the segment sums of the gz1 rows, which the feature gradient needs anyway): a product over
// the B N points instead of the B S nsample entries.  Block k sums points [k per, (k+1) per) into
// its partial row (C1 x D, fp32); thread t owns outputs t, t + 256, ...
template <int D, int C1>
__global__ __launch_bounds__(256) void bnm_gtf_kernel(const float* __restrict__ G, const float* __restrict__ feat,
                                                      int64_t fb, int64_t fn, int N, int64_t npts, int64_t per,
                                                      float* __restrict__ part) {
  constexpr int OUT = C1 * D / 256;
  __shared__ float gs[64][C1 + 1];
  __shared__ float fs[64][D + 1];
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * per;
  const int64_t p1 = p0 + per < npts ? p0 + per : npts;
  float acc[OUT];
#pragma unroll
  for (int i = 0; i < OUT; ++i) acc[i] = 0.0f;
  for (int64_t pb = p0; pb < p1; pb += 64) {
    const int np = static_cast<int>(p1 - pb < 64 ? p1 - pb : 64);
    for (int i = threadIdx.x; i < 64 * C1; i += 256) {
      const int j = i / C1, c = i % C1;
      gs[j][c] = j < np ? G[(pb + j) * C1 + c] : 0.0f;
    }
    for (int i = threadIdx.x; i < 64 * D; i += 256) {
      const int j = i / D, d = i % D;
      const int64_t row = pb + j;
      const int bb = static_cast<int>(row / N), nn = static_cast<int>(row % N);
      fs[j][d] = j < np ? feat[bb * fb + nn * fn + d] : 0.0f;
    }
    __syncthreads();
    for (int j = 0; j < np; ++j)
#pragma unroll
      for (int i = 0; i < OUT; ++i) {
        const int o = threadIdx.x + 256 * i;
        acc[i] = __fmaf_rn(gs[j][o / D], fs[j][o % D], acc[i]);
      }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < OUT; ++i) part[static_cast<int64_t>(blockIdx.x) * (C1 * D) + threadIdx.x + 256 * i] = acc[i];
}

// grads[0 : C1 C0 + C1] = dW1 | db1 from the xyz / bias sums xb (C1 x 4) and the feature columns fw (C1 x D)
template <int D, int C1>
__global__ __launch_bounds__(256) void bnm_dw1_kernel(const float* __restrict__ xb, const float* __restrict__ fw,
                                                      float* __restrict__ grads) {
  constexpr int C0 = 3 + D;
  for (int i = threadIdx.x; i < C1 * C0 + C1; i += 256) {
    if (i < C1 * C0) {
      const int c = i / C0, k = i % C0;
      grads[i] = k < 3 ? xb[4 * c + k] : fw[c * D + k - 3];
    } else {
      grads[i] = xb[4 * (i - C1 * C0) + 3];
    }
  }
}

// gfeat[b][n][d] = sum_c G[b N + n][c] W1[c][3 + d] (fp32, c ascending): thread (point, d).
template <int D, int C1>
__global__ __launch_bounds__(256) void bnm_feat_grad_kernel(const float* __restrict__ G, const float* __restrict__ pack,
                                                            int64_t rows, float* __restrict__ gfeat) {
  constexpr int C0 = 3 + D;
  __shared__ float w[C1][D];
  for (int i = threadIdx.x; i < C1 * D; i += 256) w[i / D][i % D] = pack[(i / D) * C0 + 3 + i % D];
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

int64_t bnm_align(int64_t x) { return (x + 255) / 256 * 256; }

int bnm_grid(int64_t centres) {
  const int64_t need = (centres + kBnmWaves - 1) / kBnmWaves;
  return static_cast<int>(need < kBnmMaxGrid ? (need > 0 ? need : 1) : kBnmMaxGrid);
}

// The tables: two layers (D, C1, C2) = (32, 32, 64) / (64, 64, 64), three layers (D, 16, 16, 32)
// with D = 0 / 3.
struct BnmTable {
  int nlayer, D, C1, C2, C3;
};
bool bnm_table(int nlayer, const int* chans, BnmTable* t) {
  if (!chans) return false;
  if (nlayer == 2) {
    const int D = chans[0] - 3;
    if (!((D == 32 && chans[1] == 32 && chans[2] == 64) || (D == 64 && chans[1] == 64 && chans[2] == 64))) return false;
    *t = BnmTable{2, D, chans[1], chans[2], 0};
    return true;
  }
  if (nlayer == 3) {
    const int D = chans[0] - 3;
    if (!((D == 0 || D == 3) && chans[1] == 16 && chans[2] == 16 && chans[3] == 32)) return false;
    *t = BnmTable{3, D, 16, 16, 32};
    return true;
  }
  return false;
}
int bnm_grads_floats(const BnmTable& t) {
  const int C0 = 3 + t.D;
  int n = t.C1 * C0 + t.C1 + t.C2 * t.C1 + t.C2;
  if (t.nlayer == 3) n += t.C3 * t.C2 + t.C3;
  return n;
}

// Workspace: per-wave partials | the reduction's slice sums | (two layers) dW1's xyz / bias sums
// (C1 x 4) and feature columns (C1 x D) | (backward) keys | gz1 rows | per-point sums G | segsum's own.
constexpr int kGtfBlocks = 512;
constexpr int kSumSlices = 64;
struct BnmWs {
  int64_t tmp, xb, fw, total;  // byte offsets; partials at 0
};
BnmWs bnm_ws_layout(int64_t centres, const BnmTable& t) {
  const int64_t nw = static_cast<int64_t>(bnm_grid(centres)) * kBnmWaves;
  const int64_t cmax = std::max(std::max(t.C1, t.C2), t.C3);
  int64_t b = nw * 2 * 2 * cmax * 8, pmax = 2 * cmax;
  if (t.nlayer == 3) {
    b = std::max<int64_t>(b, nw * bnm_grads_floats(t) * 4);
    pmax = std::max<int64_t>(pmax, bnm_grads_floats(t));
  } else {
    b = std::max<int64_t>(b, nw * (t.C2 * t.C1 + t.C2) * 4);
    b = std::max<int64_t>(b, nw * 4 * t.C1 * 4);
    b = std::max<int64_t>(b, static_cast<int64_t>(kGtfBlocks) * t.C1 * t.D * 4);
    pmax = std::max<int64_t>(std::max<int64_t>(pmax, t.C2 * t.C1 + t.C2), static_cast<int64_t>(t.C1) * t.D);
  }
  BnmWs w;
  w.tmp = bnm_align(b);
  w.xb = w.tmp + bnm_align(kSumSlices * pmax * 8);
  w.fw = w.xb + bnm_align(t.C1 * 4 * 4);
  w.total = w.fw + bnm_align(static_cast<int64_t>(t.C1) * t.D * 4);
  return w;
}
int64_t bnm_part_bytes(int64_t centres, const BnmTable& t) { return bnm_ws_layout(centres, t).total; }
int64_t bnm_feat_bytes(int64_t E, int64_t npts, int C1) {
  const int64_t seg = segment_sum_workspace_bytes(E, npts);
  return seg < 0 ? -1 : bnm_align(E * 4) + bnm_align(E * C1 * 4) + bnm_align(npts * C1 * 4) + seg;
}

template <int D, int C1, int C2, int PASS>
int bnm_launch(const BnmArgs& a, hipStream_t st) {
  const int grid = bnm_grid(static_cast<int64_t>(a.B) * a.S);
  hipLaunchKernelGGL((sa_bnm_kernel<D, C1, C2, PASS>), dim3(grid), dim3(kBnmThreads), 0, st, a);
  return launch_status("dvcp_sa_bnm_pass");
}
template <int D, int PASS>
int bnm3_launch(const BnmArgs& a, hipStream_t st) {
  const int grid = bnm_grid(static_cast<int64_t>(a.B) * a.S);
  hipLaunchKernelGGL((sa_bnm3_kernel<D, PASS>), dim3(grid), dim3(kBnmThreads), 0, st, a);
  return launch_status("dvcp_sa_bnm_pass");
}

// out[e] = sum of the nrows partial rows (P columns) in a fixed order: slice sums into the
// workspace's tmp area, then the slices in order.
template <typename PT, typename OT>
int bnm_reduce(const PT* part, int nrows, int P, OT* out, void* ws, int64_t tmp_off, hipStream_t st) {
  double* tmp = reinterpret_cast<double*>(static_cast<char*>(ws) + tmp_off);
  const int per = (nrows + kSumSlices - 1) / kSumSlices;
  const int ns = (nrows + per - 1) / per;
  hipLaunchKernelGGL((bnm_slice_kernel<PT>), dim3(ceil_div(P, 64), ns), dim3(1024), 0, st, part, nrows, P, per, tmp);
  hipLaunchKernelGGL((bnm_sum_kernel<double, OT>), dim3(ceil_div(P, 64)), dim3(1024), 0, st, tmp, ns, P, out);
  return launch_status("dvcp_sa_bnm_pass(sum)");
}
int bnm_sums(void* ws, int nw, int C, double* sums, int64_t tmp_off, hipStream_t st) {
  return bnm_reduce<double, double>(static_cast<const double*>(ws), 2 * nw, 2 * C, sums, ws, tmp_off, st);
}

// ABI pass codes: 1..3 statistics of layer l, 10 forward, 20 + l backward sums of layer l, 30 gradients
template <int D, int C1, int C2>
int bnm_pass2(int pass, BnmArgs a, void* ws, double* sums, float* grads, float* gfeat, hipStream_t st) {
  const int64_t centres = static_cast<int64_t>(a.B) * a.S;
  const int nw = bnm_grid(centres) * kBnmWaves;
  const BnmWs L = bnm_ws_layout(centres, BnmTable{2, D, C1, C2, 0});
  a.part = ws;
  if (pass == 1 || pass == 2 || pass == 21) {
    const int e = pass == 1 ? bnm_launch<D, C1, C2, kS1>(a, st)
                            : (pass == 2 ? bnm_launch<D, C1, C2, kS2>(a, st) : bnm_launch<D, C1, C2, kB1>(a, st));
    return e ? e : bnm_sums(ws, nw, pass == 2 ? C2 : C1, sums, L.tmp, st);
  }
  if (pass == 10) return bnm_launch<D, C1, C2, kFwd>(a, st);
  if (pass != 30) {
    set_error("dvcp_sa_bnm_pass: pass %d is not one of 1, 2, 10, 21, 30 for a two-layer table", pass);
    return DVCP_EINVAL;
  }
  // the gradients -- layer 2 (dW2 | db2); layer 1's xyz / bias columns and the per-entry gz1 rows;
  // their per-point segment sums G; dW1's feature columns G^T F; the feature gradient
  constexpr int C0 = 3 + D;
  constexpr int P1 = C1 * C0 + C1, P2 = C2 * C1 + C2;
  if (int e = bnm_launch<D, C1, C2, kB0A>(a, st)) return e;
  if (int e = bnm_reduce<float, float>(static_cast<const float*>(ws), nw, P2, grads + P1, ws, L.tmp, st)) return e;
  const int64_t E = centres * a.nsample, npts = static_cast<int64_t>(a.B) * a.N;
  char* w8 = static_cast<char*>(ws);
  float* xb = reinterpret_cast<float*>(w8 + L.xb);
  float* fw = reinterpret_cast<float*>(w8 + L.fw);
  char* fws = w8 + L.total;
  a.fkeys = reinterpret_cast<uint32_t*>(fws);
  a.frows = reinterpret_cast<float*>(fws + bnm_align(E * 4));
  float* G = reinterpret_cast<float*>(fws + bnm_align(E * 4) + bnm_align(E * C1 * 4));
  void* segws = fws + bnm_align(E * 4) + bnm_align(E * C1 * 4) + bnm_align(npts * C1 * 4);
  if (int e = bnm_launch<D, C1, C2, kB0B>(a, st)) return e;
  if (int e = bnm_reduce<float, float>(static_cast<const float*>(ws), nw, 4 * C1, xb, ws, L.tmp, st)) return e;
  if (int e = segment_sum(a.fkeys, a.frows, E, npts, C1, G, segws, st)) return e;
  const int64_t per = (npts + kGtfBlocks - 1) / kGtfBlocks;
  const int nblk = static_cast<int>((npts + per - 1) / per);
  hipLaunchKernelGGL((bnm_gtf_kernel<D, C1>), dim3(nblk), dim3(256), 0, st, G, a.feat, a.fb, a.fn, a.N, npts, per,
                     static_cast<float*>(ws));
  if (int e = bnm_reduce<float, float>(static_cast<const float*>(ws), nblk, C1 * D, fw, ws, L.tmp, st)) return e;
  hipLaunchKernelGGL((bnm_dw1_kernel<D, C1>), dim3(1), dim3(256), 0, st, xb, fw, grads);
  if (int e = launch_status("dvcp_sa_bnm_pass(dW1)")) return e;
  if (gfeat) {
    hipLaunchKernelGGL((bnm_feat_grad_kernel<D, C1>), dim3(ceil_div(npts * D, 256)), dim3(256), 0, st, G, a.pack,
                       npts, gfeat);
    return launch_status("dvcp_sa_bnm_pass(feat)");
  }
  return DVCP_OK;
}

template <int D>
int bnm_pass3(int pass, BnmArgs a, void* ws, double* sums, float* grads, hipStream_t st) {
  const int64_t centres = static_cast<int64_t>(a.B) * a.S;
  const int nw = bnm_grid(centres) * kBnmWaves;
  const BnmWs L = bnm_ws_layout(centres, BnmTable{3, D, 16, 16, 32});
  a.part = ws;
  int e = DVCP_OK, C = 16;
  switch (pass) {
    case 1: e = bnm3_launch<D, kS1>(a, st); break;
    case 2: e = bnm3_launch<D, kS2>(a, st); break;
    case 3: e = bnm3_launch<D, kS3>(a, st), C = 32; break;
    case 10: return bnm3_launch<D, kFwd>(a, st);
    case 21: e = bnm3_launch<D, kB1>(a, st); break;
    case 22: e = bnm3_launch<D, kB2>(a, st); break;
    case 30: {
      if (int e2 = bnm3_launch<D, kB0A>(a, st)) return e2;
      const int P = bnm_grads_floats(BnmTable{3, D, 16, 16, 32});
      return bnm_reduce<float, float>(static_cast<const float*>(ws), nw, P, grads, ws, L.tmp, st);
    }
    default:
      set_error("dvcp_sa_bnm_pass: pass %d is not one of 1, 2, 3, 10, 21, 22, 30 for a three-layer table", pass);
      return DVCP_EINVAL;
  }
  return e ? e : bnm_sums(ws, nw, C, sums, L.tmp, st);
}

}  // namespace
}  // namespace dvcp

extern "C" int dvcp_sa_bnm_supported(int nlayer, const int* chans) {
  dvcp::BnmTable t;
  return dvcp::bnm_table(nlayer, chans, &t) ? 1 : 0;
}

extern "C" int64_t dvcp_sa_bnm_workspace_bytes(int B, int S, int N, int nsample, int nlayer, const int* chans,
                                               int backward) {
  dvcp::BnmTable t;
  if (B < 0 || S < 0 || N < 0 || nsample < 0 || !dvcp::bnm_table(nlayer, chans, &t)) return -1;
  const int64_t centres = static_cast<int64_t>(B) * S;
  const int64_t b = dvcp::bnm_part_bytes(centres, t);
  if (!backward || t.nlayer == 3) return b;  // only the two-layer gradients need the feature part
  const int64_t f = dvcp::bnm_feat_bytes(centres * nsample, static_cast<int64_t>(B) * N, t.C1);
  return f < 0 ? -1 : b + f;
}

extern "C" int dvcp_sa_bnm_pre(const float* feat, int64_t fb, int64_t fn, int N, int B, int nlayer, const int* chans,
                               const float* pack, float* U, void* stream) {
  dvcp::BnmTable t;
  DVCP_REQUIRE(dvcp::bnm_table(nlayer, chans, &t) && t.nlayer == 2, "dvcp_sa_bnm_pre: not a two-layer table");
  DVCP_REQUIRE(feat && pack && U, "dvcp_sa_bnm_pre: null pointer");
  DVCP_REQUIRE(N >= 0 && B >= 0 && fb % 4 == 0 && fn % 4 == 0, "dvcp_sa_bnm_pre: bad sizes / strides");
  DVCP_REQUIRE(reinterpret_cast<uintptr_t>(feat) % 16 == 0, "dvcp_sa_bnm_pre: feature rows must be 16-byte aligned");
  const int64_t rows = static_cast<int64_t>(B) * N;
  if (rows == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (t.D == 32)
    hipLaunchKernelGGL((dvcp::bnm_pre_kernel<32, 32>), dim3(dvcp::ceil_div(rows, 256 / 8)), dim3(256), 0, st, feat, fb,
                       fn, N, B, pack, U);
  else
    hipLaunchKernelGGL((dvcp::bnm_pre_kernel<64, 64>), dim3(dvcp::ceil_div(rows, 256 / 16)), dim3(256), 0, st, feat,
                       fb, fn, N, B, pack, U);
  return dvcp::launch_status("dvcp_sa_bnm_pre");
}

extern "C" int dvcp_sa_bnm_pass(int pass, const float* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const float* ctr,
                                int64_t cb, int64_t cc, int64_t cn, int S, int B, const float* feat, int64_t fb,
                                int64_t fd, int64_t fn, int D, const int32_t* count, const int32_t* list, int nsample,
                                int nlayer, const int* chans, const float* pack, const float* U,
                                const float* grad_out, int32_t* arg, float* out, float* zbest, void* workspace,
                                double* sums, float* grads, float* grad_feat, void* stream) {
  dvcp::BnmTable t;
  DVCP_REQUIRE(dvcp::bnm_table(nlayer, chans, &t) && t.D == D, "dvcp_sa_bnm_pass: unsupported table");
  DVCP_REQUIRE(xyz && ctr && count && list && pack, "dvcp_sa_bnm_pass: null input");
  DVCP_REQUIRE(D == 0 || feat, "dvcp_sa_bnm_pass: D=%d but feat is NULL", D);
  DVCP_REQUIRE(t.nlayer == 3 || (U && fd == 1), "dvcp_sa_bnm_pass: two-layer tables need U and point-major rows");
  DVCP_REQUIRE(N > 0 && S >= 0 && B >= 0 && nsample > 0, "dvcp_sa_bnm_pass: bad sizes");
  DVCP_REQUIRE(static_cast<int64_t>(B) * S * nsample < (int64_t(1) << 31) &&
                   static_cast<int64_t>(B) * N < (int64_t(1) << 31),
               "dvcp_sa_bnm_pass: more than 2^31 entries / points");
  const bool stats = (pass >= 1 && pass <= t.nlayer) || (pass > 20 && pass < 20 + t.nlayer);
  DVCP_REQUIRE(stats || pass == 10 || pass == 30, "dvcp_sa_bnm_pass: bad pass %d", pass);
  DVCP_REQUIRE(!stats || sums, "dvcp_sa_bnm_pass: null sums");
  DVCP_REQUIRE(pass != 10 || (arg && out && zbest), "dvcp_sa_bnm_pass: null forward outputs");
  DVCP_REQUIRE(pass < 20 || (grad_out && arg && out), "dvcp_sa_bnm_pass: null gradient / routing");
  DVCP_REQUIRE(pass != 30 || grads, "dvcp_sa_bnm_pass: null grads");
  DVCP_REQUIRE(pass == 10 || workspace, "dvcp_sa_bnm_pass: null workspace");
  DVCP_REQUIRE(!grad_feat || t.nlayer == 2, "dvcp_sa_bnm_pass: no feature gradient for the three-layer table");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0 || S == 0) {
    const int cs[4] = {0, t.C1, t.C2, t.C3};
    if (stats) {
      const int C = cs[pass > 20 ? pass - 20 : pass];
      if (hipMemsetAsync(sums, 0, 2 * C * sizeof(double), st) != hipSuccess) return dvcp::launch_status("dvcp_sa_bnm");
    }
    if (pass == 30) {
      if (hipMemsetAsync(grads, 0, dvcp::bnm_grads_floats(t) * sizeof(float), st) != hipSuccess)
        return dvcp::launch_status("dvcp_sa_bnm");
      if (grad_feat && hipMemsetAsync(grad_feat, 0, static_cast<int64_t>(B) * N * D * sizeof(float), st) != hipSuccess)
        return dvcp::launch_status("dvcp_sa_bnm");
    }
    return DVCP_OK;
  }
  dvcp::BnmArgs a{xyz,   sb,   sc,   sn,  ctr,      cb,  cc,  cn,    S,       B,       N,      nsample, feat, fb,
                  fd,    fn,   count, list, pack,   U,   grad_out, arg, out, zbest, nullptr, nullptr, nullptr};
  if (t.nlayer == 3)
    return D == 0 ? dvcp::bnm_pass3<0>(pass, a, workspace, sums, grads, st)
                  : dvcp::bnm_pass3<3>(pass, a, workspace, sums, grads, st);
  if (D == 32) return dvcp::bnm_pass2<32, 32, 64>(pass, a, workspace, sums, grads, grad_feat, st);
  return dvcp::bnm_pass2<64, 64, 64>(pass, a, workspace, sums, grads, grad_feat, st);
}
