// cpg_bwd.hip -- backward of corresponding point generation (cpg.py:27-60) for training
// (train.py:121 loss.backward()), one 1024-thread workgroup per key point.
//
// Forward (cpg.hip): cost[f'][v] = (src[f'] - T[v*32 + f'])^2 (Q11 scramble: T[l] = tgt[f = l / C]
// [c = l % C]); h1 = conv1(cost) (32 -> 16), h2 = conv2(h1) (16 -> 4), lg = conv3(h2) (4 -> 1), all
// k3 p1 with no activations; w = softmax(lg); vcp = sum(w * cand) / sum(w).
// Backward, given dL/dvcp:
//   dL/dw_v   = sum_a g_a (cand_v,a / S - A_a / S^2)     (A = sum w cand, S = sum w)
//   dL/dlg_v  = w_v (dL/dw_v - sum_u w_u dL/dw_u)         (softmax)
//   conv k: dW[co][ci][t] = sum_v gout[co][v] in[ci][v + off_t];  db[co] = sum_v gout[co][v];
//           gin[ci][u]    = sum_co sum_t W[co][ci][t] gout[co][u - off_t]   (zero padding: taps
//           that leave the grid are skipped)
//   dL/dsrc[f'] = sum_v 2 (src[f'] - T) dL/dcost[f'][v];  dL/dT[l] = -2 (src[f'] - T) dL/dcost.
// The workgroup recomputes the forward activations (conv1 from the cost volume, one input
// channel at a time) and keeps them in LDS:
//   A (16 x C): h1, later dL/dh1;    W: dL/dlg and reduction scratch;
//   D (4 x C): the cost channel being processed, or h2 / dL/dh2.
// Convolution weights are read as wave-uniform scalar loads (SGPR operands), so the LDS traffic
// is one activation read per 16 (conv1 forward) or 32 (conv1 data backward) fmas.
// Parameter gradients are written per key point (fixed order, no atomics) and summed over key
// points by cpg_bwd_reduce_kernel in fp64.
#include "common.h"
#include "cpg_grid.h"

namespace dvcp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCbThreads = 1024;
constexpr int kCbMaxC = 1331;
constexpr int kCbA = 16 * kCbMaxC;
constexpr int kCbW = 16 * 32 * 27;
constexpr int kCbD = 4 * kCbMaxC;
constexpr int kCbV = (kCbMaxC + kCbThreads - 1) / kCbThreads;  // voxels per thread
// packed parameter layout (= cpg.packed_params()): W1, b1, W2, b2, W3, b3
constexpr int kCbOffB1 = 16 * 32 * 27;
constexpr int kCbOffW2 = kCbOffB1 + 16;
constexpr int kCbOffB2 = kCbOffW2 + 4 * 16 * 27;
constexpr int kCbOffW3 = kCbOffB2 + 4;
constexpr int kCbOffB3 = kCbOffW3 + 4 * 27;
constexpr int kCbParams = kCbOffB3 + 1;
static_assert(kCbA + kCbW + kCbD + 64 <= 160 * 1024 / 4, "LDS budget");
static_assert(kCbW + kCbD >= 8 * 13 * 13 * 13 + 1024 && kCbA >= kCbW && kCbW >= 2304 + 16 * 2 * 256,
              "conv1 MFMA staging: haloed 8-channel volume (+ partial sums) in Wr..D, W1 in A");

// tap t of a 3x3x3 kernel: (dz, dy, dx) = (t / 9 - 1, (t / 3) % 3 - 1, t % 3 - 1)
__device__ __forceinline__ int tap_off(int t, int G, int GG) {
  return (t / 9 - 1) * GG + ((t / 3) % 3 - 1) * G + (t % 3 - 1);
}

// bit t set when voxel (z, y, x) + tap t lies inside the G^3 grid
__device__ __forceinline__ uint32_t tap_mask(int z, int y, int x, int G) {
  uint32_t m = 0;
#pragma unroll
  for (int t = 0; t < 27; ++t) {
    const int zz = z + t / 9 - 1, yy = y + (t / 3) % 3 - 1, xx = x + t % 3 - 1;
    const bool ok = (static_cast<unsigned>(zz) < static_cast<unsigned>(G)) &
                    (static_cast<unsigned>(yy) < static_cast<unsigned>(G)) &
                    (static_cast<unsigned>(xx) < static_cast<unsigned>(G));
    m |= static_cast<uint32_t>(ok) << t;
  }
  return m;
}

// sum over output voxels v with z in [z0, z1) of go[v] * in[v + off_t], v + off_t inside the grid
__device__ __forceinline__ float wgrad_sum(const float* go, const float* in, int G, int GG, int t, int z0, int z1) {
  const int dz = t / 9 - 1, dy = (t / 3) % 3 - 1, dx = t % 3 - 1;
  const int zlo = max(z0, -dz), zhi = min(z1, G - dz);
  const int ylo = max(0, -dy), yhi = min(G, G - dy);
  const int xlo = max(0, -dx), xhi = min(G, G - dx);
  const int off = dz * GG + dy * G + dx;
  float acc = 0.f;
  for (int z = zlo; z < zhi; ++z)
    for (int y = ylo; y < yhi; ++y) {
      const int base = z * GG + y * G;
      for (int x = xlo; x < xhi; ++x) acc = __fmaf_rn(go[base + x], in[base + x + off], acc);
    }
  return acc;
}

__global__ __launch_bounds__(kCbThreads) void cpg_bwd_kernel(const float* __restrict__ src, const float* __restrict__ tgt,
                                                             int64_t t_p, int64_t t_f, int64_t t_c,
                                                             const float* __restrict__ cand, int G,
                                                             const float* __restrict__ params,
                                                             const float* __restrict__ gvcp, float* __restrict__ gsrc,
                                                             float* __restrict__ gtgt, float* __restrict__ gpart,
                                                             const float* __restrict__ wt) {
  __shared__ __attribute__((aligned(16))) float lds[kCbA + kCbW + kCbD];
  __shared__ float red[32];
  __shared__ float sv[32];
  float* A = lds;
  float* Wr = lds + kCbA;
  float* D = Wr + kCbW;
  const int p = blockIdx.x, tid = threadIdx.x;
  const int C = G * G * G, GG = G * G;
  const FastDiv dG(G), dGG(GG), dC(C);
  const float* P3 = params + kCbOffW3;
  // weight tables with the inner loop's index contiguous, so a tap's weights are one wide scalar
  // load (s_load_dwordx16) instead of 16-32 single ones (cpg_bwd_prep_kernel)
  const float* W1a = wt;                      // [ci][t][co]
  const float* W1b = W1a + kCbW;              // [co][t][ci]
  const float* W2a = W1b + kCbW;              // [ci][t][co4]
  const float* W2b = W2a + 4 * 16 * 27;       // [co4][t][ci]
  float* gp = gpart + static_cast<int64_t>(p) * kCbParams;
  const float* T = tgt + static_cast<int64_t>(p) * t_p;
  if (tid < 32) sv[tid] = src[static_cast<int64_t>(p) * 32 + tid];

  int vv[kCbV];
  bool vok[kCbV];
  uint32_t msk[kCbV];
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
    const int v = tid + k * kCbThreads;
    vok[k] = v < C;
    vv[k] = vok[k] ? v : 0;
    const uint32_t z = dGG.div(vv[k]), r = vv[k] - z * GG;
    const uint32_t y = dG.div(r), x = r - y * G;
    msk[k] = vok[k] ? tap_mask(z, y, x, G) : 0u;
  }
  // T[l] of the scrambled target block
  auto tval = [&](int l) -> float {
    const uint32_t f = dC.div(static_cast<uint32_t>(l));
    return T[static_cast<int64_t>(f) * t_f + static_cast<int64_t>(l - static_cast<int>(f) * C) * t_c];
  };

  // ---- forward: conv1 on the matrix cores, as cpg_kernel: an implicit GEMM on
  // v_mfma_f32_16x16x4_f32 over 8-channel haloed quarters of the cost volume (rows = 16-voxel
  // tiles, k = 4 input channels at one tap, columns = the 16 output channels).  LDS during this
  // phase: W1 [ci][t][co] in A, the haloed quarter from Wr on (8 x 13^3 floats, into D).
  float tpre[kCbV];
  {
    const int PG = G + 2, PGG = PG * PG, PV = PG * PGG;
    float* w1s = A;
    float* vol = Wr;
    for (int i = tid; i < kCbW; i += kCbThreads) w1s[i] = W1a[i];
    constexpr int kT = (kCbMaxC + 15) / 16, kW = kCbThreads / 64, kTW = (kT + kW - 1) / kW;
    const int lane = tid & 63, wave = tid >> 6, kg = lane >> 4, l16 = lane & 15;
    const int NT = (C + 15) / 16;
    int vx[kTW];
#pragma unroll
    for (int i = 0; i < kTW; ++i) {
      const int g = 16 * (wave + kW * i) + l16;
      vx[i] = cpg_halo(g < C ? g : 0, dG, dGG, PG, PGG);  // rows past C: voxel 0 (in-bounds taps, result unused)
    }
    f32x4 acc[kTW];
#pragma unroll
    for (int i = 0; i < kTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
      __syncthreads();
      for (int h = tid; h < 8 * PV; h += kCbThreads) vol[h] = 0.f;
      __syncthreads();
      for (int e = tid; e < 8 * C; e += kCbThreads) {
        const int c8 = static_cast<int>(dC.div(static_cast<uint32_t>(e))), v = e - c8 * C;
        const int ci = 8 * q + c8;
        const float d = sv[ci] - tval(v * 32 + ci);
        vol[c8 * PV + cpg_halo(v, dG, dGG, PG, PGG)] = d * d;
      }
      __syncthreads();
#pragma unroll 1
      for (int t = 0; t < 27; ++t) {
        const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
#pragma unroll
        for (int cg = 0; cg < 2; ++cg) {
          const int ci = 4 * cg + kg;
          const float bw = w1s[((8 * q + ci) * 27 + t) * 16 + l16];
          const float* vin = vol + ci * PV + off;
#pragma unroll
          for (int i = 0; i < kTW; ++i)
            if (wave + kW * i < NT) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(vin[vx[i]], bw, acc[i], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // W1 readers are done: h1 replaces it in A
    // register r of lane l: voxel 16 t + 4 (l >> 4) + r, output channel l & 15
#pragma unroll
    for (int i = 0; i < kTW; ++i) {
      const int t = wave + kW * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int g = 16 * t + 4 * kg + r;
        if (t < NT && g < C) A[l16 * C + g] = acc[i][r] + params[kCbOffB1 + l16];
      }
    }
    __syncthreads();
  }

  // ---- forward: conv2 -> D, conv3 -> logits ------------------------------------------------
  float h2[kCbV][4];
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
#pragma unroll
    for (int co = 0; co < 4; ++co) h2[k][co] = params[kCbOffB2 + co];
    if (!vok[k]) continue;
#pragma unroll 1
    for (int ci = 0; ci < 16; ++ci)
#pragma unroll 1
      for (int t = 0; t < 27; ++t) {
        if (!((msk[k] >> t) & 1u)) continue;
        const float c = A[ci * C + vv[k] + tap_off(t, G, GG)];
#pragma unroll
        for (int co = 0; co < 4; ++co) h2[k][co] = __fmaf_rn(W2a[(ci * 27 + t) * 4 + co], c, h2[k][co]);
      }
  }
#pragma unroll
  for (int k = 0; k < kCbV; ++k)
    if (vok[k])
#pragma unroll
      for (int co = 0; co < 4; ++co) D[co * C + vv[k]] = h2[k][co];
  __syncthreads();
  float lg[kCbV];
  float lmax = -__builtin_huge_valf();
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
    float a = 0.f;
    if (vok[k]) {
#pragma unroll 1
      for (int ci = 0; ci < 4; ++ci)
#pragma unroll 1
        for (int t = 0; t < 27; ++t)
          if ((msk[k] >> t) & 1u) a = __fmaf_rn(P3[ci * 27 + t], D[ci * C + vv[k] + tap_off(t, G, GG)], a);
      lmax = fmaxf(lmax, a + params[kCbOffB3]);
    }
    lg[k] = a + params[kCbOffB3];
  }

  // ---- softmax + weighted mean and their backward ------------------------------------------
  const float m = block_max_f(lmax, red);
  float w[kCbV];
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
    w[k] = vok[k] ? expf(lg[k] - m) : 0.f;
    se += w[k];
  }
  const float inv = 1.0f / block_sum(se, red);
  const float* cq = cand + static_cast<int64_t>(p) * C * 3;
  float sw = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
    w[k] *= inv;
    if (vok[k]) {
      sw += w[k];
      sx += w[k] * cq[vv[k] * 3 + 0];
      sy += w[k] * cq[vv[k] * 3 + 1];
      sz += w[k] * cq[vv[k] * 3 + 2];
    }
  }
  sw = block_sum(sw, red);
  sx = block_sum(sx, red);
  sy = block_sum(sy, red);
  sz = block_sum(sz, red);
  const float g0 = gvcp[static_cast<int64_t>(p) * 3 + 0], g1 = gvcp[static_cast<int64_t>(p) * 3 + 1],
              g2 = gvcp[static_cast<int64_t>(p) * 3 + 2];
  const float gS = -(g0 * sx + g1 * sy + g2 * sz) / (sw * sw);
  float gw[kCbV];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
    gw[k] = vok[k] ? (g0 * cq[vv[k] * 3 + 0] + g1 * cq[vv[k] * 3 + 1] + g2 * cq[vv[k] * 3 + 2]) / sw + gS : 0.f;
    dot += w[k] * gw[k];
  }
  dot = block_sum(dot, red);
  float* gl = Wr;
  float gls = 0.f;
#pragma unroll
  for (int k = 0; k < kCbV; ++k)
    if (vok[k]) {
      const float v = w[k] * (gw[k] - dot);
      gl[vv[k]] = v;
      gls += v;
    }
  gls = block_sum(gls, red);  // (its barriers also publish gl)
  if (tid == 0) gp[kCbOffB3] = gls;

  // ---- conv3 backward: dW3 (z-chunked), dL/dh2 -------------------------------------------
  float* scr = Wr + kCbMaxC + 16;
  {
    constexpr int kZc = 9;  // 108 taps x 9 z-chunks
    if (tid < 108 * kZc) {
      const int o = tid % 108, zc = tid / 108;
      const int ci = o / 27, t = o % 27;
      scr[tid] = wgrad_sum(gl, D + ci * C, G, GG, t, (zc * G) / kZc, ((zc + 1) * G) / kZc);
    }
    __syncthreads();
    if (tid < 108) {
      float s = 0.f;
      for (int zc = 0; zc < kZc; ++zc) s += scr[zc * 108 + tid];
      gp[kCbOffW3 + tid] = s;
    }
  }
  float gh2[kCbV][4];
#pragma unroll
  for (int k = 0; k < kCbV; ++k)
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      float a = 0.f;
      if (vok[k])
#pragma unroll 1
        for (int t = 0; t < 27; ++t)
          if ((msk[k] >> (26 - t)) & 1u) a = __fmaf_rn(P3[ci * 27 + t], gl[vv[k] - tap_off(t, G, GG)], a);
      gh2[k][ci] = a;
    }
  __syncthreads();  // h2 readers done
#pragma unroll
  for (int k = 0; k < kCbV; ++k)
    if (vok[k])
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) D[ci * C + vv[k]] = gh2[k][ci];
#pragma unroll
  for (int ci = 0; ci < 4; ++ci) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kCbV; ++k) s += gh2[k][ci];
    s = block_sum(s, red);
    if (tid == 0) gp[kCbOffB2 + ci] = s;
  }

  // ---- conv2 backward: dW2, dL/dh1 -----------------------------------------------------------
  for (int o = tid; o < 4 * 16 * 27; o += kCbThreads) {
    const int co = o / (16 * 27), r = o % (16 * 27), ci = r / 27, t = r % 27;
    gp[kCbOffW2 + o] = wgrad_sum(D + co * C, A + ci * C, G, GG, t, 0, G);
  }
  float gh1[kCbV][16];
#pragma unroll
  for (int k = 0; k < kCbV; ++k) {
#pragma unroll
    for (int ci = 0; ci < 16; ++ci) gh1[k][ci] = 0.f;
    if (!vok[k]) continue;
#pragma unroll 1
    for (int co = 0; co < 4; ++co)
#pragma unroll 1
      for (int t = 0; t < 27; ++t) {
        if (!((msk[k] >> (26 - t)) & 1u)) continue;
        const float g = D[co * C + vv[k] - tap_off(t, G, GG)];
#pragma unroll
        for (int ci = 0; ci < 16; ++ci) gh1[k][ci] = __fmaf_rn(W2b[(co * 27 + t) * 16 + ci], g, gh1[k][ci]);
      }
  }
  __syncthreads();  // h1 readers done
#pragma unroll
  for (int k = 0; k < kCbV; ++k)
    if (vok[k])
#pragma unroll
      for (int ci = 0; ci < 16; ++ci) A[ci * C + vv[k]] = gh1[k][ci];
#pragma unroll 1
  for (int ci = 0; ci < 16; ++ci) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kCbV; ++k) s += gh1[k][ci];
    s = block_sum(s, red);
    if (tid == 0) gp[kCbOffB1 + ci] = s;
  }

  // ---- conv1 backward, data side, on the matrix cores: dL/dcost[ci][u] = sum_co sum_t
  // W1[co][ci][t] dL/dh1[co][u - off_t], an implicit GEMM over haloed 8-channel halves of dL/dh1
  // (rows = 16-voxel tiles, k = 4 dL/dh1 channels at one tap, columns = 16 cost channels), then
  // the cost volume's own derivative: dL/dsrc[f'] = sum 2 (src - T) dL/dcost, dL/dT = -2 (src - T)
  // dL/dcost.  LDS: the haloed half from Wr on (into D), then 1024 partial sums of dL/dsrc.
  float* gT = gtgt + static_cast<int64_t>(p) * 32 * C;
  {
    const int PG = G + 2, PGG = PG * PG, PV = PG * PGG;
    float* vol = Wr;
    float* gpart_s = Wr + 8 * 13 * 13 * 13;  // [wave][kg][16]
    constexpr int kT = (kCbMaxC + 15) / 16, kW = kCbThreads / 64, kTW = (kT + kW - 1) / kW;
    const int lane = tid & 63, wave = tid >> 6, kg = lane >> 4, l16 = lane & 15;
    const int NT = (C + 15) / 16;
    int vx[kTW];
#pragma unroll
    for (int i = 0; i < kTW; ++i) {
      const int g = 16 * (wave + kW * i) + l16;
      vx[i] = cpg_halo(g < C ? g : 0, dG, dGG, PG, PGG);  // rows past C: voxel 0 (in-bounds taps, result unused)
    }
#pragma unroll 1
    for (int cb = 0; cb < 2; ++cb) {
      f32x4 acc[kTW];
#pragma unroll
      for (int i = 0; i < kTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int hc = 0; hc < 2; ++hc) {
        __syncthreads();
        for (int h = tid; h < 8 * PV; h += kCbThreads) vol[h] = 0.f;
        __syncthreads();
        for (int e = tid; e < 8 * C; e += kCbThreads) {
          const int c8 = static_cast<int>(dC.div(static_cast<uint32_t>(e))), v = e - c8 * C;
          vol[c8 * PV + cpg_halo(v, dG, dGG, PG, PGG)] = A[(8 * hc + c8) * C + v];
        }
        __syncthreads();
#pragma unroll 1
        for (int t = 0; t < 27; ++t) {
          const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
#pragma unroll
          for (int cg = 0; cg < 2; ++cg) {
            const int col = 4 * cg + kg;  // dL/dh1 channel within the half
            const float bw = W1b[((8 * hc + col) * 27 + t) * 32 + 16 * cb + l16];
            const float* vin = vol + col * PV - off;
#pragma unroll
            for (int i = 0; i < kTW; ++i)
              if (wave + kW * i < NT) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(vin[vx[i]], bw, acc[i], 0, 0, 0);
          }
        }
      }
      // register r of lane l: voxel 16 t + 4 (l >> 4) + r, cost channel 16 cb + (l & 15)
      const int ci = 16 * cb + l16;
      float gsl = 0.f;
#pragma unroll
      for (int i = 0; i < kTW; ++i) {
        const int t = wave + kW * i;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = 16 * t + 4 * kg + r;
          if (t < NT && u < C) {
            const int l = u * 32 + ci;
            const float d = sv[ci] - tval(l);
            const float gd = 2.0f * d * acc[i][r];
            gsl += gd;
            gT[l] = -gd;
          }
        }
      }
      gpart_s[(wave * 4 + kg) * 16 + l16] = gsl;
      __syncthreads();
      if (tid < 16) {  // fixed order over (wave, kg)
        float sum = 0.f;
        for (int w = 0; w < kW * 4; ++w) sum += gpart_s[w * 16 + tid];
        gsrc[static_cast<int64_t>(p) * 32 + 16 * cb + tid] = sum;
      }
    }
  }

  // ---- conv1 backward, weight side, on the matrix cores: for each cost channel ci,
  // dW1[co][ci][t] = sum_v dL/dh1[co][v] cost[ci][v + off_t] is a 16 x 27 (x voxels) GEMM:
  // rows = the 16 output channels, k = 4 voxels, columns = 16 taps (two blocks, 27 padded to 32).
  // The voxels are split over the 16 waves; their partial products are summed in wave order.
  // LDS: the haloed cost channel from Wr on, the partials after it.
  {
    const int PG = G + 2, PGG = PG * PG, PV = PG * PGG;
    float* ch = Wr;                  // haloed cost[ci] (<= 13^3)
    float* wpart = Wr + 2304;        // [wave][block][lane][4]: 16 x 2 x 256
    constexpr int kW = kCbThreads / 64;
    const int lane = tid & 63, wave = tid >> 6, kg = lane >> 4, l16 = lane & 15;
    // this wave's voxel range, 4-aligned
    const int nstep = (C + 3) / 4;
    const int s0 = (wave * nstep) / kW, s1 = ((wave + 1) * nstep) / kW;
    int toff[2];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int t = 16 * tb + l16;
      toff[tb] = t < 27 ? (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1) : 0;
    }
#pragma unroll
    for (int k = 0; k < kCbV; ++k) tpre[k] = vok[k] ? tval(vv[k] * 32) : 0.f;
    __syncthreads();
    for (int h = tid; h < PV; h += kCbThreads) ch[h] = 0.f;  // the zero border stays; interiors are rewritten
#pragma unroll 1
    for (int ci = 0; ci < 32; ++ci) {
      __syncthreads();  // previous channel's readers of ch / wpart are done (and the zeroing)
#pragma unroll
      for (int k = 0; k < kCbV; ++k) {
        const float d = sv[ci] - tpre[k];
        if (vok[k]) ch[cpg_halo(vv[k], dG, dGG, PG, PGG)] = d * d;
        if (ci + 1 < 32) tpre[k] = vok[k] ? tval(vv[k] * 32 + ci + 1) : 0.f;
      }
      __syncthreads();
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int st = s0; st < s1; ++st) {
        const int v = 4 * st + kg;  // this lane's voxel of the k-step
        const bool okv = v < C;
        const float a = okv ? A[l16 * C + v] : 0.f;  // dL/dh1[co = l16][v]
        const int hv = okv ? cpg_halo(v, dG, dGG, PG, PGG) : 0;
        const float b0 = okv ? ch[hv + toff[0]] : 0.f;
        const float b1 = (okv && l16 + 16 < 27) ? ch[hv + toff[1]] : 0.f;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b1, acc1, 0, 0, 0);
      }
      // register r of lane l: row co = 4 (l >> 4) + r, column tap 16 tb + (l & 15)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        wpart[((wave * 2 + 0) * 64 + lane) * 4 + r] = acc0[r];
        wpart[((wave * 2 + 1) * 64 + lane) * 4 + r] = acc1[r];
      }
      __syncthreads();
      if (tid < 432) {  // (co, t), summed over the waves in order
        const int co = tid / 27, t = tid % 27;
        const int tb = t >> 4, l = ((co >> 2) << 4) | (t & 15), r = co & 3;
        float sum = 0.f;
        for (int w = 0; w < kW; ++w) sum += wpart[((w * 2 + tb) * 64 + l) * 4 + r];
        gp[(co * 32 + ci) * 27 + t] = sum;
      }
    }
  }
}

__global__ void cpg_bwd_prep_kernel(const float* __restrict__ params, float* __restrict__ wt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < kCbW) {  // torch (co, ci, t)
    const int co = i / 864, ci = (i / 27) % 32, t = i % 27;
    wt[(ci * 27 + t) * 16 + co] = params[i];
    wt[kCbW + (co * 27 + t) * 32 + ci] = params[i];
  }
  if (i < 4 * 16 * 27) {
    const int co = i / 432, ci = (i / 27) % 16, t = i % 27;
    wt[2 * kCbW + (ci * 27 + t) * 4 + co] = params[kCbOffW2 + i];
    wt[2 * kCbW + 4 * 16 * 27 + (co * 27 + t) * 16 + ci] = params[kCbOffW2 + i];
  }
}
constexpr int kCbWt = 2 * kCbW + 2 * 4 * 16 * 27;

// grad[i] = sum over key points of part[p][i], in fp64, key-point order
__global__ void cpg_bwd_reduce_kernel(const float* __restrict__ part, int P, float* __restrict__ grad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kCbParams) return;
  double s = 0.0;
  for (int p = 0; p < P; ++p) s += static_cast<double>(part[static_cast<int64_t>(p) * kCbParams + i]);
  grad[i] = static_cast<float>(s);
}

}  // namespace dvcp

extern "C" int64_t dvcp_cpg_backward_workspace_bytes(int P) {
  return (static_cast<int64_t>(P > 0 ? P : 0) * dvcp::kCbParams + dvcp::kCbWt) * static_cast<int64_t>(sizeof(float));
}

extern "C" int dvcp_cpg_backward(const float* src, const float* tgt, int64_t t_p, int64_t t_f, int64_t t_c,
                                 const float* cand, int P, int G, const float* params, const float* grad_vcp,
                                 float* grad_src, float* grad_tgt, float* ws, float* grad_params, void* stream) {
  DVCP_REQUIRE(params && grad_params, "dvcp_cpg_backward: null pointer");
  DVCP_REQUIRE(P <= 0 || (src && tgt && cand && grad_vcp && grad_src && grad_tgt && ws),
               "dvcp_cpg_backward: null pointer");
  DVCP_REQUIRE(G >= 2 && G * G * G <= dvcp::kCbMaxC, "dvcp_cpg_backward: grid side G=%d unsupported (2..11)", G);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (P > 0) {
    float* wt = ws + static_cast<int64_t>(P) * dvcp::kCbParams;  // after the per-key-point partials
    hipLaunchKernelGGL(dvcp::cpg_bwd_prep_kernel, dim3(dvcp::ceil_div(dvcp::kCbW, 256)), dim3(256), 0, st, params, wt);
    hipLaunchKernelGGL(dvcp::cpg_bwd_kernel, dim3(P), dim3(dvcp::kCbThreads), 0, st, src, tgt, t_p, t_f, t_c, cand, G,
                       params, grad_vcp, grad_src, grad_tgt, ws, wt);
  }
  hipLaunchKernelGGL(dvcp::cpg_bwd_reduce_kernel, dim3(dvcp::ceil_div(dvcp::kCbParams, 256)), dim3(256), 0, st, ws,
                     P > 0 ? P : 0, grad_params);
  return dvcp::launch_status("dvcp_cpg_backward");
}
