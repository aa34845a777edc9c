// cpg.hip -- corresponding point generation (cpg.py:27-60), one workgroup per key point.
//
//   cost[f'][g] = (src[f'] - T[g*32 + f'])^2 where T is the reference's reshape of the
//                 permuted (32, C) target tensor (Q11: T[l] = tgt[f = l / C][c = l % C]);
//   Conv3d 32->16 -> 16->4 -> 4->1 (k3, p1, cross-correlation, no activations);
//   softmax over the C = G^3 logits; vcp = sum(w * cand) / sum(w).
//
// Plan (G <= 11, C <= 1331), one 1024-thread workgroup per key point: the key point's (C, 32)
// target block is loaded once into registers; the cost volume is built in LDS one 8-channel
// quarter at a time with a zero halo (13^3 cells, 70 KB) next to conv1's weights ([ci][tap][co],
// 55 KB); conv1 runs on the matrix cores (see below), accumulating the quarters in registers;
// its output (haloed) then replaces volume and weights in LDS for conv2 (VALU: its 4 output
// channels would fill a quarter of an MFMA tile); conv2's haloed output feeds conv3 (VALU,
// maskless), and the softmax and weighted mean finish in registers.
#include "common.h"
#include "cpg_grid.h"

namespace dvcp {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// DVCP_CPG_SPLIT3 (default): conv1 on the bf16 matrix cores (v_mfma_f32_16x16x32_bf16) with the
// fp32-accurate three-way split of sa_mlp_mfma.hip: each 8-channel quarter of the cost volume is
// stored in LDS as three bf16 piece images ([piece][cell][8 channels], 16 B per cell and piece,
// split once when the volume is built) and each quarter's weights as three B-fragment images; a
// k-step covers 4 taps x 8 channels (K = 32), 7 k-steps per quarter (taps 0..26 + one zero tap),
// six bf16 MFMAs (16 cycles) each, instead of 27 x 2 fp32 16x16x4 MFMAs (32 cycles) per quarter.
#ifndef DVCP_CPG_SPLIT3
#define DVCP_CPG_SPLIT3 1
#endif
// DVCP_CPG_C2: conv2's loop.  2 (default): (ci, kd) planes of scalar weights loaded at once, the
// second voxel chosen per wave; 1: the round-4 tap loop (a scalar load, a divergent branch and an
// LDS + scalar-cache wait per tap).  C3 (8 x 64 key points), A/B on one box: 0.249 / 0.250 ->
// 0.231 / 0.230 ms, conv2's phase 80.5k -> 52.5k clk and scratch 8 -> 0 B.  Measured and not kept:
// the next plane's weights prefetched into a second SGPR set (spills to VGPR lanes), and W2
// transposed into LDS read as broadcast float4 per tap (0.249 ms: the LDS pipe bounds it), the
// same with a register prefetch 0.287 ms (profiles/round5/r5v_cpg_ab.log, r5x_cpg_ab.log).
#ifndef DVCP_CPG_C2
#define DVCP_CPG_C2 2
#endif

// x = x0 + x1 + x2 exactly (bf16 pieces, as sa_mlp_mfma.hip's split3)
__device__ __forceinline__ void cpg_split3(float x, __bf16& p0, __bf16& p1, __bf16& p2) {
  p0 = static_cast<__bf16>(x);
  const float r1 = x - static_cast<float>(p0);
  p1 = static_cast<__bf16>(r1);
  p2 = static_cast<__bf16>(r1 - static_cast<float>(p1));
}
__device__ __forceinline__ f32x4 cpg_mfma_split3(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2,
                                                const bf16x8& b0, const bf16x8& b1, const bf16x8& b2, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
}

// DVCP_CPG_DIAG (diagnostic builds only): wave 0 of each workgroup records the shader clock at the
// phase boundaries and writes the deltas over the key point's softmax weights (tools/cpg_diag.py).
#ifdef DVCP_CPG_DIAG
#define DVCP_CPG_TICK(k) \
  if (tid == 0) dg[k] = __builtin_readcyclecounter();
#else
#define DVCP_CPG_TICK(k)
#endif

constexpr int kCpgThreads = 1024;  // 16 waves: four per SIMD (LDS allows one workgroup per CU)
constexpr int kCpgMaxC = 1331;
constexpr int kCpgMaxG = 11;
constexpr int kCpgV = (kCpgMaxC + kCpgThreads - 1) / kCpgThreads;  // voxels per thread (conv2/3)
constexpr int kCpgPV = (kCpgMaxG + 2) * (kCpgMaxG + 2) * (kCpgMaxG + 2);  // haloed voxels (13^3)
constexpr int kCpgQ = 8;                                                  // channels per quarter
constexpr int kCpgVolF = kCpgQ * kCpgPV;                                  // haloed quarter volume
constexpr int kCpgW1F = 32 * 27 * 16;
constexpr int kCpgBigF = 16 * kCpgPV;  // quarter volume + conv1 weights, later haloed conv1 / conv2 outputs
constexpr int kCpgE = (32 * kCpgMaxC + kCpgThreads - 1) / kCpgThreads;  // target values per thread
static_assert(kCpgVolF + kCpgW1F <= kCpgBigF, "quarter volume + conv1 weights must fit the area");

// Each 8-channel quarter of the cost volume takes the target values l = 32 g + f' with f' in the
// quarter (Q11: l = f C + c).  QBAL (every residue c mod 32 has exactly 8 channels f per quarter,
// cpg_balanced(C): G = 11 and G = 6, the forward's grids): each thread loads, per quarter, the
// values of that quarter (wave w, step u: rows c = 8 (16 u + w) + lane / 8, the (lane % 8)-th f of
// the row in the quarter), so every lane builds cost cells in every quarter; otherwise a thread's
// values all fall in one quarter (their l mod 32 is the same) and three quarters of the lanes idle
// through each quarter's build.
__host__ __device__ inline bool cpg_balanced(int C) {
  const int m = C & 31;
  for (int cr = 0; cr < 32; ++cr) {
    int n[4] = {0, 0, 0, 0};
    for (int f = 0; f < 32; ++f) ++n[((m * f + cr) & 31) >> 3];
    if (n[0] != 8 || n[1] != 8 || n[2] != 8 || n[3] != 8) return false;
  }
  return true;
}
constexpr int kCpgBalU = (kCpgMaxC + 127) / 128;  // QBAL load steps (128 rows per step)

template <bool QBAL>
__global__ __launch_bounds__(kCpgThreads) void cpg_kernel(const float* __restrict__ src, const float* __restrict__ tgt,
                                                          int64_t t_p, int64_t t_f, int64_t t_c,
                                                          const float* __restrict__ cand, int G,
                                                          const float* __restrict__ params, float* __restrict__ vcp,
                                                          float* __restrict__ weight) {
  __shared__ __attribute__((aligned(16))) float big[kCpgBigF];
  __shared__ float w3[4 * 27];
  __shared__ float bias[16 + 4 + 1];
  __shared__ float sv[32];
  __shared__ float red[32];
#if !DVCP_CPG_SPLIT3
  float* vol = big;            // conv1 input: a haloed 8-channel quarter of the cost volume
  float* w1 = big + kCpgVolF;  // conv1 W [ci][tap][co]
#endif
  float* out1 = big;           // after conv1: its output, haloed [co][cell] (16 x PV)
  float* out2 = big;           // after conv2: its output, haloed [co][cell] (4 x PV)

  const int p = blockIdx.x, tid = threadIdx.x;
#ifdef DVCP_CPG_DIAG
  uint64_t dg[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) dg[i] = 0;
#endif
  DVCP_CPG_TICK(0)
  const int C = G * G * G, GG = G * G;
  const int PG = G + 2, PGG = PG * PG, PV = PG * PGG;
  const FastDiv dG(G), dGG(GG);
  const float* P1 = params;
  const float* P2 = P1 + 16 * 32 * 27 + 16;
  const float* P3 = P2 + 4 * 16 * 27 + 4;
  // the whole (C, 32) target block of this key point, coalesced, all loads in flight
  const float* T = tgt + static_cast<int64_t>(p) * t_p;
  __shared__ uint8_t fsel[32][4][8];  // QBAL: the j-th channel f of residue c mod 32 in quarter q
  constexpr int kTv = QBAL ? 4 * kCpgBalU : kCpgE;
  float tv[kTv];
  if constexpr (QBAL) {
    if (tid < 128) {
      const int cr = tid >> 2, q = tid & 3, m = C & 31;
      int j = 0;
      for (int f = 0; f < 32; ++f)
        if ((((m * f + cr) & 31) >> 3) == q) fsel[cr][q][j++] = static_cast<uint8_t>(f);
    }
    __syncthreads();
    const int wv = tid >> 6, ln = tid & 63;
#pragma unroll
    for (int u = 0; u < kCpgBalU; ++u) {
      const int c = 8 * (16 * u + wv) + (ln >> 3);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = fsel[c & 31][q][ln & 7];
        tv[q * kCpgBalU + u] = c < C ? T[f * t_f + c * t_c] : 0.f;
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < kCpgE; ++u) {
      const int e = u * kCpgThreads + tid;  // memory order (c, f)
      tv[u] = e < 32 * C ? T[(e % 32) * t_f + (e / 32) * t_c] : 0.f;
    }
  }
#if !DVCP_CPG_SPLIT3
#pragma unroll 6
  for (int i = tid; i < 16 * 32 * 27; i += kCpgThreads) {  // torch (co, ci, kd, kh, kw)
    const int co = i / (32 * 27), r = i % (32 * 27);
    w1[r * 16 + co] = P1[i];
  }
#endif
  if (tid < 4 * 27) w3[tid] = P3[tid];
  if (tid < 16) bias[tid] = P1[16 * 32 * 27 + tid];
  if (tid < 4) bias[16 + tid] = P2[4 * 16 * 27 + tid];
  if (tid == 0) bias[20] = P3[4 * 27];
  if (tid < 32) sv[tid] = src[static_cast<int64_t>(p) * 32 + tid];

  DVCP_CPG_TICK(1)
  // per-thread voxels (conv3, softmax)
  int gv[kCpgV];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) gv[v] = tid + v * kCpgThreads;

  // conv1 (32 -> 16, k3) as an implicit GEMM on v_mfma_f32_16x16x4_f32: rows = 16-voxel tiles,
  // k = 4 input channels at one tap, columns = the 16 output channels.  Wave w owns tiles
  // w, w + 8, ... with their accumulators in registers: each k-step is one B fragment (weights)
  // and up to kTW independent MFMAs.  The input is haloed (zero border), so a tap is a constant
  // address shift and needs no mask; lane reads voxel 16 t + (lane & 15), channel 4 cg + (lane >> 4).
  constexpr int kT = (kCpgMaxC + 15) / 16;          // voxel tiles at C = 1331
  constexpr int kW = kCpgThreads / 64;
  constexpr int kTW = (kT + kW - 1) / kW;           // per wave
  const int lane = tid & 63, wave = tid >> 6, kg = lane >> 4, l16 = lane & 15;
  const int NT = (C + 15) / 16;
  int vx[kTW];  // haloed address of the lane's voxel per tile (voxel 0's cell past the end: every
                // tap of a padding row stays inside the volume; its output row is discarded)
#pragma unroll
  for (int i = 0; i < kTW; ++i) {
    const int g = 16 * (wave + kW * i) + l16;
    vx[i] = cpg_halo(g < C ? g : 0, dG, dGG, PG, PGG);
  }
  f32x4 acc[kTW];
#pragma unroll
  for (int i = 0; i < kTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

#if DVCP_CPG_SPLIT3
  {
    uint4* vsp = reinterpret_cast<uint4*>(big);                    // [piece][cell]: 8 bf16 channels
    uint4* w1p = vsp + 3 * PV;                                     // [k-step][piece][lane]
    static_assert(3 * kCpgPV * 16 + 7 * 3 * 64 * 16 <= kCpgBigF * 4, "split images must fit the area");
#pragma unroll 1
    for (int q = 0; q < 32 / kCpgQ; ++q) {
      __syncthreads();
      DVCP_CPG_TICK(2 + 3 * q)
      for (int i = tid; i < 3 * PV; i += kCpgThreads) vsp[i] = make_uint4(0u, 0u, 0u, 0u);
      // this quarter's conv1 weights: k-step s, lane (co = l & 15, tap 4 s + (l >> 4)), channel j
      for (int i = tid; i < 7 * 64; i += kCpgThreads) {
        const int l = i & 63, st = i >> 6, co = l & 15, tap = 4 * st + (l >> 4);
        bf16x8 b0, b1, b2;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float w = tap < 27 ? P1[(co * 32 + kCpgQ * q + jj) * 27 + tap] : 0.0f;
          __bf16 x0, x1, x2;
          cpg_split3(w, x0, x1, x2);
          b0[jj] = x0;
          b1[jj] = x1;
          b2[jj] = x2;
        }
        w1p[(st * 3 + 0) * 64 + l] = __builtin_bit_cast(uint4, b0);
        w1p[(st * 3 + 1) * 64 + l] = __builtin_bit_cast(uint4, b1);
        w1p[(st * 3 + 2) * 64 + l] = __builtin_bit_cast(uint4, b2);
      }
      __syncthreads();
      DVCP_CPG_TICK(3 + 3 * q)
      // cost volume quarter as bf16 pieces (see the fp32 path below for the Q11 index map)
      int zo = 0;
      asm volatile("" : "+v"(zo));
      uint16_t* vh = reinterpret_cast<uint16_t*>(vsp);
      auto put = [&](int l, float t) {  // cost cell of target value l (Q11), as three bf16 pieces
        const int g = l >> 5, fp = l & 31;
        const float d = sv[fp] - t;
        __bf16 x0, x1, x2;
        cpg_split3(d * d, x0, x1, x2);
        const int c8 = cpg_halo(g, dG, dGG, PG, PGG) * 8 + (fp & 7);
        vh[c8] = __builtin_bit_cast(uint16_t, x0);
        vh[8 * PV + c8] = __builtin_bit_cast(uint16_t, x1);
        vh[16 * PV + c8] = __builtin_bit_cast(uint16_t, x2);
      };
      if constexpr (QBAL) {
        // this quarter's values, one per step, every lane (no divergence but the tail rows)
        const int wv = tid >> 6, ln = tid & 63;
#pragma unroll
        for (int u = 0; u < kCpgBalU; ++u) {
          const int c = 8 * (16 * u + wv) + (ln >> 3) + zo;
          if (c < C) {
            const int f = fsel[c & 31][q][ln & 7];
            float t = tv[0];
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) t = qq == q ? tv[qq * kCpgBalU + u] : t;  // (q is uniform)
            put(f * C + c, t);
          }
        }
      } else {
        const int f0 = tid & 31;
        const int l0 = f0 * C + (tid >> 5) + zo;
#pragma unroll
        for (int u = 0; u < kCpgE; ++u) {
          const int e = u * kCpgThreads + tid;
          const int l = l0 + (kCpgThreads / 32) * u;
          if (e < 32 * C && ((l & 31) >> 3) == q) put(l, tv[u]);
        }
      }
      __syncthreads();
      DVCP_CPG_TICK(4 + 3 * q)
#pragma unroll 1
      for (int st = 0; st < 7; ++st) {
        // lane's tap 4 st + kg (tap 27: zero weights, any in-range cell)
        const int tap = 4 * st + kg;
        const int off = tap < 27 ? (tap / 9 - 1) * PGG + ((tap / 3) % 3 - 1) * PG + (tap % 3 - 1) : 0;
        const bf16x8 b0 = __builtin_bit_cast(bf16x8, w1p[(st * 3 + 0) * 64 + lane + zo]);
        const bf16x8 b1 = __builtin_bit_cast(bf16x8, w1p[(st * 3 + 1) * 64 + lane + zo]);
        const bf16x8 b2 = __builtin_bit_cast(bf16x8, w1p[(st * 3 + 2) * 64 + lane + zo]);
#pragma unroll
        for (int i = 0; i < kTW; ++i)
          if (wave + kW * i < NT) {  // wave-uniform
            const int cell = vx[i] + off;
            const bf16x8 a0 = __builtin_bit_cast(bf16x8, vsp[cell]);
            const bf16x8 a1 = __builtin_bit_cast(bf16x8, vsp[PV + cell]);
            const bf16x8 a2 = __builtin_bit_cast(bf16x8, vsp[2 * PV + cell]);
            acc[i] = cpg_mfma_split3(a0, a1, a2, b0, b1, b2, acc[i]);
          }
      }
    }
  }
#else
#pragma unroll 1
  for (int q = 0; q < 32 / kCpgQ; ++q) {
    __syncthreads();
    for (int i = tid; i < kCpgQ * PV; i += kCpgThreads) vol[i] = 0.f;
    __syncthreads();
    // cost volume quarter: channels f' in [8q, 8q + 8) of cost[f'][g] = (src[f'] - T[l])^2,
    // l = g*32 + f' = f*C + c (the reference's reshape, Q11).  (The opaque zero keeps the
    // compiler from hoisting 84 addresses per thread out of the quarter loop into registers.)
    int zo = 0;
    asm volatile("" : "+v"(zo));
    // element e = u*kCpgThreads + tid of the block is (c = e / 32, f = e % 32): f is fixed per
    // thread (kCpgThreads % 32 == 0) and c advances by kCpgThreads / 32 per u, and so does l = f*C + c.
    const int f0 = tid & 31;
    const int l0 = f0 * C + (tid >> 5) + zo;
#pragma unroll
    for (int u = 0; u < kCpgE; ++u) {
      const int e = u * kCpgThreads + tid;
      const int l = l0 + (kCpgThreads / 32) * u;
      const int g = l >> 5, fp = l & 31;
      if (e < 32 * C && (fp >> 3) == q) {
        const float d = sv[fp] - tv[u];
        vol[(fp & 7) * PV + cpg_halo(g, dG, dGG, PG, PGG)] = d * d;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int t = 0; t < 27; ++t) {
      const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
#pragma unroll
      for (int cg = 0; cg < kCpgQ / 4; ++cg) {
        const int ci = 4 * cg + kg;  // channel within the quarter
        const float bw = w1[((kCpgQ * q + ci) * 27 + t) * 16 + l16];
        const float* vin = vol + ci * PV + off;
#pragma unroll
        for (int i = 0; i < kTW; ++i)
          if (wave + kW * i < NT)  // wave-uniform
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(vin[vx[i]], bw, acc[i], 0, 0, 0);
      }
    }
  }
#endif
  __syncthreads();
  DVCP_CPG_TICK(14)
  // conv1 output -> out1 (haloed, zero border); accumulator register r of lane l is voxel
  // 16 t + 4 (l >> 4) + r, output channel l & 15
  for (int i = tid; i < 16 * PV; i += kCpgThreads) out1[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kTW; ++i) {
    const int t = wave + kW * i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int g = 16 * t + 4 * kg + r;
      if (t < NT && g < C) out1[l16 * PV + cpg_halo(g, dG, dGG, PG, PGG)] = acc[i][r] + bias[l16];
    }
  }
  __syncthreads();

  // conv2 (16 -> 4) on VALU, one voxel per thread: a 16-column MFMA tile would leave 12 of its
  // 16 output columns empty (4x the MFMA time of the useful work).
  DVCP_CPG_TICK(15)
  int hv[kCpgV];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) hv[v] = cpg_halo(gv[v] < C ? gv[v] : 0, dG, dGG, PG, PGG);
  float o2[kCpgV][4];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
#pragma unroll
    for (int co = 0; co < 4; ++co) o2[v][co] = 0.f;
#if DVCP_CPG_C2 == 2
  // The 48 (ci, kd) planes in turn; a plane's 36 weights W2[co][ci][kd][.][.] (9 contiguous floats
  // per co) are loaded at once (four s_load_dwordx8 + four dwords), one scalar-cache wait per plane
  // instead of one per tap.  A wave runs its second voxel (tid + 1024 < C: waves 0..4 at C = 1331)
  // only when some lane has one -- a wave-uniform choice outside the loop, no branch per tap.
  static_assert(kCpgV == 2, "conv2 plane loop: two voxels per thread at most");
  {
    const int hv0 = hv[0], hv1 = hv[1];
    auto planes = [&](auto two) {
      constexpr bool T2 = decltype(two)::value;
      float w[4][9];
      auto loadw = [&](int pl, float (&wt)[4][9]) {  // pl = 3 ci + kd
#pragma unroll
        for (int co = 0; co < 4; ++co)
#pragma unroll
          for (int t = 0; t < 9; ++t) wt[co][t] = P2[co * 16 * 27 + 9 * pl + t];
      };
      auto plane = [&](int pl, const float (&wt)[4][9]) {
        const int ci = pl / 3, kd = pl - 3 * ci;
        const float* xin = out1 + ci * PV + (kd - 1) * PGG;
#pragma unroll
        for (int t9 = 0; t9 < 9; ++t9) {
          const int off = (t9 / 3 - 1) * PG + (t9 % 3 - 1);
          const float xa = xin[hv0 + off];
#pragma unroll
          for (int co = 0; co < 4; ++co) o2[0][co] = __fmaf_rn(wt[co][t9], xa, o2[0][co]);
          if constexpr (T2) {
            const float xb = xin[hv1 + off];
#pragma unroll
            for (int co = 0; co < 4; ++co) o2[1][co] = __fmaf_rn(wt[co][t9], xb, o2[1][co]);
          }
        }
      };
#pragma unroll 1
      for (int pl = 0; pl < 48; ++pl) {
        loadw(pl, w);
        plane(pl, w);
      }
    };
    if (__builtin_amdgcn_readfirstlane(tid & ~63) + kCpgThreads < C)
      planes(std::true_type{});
    else
      planes(std::false_type{});
  }
#else
  // W2[co][ci][tap] comes through the scalar cache (wave-uniform), one tap plane (4 x 9 weights)
  // at a time.
#pragma unroll 1
  for (int ci = 0; ci < 16; ++ci) {
    const float* xin = out1 + ci * PV;
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      // (an opaque zero ordered after the running sums keeps all 108 weights of the channel from
      // being loaded into SGPRs at once)
      int zw = 0;
      asm volatile("" : "+s"(zw) : "v"(o2[0][0]));
      const float* w2c = P2 + ci * 27 + 9 * kd + zw;
#pragma unroll
      for (int t9 = 0; t9 < 9; ++t9) {
        const int t = 9 * kd + t9;
        const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
#pragma unroll
        for (int v = 0; v < kCpgV; ++v) {
          if (v == 0 || gv[v] < C) {  // (v = 0: every thread, C >= 1024 or a clamped in-range cell)
            const float x = xin[hv[v] + off];
#pragma unroll
            for (int co = 0; co < 4; ++co) o2[v][co] = __fmaf_rn(w2c[co * 16 * 27 + t9], x, o2[v][co]);
          }
        }
      }
    }
  }
#endif
  __syncthreads();  // every conv1 output read; out2 overwrites them
#ifdef DVCP_CPG_DIAG
  uint64_t dg_c2 = __builtin_readcyclecounter();
#endif
  for (int i = tid; i < 4 * PV; i += kCpgThreads) out2[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
    if (gv[v] < C)
#pragma unroll
      for (int co = 0; co < 4; ++co) out2[co * PV + hv[v]] = o2[v][co] + bias[16 + co];
  __syncthreads();

  // conv3: 4 -> 1, one voxel per thread (haloed input: no masks)
  float lg[kCpgV];
  float lmax = -__builtin_huge_valf();
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) {
    float a = 0.f;
#pragma unroll
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
        a = __fmaf_rn(w3[ci * 27 + t], out2[ci * PV + hv[v] + off], a);
      }
    lg[v] = a + bias[20];
    if (gv[v] < C) lmax = fmaxf(lmax, lg[v]);
  }

  // softmax over C (torch: exp(x - max), sum, multiply by 1/sum) and the weighted mean
  const float m = block_max_f(lmax, red);
  float e[kCpgV];
  float se = 0.f;
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) {
    e[v] = gv[v] < C ? expf(lg[v] - m) : 0.f;
    se += e[v];
  }
  const float sum = block_sum(se, red);
  const float inv = 1.0f / sum;
  const float* cq = cand + static_cast<int64_t>(p) * C * 3;
  float sw = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) {
    if (gv[v] < C) {
      const float w = e[v] * inv;
      if (weight) weight[static_cast<int64_t>(p) * C + gv[v]] = w;
      sw += w;
      sx += w * cq[gv[v] * 3 + 0];
      sy += w * cq[gv[v] * 3 + 1];
      sz += w * cq[gv[v] * 3 + 2];
    }
  }
  sw = block_sum(sw, red);
  sx = block_sum(sx, red);
  sy = block_sum(sy, red);
  sz = block_sum(sz, red);
#ifdef DVCP_CPG_DIAG
  if (tid == 0 && weight) {  // phase deltas: [load, q0 zero, q0 build, q0 mfma, ..., out1, conv2, rest]
    const uint64_t end = __builtin_readcyclecounter();
    float* o = weight + static_cast<int64_t>(p) * C;
    o[0] = static_cast<float>(dg[1] - dg[0]);
    for (int q = 0; q < 4; ++q) {
      o[1 + 3 * q] = static_cast<float>(dg[3 + 3 * q] - dg[2 + 3 * q]);
      o[2 + 3 * q] = static_cast<float>(dg[4 + 3 * q] - dg[3 + 3 * q]);
      o[3 + 3 * q] = static_cast<float>((q < 3 ? dg[5 + 3 * q] : dg[14]) - dg[4 + 3 * q]);
    }
    o[13] = static_cast<float>(dg[15] - dg[14]);
    o[14] = static_cast<float>(dg_c2 - dg[15]);
    o[15] = static_cast<float>(end - dg_c2);
    o[16] = static_cast<float>(end - dg[0]);
  }
#endif
  if (tid == 0) {
    vcp[static_cast<int64_t>(p) * 3 + 0] = sx / sw;
    vcp[static_cast<int64_t>(p) * 3 + 1] = sy / sw;
    vcp[static_cast<int64_t>(p) * 3 + 2] = sz / sw;
  }
}

}  // namespace dvcp

extern "C" int dvcp_cpg(const float* src, const float* tgt, int64_t t_p, int64_t t_f, int64_t t_c, const float* cand,
                        int P, int G, const float* params, float* vcp, float* weight, void* stream) {
  DVCP_REQUIRE(src && tgt && cand && params && vcp, "dvcp_cpg: null pointer");
  DVCP_REQUIRE(G >= 1 && G * G * G <= dvcp::kCpgMaxC, "dvcp_cpg: grid side G=%d unsupported (C <= 1331)", G);
  if (P <= 0) return DVCP_OK;
  if (dvcp::cpg_balanced(G * G * G))
    hipLaunchKernelGGL(dvcp::cpg_kernel<true>, dim3(P), dim3(dvcp::kCpgThreads), 0, static_cast<hipStream_t>(stream),
                       src, tgt, t_p, t_f, t_c, cand, G, params, vcp, weight);
  else
    hipLaunchKernelGGL(dvcp::cpg_kernel<false>, dim3(P), dim3(dvcp::kCpgThreads), 0, static_cast<hipStream_t>(stream),
                       src, tgt, t_p, t_f, t_c, cand, G, params, vcp, weight);
  return dvcp::launch_status("dvcp_cpg");
}
