// cpg.hip -- corresponding point generation (cpg.py:27-60), one workgroup per key point.
//
//   cost[f'][g] = (src[f'] - T[g*32 + f'])^2 where T is the reference's reshape of the
//                 permuted (32, C) target tensor (Q11: T[l] = tgt[f = l / C][c = l % C]);
//   Conv3d 32->16 -> 16->4 -> 4->1 (k3, p1, cross-correlation, no activations);
//   softmax over the C = G^3 logits; vcp = sum(w * cand) / sum(w).
//
// Plan (G <= 11, C <= 1331), one 1024-thread workgroup per key point, 71 KB of LDS (so other
// kernels' workgroups share the CU while it runs): the key point's (C, 32) target block is loaded
// once into registers; the cost volume is built in LDS one 4-channel eighth at a time with a
// zero halo (13^3 cells, 35 KB) next to that eighth's conv1 weights (7 KB); conv1 runs on the
// matrix cores (see below), accumulating the eighths in registers; its 16 output channels then go
// through LDS in two haloed 8-channel halves (70 KB), each consumed by conv2 (16 -> 4) on VALU
// with the weights as wave-uniform scalar loads (the 4 output channels would fill a quarter of
// an MFMA tile); conv2's haloed output feeds conv3 (VALU, maskless), and the softmax and weighted
// mean finish in registers.
#include "common.h"
#include "cpg_grid.h"

namespace dvcp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCpgThreads = 1024;  // 16 waves: four per SIMD
constexpr int kCpgMaxC = 1331;
constexpr int kCpgMaxG = 11;
constexpr int kCpgV = (kCpgMaxC + kCpgThreads - 1) / kCpgThreads;  // voxels per thread (conv2/3)
constexpr int kCpgPV = (kCpgMaxG + 2) * (kCpgMaxG + 2) * (kCpgMaxG + 2);  // haloed voxels (13^3)
constexpr int kCpgQ = 4;                                                  // channels per conv1 round
constexpr int kCpgVolF = kCpgQ * kCpgPV;                                  // haloed round volume
constexpr int kCpgW1F = kCpgQ * 27 * 16;                                  // the round's conv1 weights
constexpr int kCpgHalf = 8;                                               // conv1 outputs per conv2 pass
constexpr int kCpgBigF = kCpgHalf * kCpgPV;  // round volume + weights, later a conv1 half / conv2 output
constexpr int kCpgE = (32 * kCpgMaxC + kCpgThreads - 1) / kCpgThreads;  // target values per thread
static_assert(kCpgVolF + kCpgW1F <= kCpgBigF, "round volume + conv1 weights must fit the area");

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
  float* vol = big;            // conv1 input: a haloed 4-channel eighth of the cost volume
  float* w1 = big + kCpgVolF;  // that eighth's conv1 W [ci][tap][co]
  float* out1 = big;           // after conv1: half of its output, haloed [co][cell] (8 x PV)
  float* out2 = big;           // after conv2: its output, haloed [co][cell] (4 x PV)

  const int p = blockIdx.x, tid = threadIdx.x;
  const int C = G * G * G, GG = G * G;
  const int PG = G + 2, PGG = PG * PG, PV = PG * PGG;
  const FastDiv dG(G), dGG(GG);
  const float* P1 = params;
  const float* P2 = P1 + 16 * 32 * 27 + 16;
  const float* P3 = P2 + 4 * 16 * 27 + 4;
  // the whole (C, 32) target block of this key point, coalesced, all loads in flight
  const float* T = tgt + static_cast<int64_t>(p) * t_p;
  float tv[kCpgE];
#pragma unroll
  for (int u = 0; u < kCpgE; ++u) {
    const int e = u * kCpgThreads + tid;  // memory order (c, f)
    tv[u] = e < 32 * C ? T[(e % 32) * t_f + (e / 32) * t_c] : 0.f;
  }
  for (int i = tid; i < kCpgVolF; i += kCpgThreads) vol[i] = 0.f;  // the halo stays zero
  if (tid < 4 * 27) w3[tid] = P3[tid];
  if (tid < 16) bias[tid] = P1[16 * 32 * 27 + tid];
  if (tid < 4) bias[16 + tid] = P2[4 * 16 * 27 + tid];
  if (tid == 0) bias[20] = P3[4 * 27];
  if (tid < 32) sv[tid] = src[static_cast<int64_t>(p) * 32 + tid];

  // per-thread voxels (conv2, conv3, softmax)
  int gv[kCpgV];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) gv[v] = tid + v * kCpgThreads;

  // conv1 (32 -> 16, k3) as an implicit GEMM on v_mfma_f32_16x16x4_f32: rows = 16-voxel tiles,
  // k = the round's 4 input channels at one tap, columns = the 16 output channels.  Wave w owns
  // tiles w, w + 16, ... with their accumulators in registers: each k-step is one B fragment
  // (weights) and up to kTW independent MFMAs.  The input is haloed (zero border), so a tap is a
  // constant address shift and needs no mask; lane reads voxel 16 t + (lane & 15), channel
  // lane >> 4 of the round.
  constexpr int kT = (kCpgMaxC + 15) / 16;          // voxel tiles at C = 1331
  constexpr int kW = kCpgThreads / 64;
  constexpr int kTW = (kT + kW - 1) / kW;           // per wave
  const int lane = tid & 63, wave = tid >> 6, kg = lane >> 4, l16 = lane & 15;
  const int NT = (C + 15) / 16;
  int vx[kTW];  // haloed address of the lane's voxel per tile (a border cell past the end)
#pragma unroll
  for (int i = 0; i < kTW; ++i) {
    const int g = 16 * (wave + kW * i) + l16;
    vx[i] = g < C ? cpg_halo(g, dG, dGG, PG, PGG) : 0;
  }
  f32x4 acc[kTW];
#pragma unroll
  for (int i = 0; i < kTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int q = 0; q < 32 / kCpgQ; ++q) {
    __syncthreads();  // the previous round's readers are done
    for (int i = tid; i < kCpgW1F; i += kCpgThreads) {  // w1[ci][tap][co] = W1[co][4q + ci][tap]
      const int co = i % 16, r = i / 16;
      w1[i] = P1[co * (32 * 27) + kCpgQ * q * 27 + r];
    }
    // cost volume round: channels f' in [4q, 4q + 4) of cost[f'][g] = (src[f'] - T[l])^2,
    // l = g*32 + f' = f*C + c (the reference's reshape, Q11).  (The opaque zero keeps the
    // compiler from hoisting 84 addresses per thread out of the round loop into registers.)
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
      if (e < 32 * C && (fp >> 2) == q) {
        const float d = sv[fp] - tv[u];
        vol[(fp & 3) * PV + cpg_halo(g, dG, dGG, PG, PGG)] = d * d;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int t = 0; t < 27; ++t) {
      const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
      const float bw = w1[(kg * 27 + t) * 16 + l16];
      const float* vin = vol + kg * PV + off;
#pragma unroll
      for (int i = 0; i < kTW; ++i)
        if (wave + kW * i < NT)  // wave-uniform
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(vin[vx[i]], bw, acc[i], 0, 0, 0);
    }
  }

  // conv2 (16 -> 4) on VALU, one voxel per thread, conv1's output through LDS in two haloed
  // 8-channel halves; accumulator register r of conv1 lane l is voxel 16 t + 4 (l >> 4) + r,
  // output channel l & 15
  int hv[kCpgV];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) hv[v] = cpg_halo(gv[v] < C ? gv[v] : 0, dG, dGG, PG, PGG);
  float o2[kCpgV][4];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
#pragma unroll
    for (int co = 0; co < 4; ++co) o2[v][co] = 0.f;
#pragma unroll 1
  for (int h = 0; h < 16 / kCpgHalf; ++h) {
    __syncthreads();
    if (h == 0)
      for (int i = tid; i < kCpgHalf * PV; i += kCpgThreads) out1[i] = 0.f;  // zero halo (interior rewritten)
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kTW; ++i) {
      const int t = wave + kW * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int g = 16 * t + 4 * kg + r;
        if (t < NT && g < C && (l16 >> 3) == h)
          out1[(l16 & 7) * PV + cpg_halo(g, dG, dGG, PG, PGG)] = acc[i][r] + bias[l16];
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int ci = 0; ci < kCpgHalf; ++ci) {
      // W2[co][8h + ci][tap] for the 4 outputs: wave-uniform scalar loads, one input channel at a time
      const float* xin = out1 + ci * PV;
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        // one tap plane's 4 x 9 weights at a time (an opaque zero ordered after the running sums
        // keeps all 108 from being loaded into SGPRs at once)
        int zw = 0;
        asm volatile("" : "+s"(zw) : "v"(o2[0][0]));
        const float* w2c = P2 + (kCpgHalf * h + ci) * 27 + 9 * kd + zw;
#pragma unroll
        for (int t9 = 0; t9 < 9; ++t9) {
          const int t = 9 * kd + t9;
          const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
#pragma unroll
          for (int v = 0; v < kCpgV; ++v) {
            if (v == 0 || gv[v] < C) {
              const float x = xin[hv[v] + off];
#pragma unroll
              for (int co = 0; co < 4; ++co) o2[v][co] = __fmaf_rn(w2c[co * 16 * 27 + t9], x, o2[v][co]);
            }
          }
        }
      }
    }
  }
  __syncthreads();
  // conv2 output -> out2 (haloed; the border cells are still zero from the halves)
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
    const int g = gv[v] < C ? gv[v] : 0;
    const int hv = cpg_halo(g, dG, dGG, PG, PGG);
    float a = 0.f;
#pragma unroll
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int off = (t / 9 - 1) * PGG + ((t / 3) % 3 - 1) * PG + (t % 3 - 1);
        a = __fmaf_rn(w3[ci * 27 + t], out2[ci * PV + hv + off], a);
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
  hipLaunchKernelGGL(dvcp::cpg_kernel, dim3(P), dim3(dvcp::kCpgThreads), 0, static_cast<hipStream_t>(stream), src, tgt,
                     t_p, t_f, t_c, cand, G, params, vcp, weight);
  return dvcp::launch_status("dvcp_cpg");
}
