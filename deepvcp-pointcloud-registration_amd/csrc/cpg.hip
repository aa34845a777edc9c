// cpg.hip -- corresponding point generation (cpg.py:27-60), one workgroup per key point.
//
//   cost[f'][g] = (src[f'] - T[g*32 + f'])^2 where T is the reference's reshape of the
//                 permuted (32, C) target tensor (Q11: T[l] = tgt[f = l / C][c = l % C]);
//   Conv3d 32->16 -> 16->4 -> 4->1 (k3, p1, cross-correlation, no activations);
//   softmax over the C = G^3 logits; vcp = sum(w * cand) / sum(w).
//
// LDS plan (G <= 11, C <= 1331): a 16-channel half of the cost volume (85 KB) plus conv1's
// weights ([ci][tap][co], 55 KB, broadcast b128 reads).  conv1 runs as two input-channel
// halves accumulating into VGPRs (<= 6 voxels x 16 channels per thread); its output then
// replaces the cost volume in LDS for conv2, and conv2/conv3 outputs reuse the weight area.
#include "common.h"

namespace dvcp {

constexpr int kCpgThreads = 256;
constexpr int kCpgMaxC = 1331;
constexpr int kCpgV = (kCpgMaxC + kCpgThreads - 1) / kCpgThreads;  // voxels per thread

__global__ __launch_bounds__(kCpgThreads) void cpg_kernel(const float* __restrict__ src, const float* __restrict__ tgt,
                                                          int64_t t_p, int64_t t_f, int64_t t_c,
                                                          const float* __restrict__ cand, int G,
                                                          const float* __restrict__ params, float* __restrict__ vcp,
                                                          float* __restrict__ weight) {
  __shared__ __attribute__((aligned(16))) float vol[16 * kCpgMaxC];  // cost half / conv1 output
  __shared__ __attribute__((aligned(16))) float w1[32 * 27 * 16];    // conv1 W [ci][tap][co]; later conv2/3 outputs
  __shared__ __attribute__((aligned(16))) float w2[16 * 27 * 4];     // conv2 W [ci][tap][co]
  __shared__ float w3[4 * 27];
  __shared__ float bias[16 + 4 + 1];
  __shared__ float sv[32];
  __shared__ float red[32];

  const int p = blockIdx.x, tid = threadIdx.x;
  const int C = G * G * G, GG = G * G;
  const float* P1 = params;
  const float* P2 = P1 + 16 * 32 * 27 + 16;
  const float* P3 = P2 + 4 * 16 * 27 + 4;
  for (int i = tid; i < 16 * 32 * 27; i += kCpgThreads) {  // torch (co, ci, kd, kh, kw)
    const int co = i / (32 * 27), r = i % (32 * 27);
    w1[r * 16 + co] = P1[i];
  }
  for (int i = tid; i < 4 * 16 * 27; i += kCpgThreads) {
    const int co = i / (16 * 27), r = i % (16 * 27);
    w2[r * 4 + co] = P2[i];
  }
  if (tid < 4 * 27) w3[tid] = P3[tid];
  if (tid < 16) bias[tid] = P1[16 * 32 * 27 + tid];
  if (tid < 4) bias[16 + tid] = P2[4 * 16 * 27 + tid];
  if (tid == 0) bias[20] = P3[4 * 27];
  if (tid < 32) sv[tid] = src[static_cast<int64_t>(p) * 32 + tid];

  // per-thread voxels and their 27-tap validity masks (zero padding)
  int gv[kCpgV];
  uint32_t mask[kCpgV];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) {
    const int g = tid + v * kCpgThreads;
    gv[v] = g;
    uint32_t m = 0;
    if (g < C) {
      const int x = g / GG, y = (g / G) % G, z = g % G;
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int dx = t / 9 - 1, dy = (t / 3) % 3 - 1, dz = t % 3 - 1;
        const bool ok = x + dx >= 0 && x + dx < G && y + dy >= 0 && y + dy < G && z + dz >= 0 && z + dz < G;
        m |= (ok ? 1u : 0u) << t;
      }
    }
    mask[v] = m;
  }

  float acc[kCpgV][16];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
#pragma unroll
    for (int co = 0; co < 16; ++co) acc[v][co] = 0.f;

  const float* T = tgt + static_cast<int64_t>(p) * t_p;
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
    // cost volume half: channel f' in [16*half, 16*half+16); iterate the target in memory
    // order (c, f) and scatter l = f*C + c -> (g = l / 32, f' = l % 32).
    for (int e = tid; e < 32 * C; e += kCpgThreads) {
      const int c = e / 32, f = e % 32;
      const int l = f * C + c;
      const int g = l >> 5, fp = l & 31;
      if ((fp >> 4) == half) {
        const float d = sv[fp] - T[f * t_f + c * t_c];
        vol[(fp & 15) * C + g] = d * d;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int cl = 0; cl < 16; ++cl) {
      const float* vin = vol + cl * C;
      const float* wrow = w1 + (half * 16 + cl) * 27 * 16;
#pragma unroll 1
      for (int t = 0; t < 27; ++t) {
        const int off = (t / 9 - 1) * GG + ((t / 3) % 3 - 1) * G + (t % 3 - 1);
        const float4* w4 = reinterpret_cast<const float4*>(wrow + t * 16);
        const float4 wa = w4[0], wb = w4[1], wc = w4[2], wd = w4[3];
        const float w[16] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w,
                             wc.x, wc.y, wc.z, wc.w, wd.x, wd.y, wd.z, wd.w};
#pragma unroll
        for (int v = 0; v < kCpgV; ++v) {
          const float xin = ((mask[v] >> t) & 1u) ? vin[gv[v] + off] : 0.f;
#pragma unroll
          for (int co = 0; co < 16; ++co) acc[v][co] = __fmaf_rn(w[co], xin, acc[v][co]);
        }
      }
    }
  }
  __syncthreads();
  // conv1 output -> vol[co][g]
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
    if (gv[v] < C)
#pragma unroll
      for (int co = 0; co < 16; ++co) vol[co * C + gv[v]] = acc[v][co] + bias[co];
  __syncthreads();

  // conv2: 16 -> 4
  float a2[kCpgV][4];
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
#pragma unroll
    for (int co = 0; co < 4; ++co) a2[v][co] = 0.f;
#pragma unroll 1
  for (int ci = 0; ci < 16; ++ci) {
    const float* vin = vol + ci * C;
#pragma unroll 1
    for (int t = 0; t < 27; ++t) {
      const int off = (t / 9 - 1) * GG + ((t / 3) % 3 - 1) * G + (t % 3 - 1);
      const float4 w = reinterpret_cast<const float4*>(w2 + (ci * 27 + t) * 4)[0];
#pragma unroll
      for (int v = 0; v < kCpgV; ++v) {
        const float xin = ((mask[v] >> t) & 1u) ? vin[gv[v] + off] : 0.f;
        a2[v][0] = __fmaf_rn(w.x, xin, a2[v][0]);
        a2[v][1] = __fmaf_rn(w.y, xin, a2[v][1]);
        a2[v][2] = __fmaf_rn(w.z, xin, a2[v][2]);
        a2[v][3] = __fmaf_rn(w.w, xin, a2[v][3]);
      }
    }
  }
  float* out2 = w1;  // conv1 weights are dead now
#pragma unroll
  for (int v = 0; v < kCpgV; ++v)
    if (gv[v] < C)
#pragma unroll
      for (int co = 0; co < 4; ++co) out2[co * C + gv[v]] = a2[v][co] + bias[16 + co];
  __syncthreads();

  // conv3: 4 -> 1
  float lg[kCpgV];
  float lmax = -__builtin_huge_valf();
#pragma unroll
  for (int v = 0; v < kCpgV; ++v) {
    float a = 0.f;
#pragma unroll 1
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll 1
      for (int t = 0; t < 27; ++t) {
        const int off = (t / 9 - 1) * GG + ((t / 3) % 3 - 1) * G + (t % 3 - 1);
        const float xin = ((mask[v] >> t) & 1u) ? out2[ci * C + gv[v] + off] : 0.f;
        a = __fmaf_rn(w3[ci * 27 + t], xin, a);
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
