// paper.hip -- the paper-faithful mode's own stages (DeepVCP paper, Lu et al. ICCV 2019; SURVEY.md
// 8(f) rank 4; NOT reference parity -- the reference repository never runs these):
//
//   fp_kernel        PointNet++ feature propagation (the reference's dead PointNetFeaturePropagation,
//                    pointnet2_utils.py:265-315): 3-NN of every xyz1 point among xyz2 under the
//                    expansion-form squared distance (:296, square_distance, ties to the lower
//                    index), inverse-distance weights 1 / (d + 1e-8) normalised (:300-302), the
//                    interpolated rows concatenated after points1 (:305-307), then per layer a 1x1
//                    conv with folded eval-mode BN and ReLU (:312-314); an optional last layer
//                    without BN / ReLU carries the FE's fully connected layer (paper supplement).
//   group_rows_kernel  the DFE input of paper Sec. 3.3: for each centre, rows [(p - c) / d, f(p)]
//                    over its ball-query list (dvcp_ball_query), padded with the first hit
//                    (pointnet2_utils.py:104-106); a centre with no point within d gets zero rows.
//   cpg1d_kernel     the duplicated network's CPG (paper Sec. 3.6): cost (src - tgt)^2 over the Gz
//                    candidates of a z line, Conv1d 32-16-4-1 (k 3, p 1, no activations, like
//                    cpg.py:45-47), softmax over the line and the weighted candidate mean
//                    (cpg.py:53-58).
#include "common.h"

namespace dvcp {

// ------------------------------------------------------------------------ feature propagation
constexpr int kFpRows = 32;      // points per workgroup
constexpr int kFpThreads = 256;  // 8 threads per point in the 3-NN scan
constexpr int kFpTile = 1024;    // xyz2 points per LDS tile
constexpr int kFpMaxC = 128;     // widest row / layer input
constexpr int kFpMaxCo = 64;     // widest layer output
constexpr int kFpMaxL = 4;

struct FpLayers {
  int L;
  int ch[kFpMaxL + 1];
  int relu[kFpMaxL];
};

__device__ __forceinline__ uint64_t fp_key(float d2, int idx) {
  return (static_cast<uint64_t>(float_order(d2)) << 32) | static_cast<uint32_t>(idx);
}
__device__ __forceinline__ float fp_key_d2(uint64_t k) {  // inverse of float_order
  const uint32_t u = static_cast<uint32_t>(k >> 32);
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ void top3_insert(uint64_t (&k)[3], uint64_t v) {
  if (v < k[2]) {
    if (v < k[1]) {
      k[2] = k[1];
      if (v < k[0]) {
        k[1] = k[0];
        k[0] = v;
      } else {
        k[1] = v;
      }
    } else {
      k[2] = v;
    }
  }
}

__global__ __launch_bounds__(kFpThreads) void fp_kernel(PointsView<float> xyz1, int N1, PointsView<float> xyz2, int N2,
                                                        const float* __restrict__ p1, int64_t p1b, int64_t p1d,
                                                        int64_t p1n, int D1, const float* __restrict__ p2, int64_t p2b,
                                                        int64_t p2n, int D2, FpLayers lay,
                                                        const float* __restrict__ params, float* __restrict__ out) {
  __shared__ float4 tile[kFpTile];
  __shared__ float buf[2][kFpRows][kFpMaxC + 1];
  __shared__ float wsh[kFpMaxCo * kFpMaxC];
  __shared__ float bsh[3][kFpMaxCo];
  __shared__ int nidx[kFpRows][3];
  __shared__ float nwt[kFpRows][3];
  const int b = blockIdx.y, r0 = blockIdx.x * kFpRows, tid = threadIdx.x;
  const int row = tid >> 3, part = tid & 7;
  const int n = r0 + row;
  const bool live = n < N1;
  float cx = 0.f, cy = 0.f, cz = 0.f;
  if (live) {
    cx = xyz1.at(b, 0, n);
    cy = xyz1.at(b, 1, n);
    cz = xyz1.at(b, 2, n);
  }
  const float ssc = sumsq3(cx, cy, cz);
  uint64_t k3[3] = {~0ull, ~0ull, ~0ull};
  for (int t0 = 0; t0 < N2; t0 += kFpTile) {
    const int nt = min(kFpTile, N2 - t0);
    __syncthreads();
    for (int j = tid; j < nt; j += kFpThreads) {
      const float x = xyz2.at(b, 0, t0 + j), y = xyz2.at(b, 1, t0 + j), z = xyz2.at(b, 2, t0 + j);
      tile[j] = make_float4(x, y, z, sumsq3(x, y, z));
    }
    __syncthreads();
    for (int j = part; j < nt; j += 8) {
      const float4 p = tile[j];
      top3_insert(k3, fp_key(expansion_d2(dot3_blas(cx, cy, cz, p.x, p.y, p.z), ssc, p.w), t0 + j));
    }
  }
  // merge the 8 partial lists of a row (8 consecutive lanes; the partners' sets are disjoint)
#pragma unroll
  for (int off = 1; off < 8; off <<= 1) {
    uint64_t o[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = __shfl_xor(k3[i], off, kWave);
#pragma unroll
    for (int i = 0; i < 3; ++i) top3_insert(k3, o[i]);
  }
  if (part == 0) {
    const int nk = N2 < 3 ? N2 : 3;
    float w[3] = {0.f, 0.f, 0.f};
    int id[3] = {0, 0, 0};
    if (N2 == 1) {  // :293-294 points2.repeat
      w[0] = 1.0f;
    } else {
      float rc[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        id[i] = i < nk ? static_cast<int>(k3[i] & 0xFFFFFFFFull) : 0;
        rc[i] = i < nk ? 1.0f / (fp_key_d2(k3[i]) + 1e-8f) : 0.f;  // :300
      }
      float norm = rc[0] + rc[1];  // :301 (sum over the 3 neighbours, in order)
      if (nk > 2) norm = norm + rc[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) w[i] = i < nk ? rc[i] / norm : 0.f;  // :302
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      nidx[row][i] = id[i];
      nwt[row][i] = w[i];
    }
  }
  __syncthreads();
  // layer-0 rows: [points1, interpolated] (:303-307)
  const int C0 = D1 + D2;
  const int nk = N2 < 3 ? N2 : 3;
  const float* q2 = p2 + b * p2b;
  for (int e = tid; e < kFpRows * C0; e += kFpThreads) {
    const int rr = e / C0, c = e % C0, nn = r0 + rr;
    float v = 0.f;
    if (nn < N1) {
      if (c < D1) {
        v = p1[b * p1b + c * p1d + nn * p1n];
      } else {
        const int cc = c - D1;
        v = q2[nidx[rr][0] * p2n + cc] * nwt[rr][0];
        if (nk > 1) v = v + q2[nidx[rr][1] * p2n + cc] * nwt[rr][1];
        if (nk > 2) v = v + q2[nidx[rr][2] * p2n + cc] * nwt[rr][2];
      }
    }
    buf[0][rr][c] = v;
  }
  int cur = 0;
  const float* P = params;
  for (int l = 0; l < lay.L; ++l) {
    const int ci = lay.ch[l], co = lay.ch[l + 1];
    __syncthreads();
    for (int e = tid; e < ci * co; e += kFpThreads) wsh[e] = P[e];  // W (co x ci)
    for (int e = tid; e < co; e += kFpThreads) {
      bsh[0][e] = P[ci * co + e];
      bsh[1][e] = P[ci * co + co + e];
      bsh[2][e] = P[ci * co + 2 * co + e];
    }
    __syncthreads();
    for (int e = tid; e < kFpRows * co; e += kFpThreads) {
      const int rr = e / co, o = e % co;
      float acc = 0.f;
      for (int k = 0; k < ci; ++k) acc = __fmaf_rn(wsh[o * ci + k], buf[cur][rr][k], acc);
      float v = (acc + bsh[0][o]) * bsh[1][o] + bsh[2][o];
      if (lay.relu[l]) v = v > 0.f ? v : 0.f;
      buf[cur ^ 1][rr][o] = v;
    }
    cur ^= 1;
    P += ci * co + 3 * co;
  }
  __syncthreads();
  const int CL = lay.ch[lay.L];
  for (int e = tid; e < kFpRows * CL; e += kFpThreads) {
    const int rr = e / CL, o = e % CL, nn = r0 + rr;
    if (nn < N1) out[(static_cast<int64_t>(b) * N1 + nn) * CL + o] = buf[cur][rr][o];
  }
}

// --------------------------------------------------------------------------------- group rows
__global__ void group_rows_kernel(PointsView<float> ctr, int Q, PointsView<float> xyz, const float* __restrict__ feat,
                                  int64_t fb, int64_t fn, int D, const int32_t* __restrict__ count,
                                  const int32_t* __restrict__ list, int ns_list, int ns_out, float radius, int B,
                                  float* __restrict__ rows) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t total = static_cast<int64_t>(B) * Q * ns_out;
  if (i >= total) return;
  const int slot = static_cast<int>(i % ns_out);
  const int64_t bq = i / ns_out;
  const int b = static_cast<int>(bq / Q), q = static_cast<int>(bq % Q);
  float* o = rows + i * (3 + D);
  const int cnt = count[bq];
  if (cnt <= 0) {
    for (int c = 0; c < 3 + D; ++c) o[c] = 0.f;
    return;
  }
  const int n = list[bq * ns_list + (slot < cnt ? slot : 0)];
  o[0] = (xyz.at(b, 0, n) - ctr.at(b, 0, q)) / radius;
  o[1] = (xyz.at(b, 1, n) - ctr.at(b, 1, q)) / radius;
  o[2] = (xyz.at(b, 2, n) - ctr.at(b, 2, q)) / radius;
  const float* f = feat + b * fb + static_cast<int64_t>(n) * fn;
  for (int c = 0; c < D; ++c) o[3 + c] = f[c];
}

// ------------------------------------------------------------------------------------- 1-D CPG
constexpr int kC1MaxG = 64;
constexpr int kCpg1dParams = 16 * 32 * 3 + 16 + 4 * 16 * 3 + 4 + 1 * 4 * 3 + 1;

__global__ __launch_bounds__(kC1MaxG) void cpg1d_kernel(const float* __restrict__ src, const float* __restrict__ tgt,
                                                        const float* __restrict__ cand, int Gz,
                                                        const float* __restrict__ params, float* __restrict__ vcp,
                                                        float* __restrict__ weight) {
  __shared__ float cost[32][kC1MaxG + 2];
  __shared__ float h1[16][kC1MaxG + 2];
  __shared__ float h2[4][kC1MaxG + 2];
  const int p = blockIdx.x, z = threadIdx.x;
  const bool in = z < Gz;
  const float* W1 = params;
  const float* b1 = W1 + 16 * 32 * 3;
  const float* W2 = b1 + 16;
  const float* b2 = W2 + 4 * 16 * 3;
  const float* W3 = b2 + 4;
  const float* b3 = W3 + 4 * 3;
  // column z + 1 holds candidate z; columns 0 and Gz + 1 (and beyond) are the zero padding
  for (int f = 0; f < 32; ++f) {
    float v = 0.f;
    if (in) {
      const float d = src[static_cast<int64_t>(p) * 32 + f] - tgt[(static_cast<int64_t>(p) * Gz + z) * 32 + f];
      v = d * d;
    }
    cost[f][z + 1] = v;
    if (z == 0) cost[f][0] = 0.f;
    if (z == 0) cost[f][kC1MaxG + 1] = 0.f;
  }
  __syncthreads();
  for (int co = 0; co < 16; ++co) {
    float acc = 0.f;
    for (int ci = 0; ci < 32; ++ci)
#pragma unroll
      for (int k = 0; k < 3; ++k) acc = __fmaf_rn(W1[(co * 32 + ci) * 3 + k], cost[ci][z + k], acc);
    h1[co][z + 1] = in ? acc + b1[co] : 0.f;
    if (z == 0) h1[co][0] = 0.f;
    if (z == 0) h1[co][kC1MaxG + 1] = 0.f;
  }
  __syncthreads();
  for (int co = 0; co < 4; ++co) {
    float acc = 0.f;
    for (int ci = 0; ci < 16; ++ci)
#pragma unroll
      for (int k = 0; k < 3; ++k) acc = __fmaf_rn(W2[(co * 16 + ci) * 3 + k], h1[ci][z + k], acc);
    h2[co][z + 1] = in ? acc + b2[co] : 0.f;
    if (z == 0) h2[co][0] = 0.f;
    if (z == 0) h2[co][kC1MaxG + 1] = 0.f;
  }
  __syncthreads();
  float lg = 0.f;
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int k = 0; k < 3; ++k) lg = __fmaf_rn(W3[ci * 3 + k], h2[ci][z + k], lg);
  lg = lg + b3[0];
  // softmax over the line (exp(x - max), sum, multiply by 1 / sum) and the weighted mean
  const float m = wave_max_f(in ? lg : -__builtin_huge_valf());
  const float e = in ? expf(lg - m) : 0.f;
  const float inv = 1.0f / wave_sum(e);
  const float w = e * inv;
  if (weight && in) weight[static_cast<int64_t>(p) * Gz + z] = w;
  const float* cq = cand + (static_cast<int64_t>(p) * Gz + (in ? z : 0)) * 3;
  const float sw = wave_sum(w);
  const float sx = wave_sum(in ? w * cq[0] : 0.f);
  const float sy = wave_sum(in ? w * cq[1] : 0.f);
  const float sz = wave_sum(in ? w * cq[2] : 0.f);
  if (z == 0) {
    vcp[static_cast<int64_t>(p) * 3 + 0] = sx / sw;
    vcp[static_cast<int64_t>(p) * 3 + 1] = sy / sw;
    vcp[static_cast<int64_t>(p) * 3 + 2] = sz / sw;
  }
}

}  // namespace dvcp

extern "C" int dvcp_feature_propagation(const float* xyz1, int64_t x1b, int64_t x1c, int64_t x1n, int N1,
                                        const float* xyz2, int64_t x2b, int64_t x2c, int64_t x2n, int N2, int B,
                                        const float* p1, int64_t p1b, int64_t p1d, int64_t p1n, int D1,
                                        const float* p2, int64_t p2b, int64_t p2n, int D2, int nlayer,
                                        const int* chans, const int* relu, const float* params, float* out,
                                        void* stream) {
  DVCP_REQUIRE(xyz1 && xyz2 && p2 && chans && relu && params && out, "dvcp_feature_propagation: null pointer");
  DVCP_REQUIRE(N1 >= 0 && N2 >= 1 && B >= 0 && B <= 65535 && D1 >= 0 && D2 >= 1 && (D1 == 0 || p1),
               "dvcp_feature_propagation: bad sizes N1=%d N2=%d B=%d D1=%d D2=%d", N1, N2, B, D1, D2);
  DVCP_REQUIRE(N2 != 2, "dvcp_feature_propagation: N2 = 2 (the reference's weight.view(B, N, 3, 1), "
               "pointnet2_utils.py:303, fails for two interpolation points)");
  DVCP_REQUIRE(nlayer >= 1 && nlayer <= dvcp::kFpMaxL, "dvcp_feature_propagation: 1..%d layers", dvcp::kFpMaxL);
  DVCP_REQUIRE(chans[0] == D1 + D2, "dvcp_feature_propagation: chans[0]=%d != D1 + D2", chans[0]);
  dvcp::FpLayers lay{};
  lay.L = nlayer;
  for (int l = 0; l <= nlayer; ++l) {
    DVCP_REQUIRE(chans[l] >= 1 && chans[l] <= (l == 0 ? dvcp::kFpMaxC : dvcp::kFpMaxCo),
                 "dvcp_feature_propagation: layer width %d out of range", chans[l]);
    lay.ch[l] = chans[l];
  }
  for (int l = 0; l < nlayer; ++l) lay.relu[l] = relu[l] != 0;
  if (B == 0 || N1 == 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::fp_kernel, dim3(dvcp::ceil_div(N1, dvcp::kFpRows), B), dim3(dvcp::kFpThreads), 0,
                     static_cast<hipStream_t>(stream), dvcp::PointsView<float>{xyz1, x1b, x1c, x1n}, N1,
                     dvcp::PointsView<float>{xyz2, x2b, x2c, x2n}, N2, p1, p1b, p1d, p1n, D1, p2, p2b, p2n, D2, lay,
                     params, out);
  return dvcp::launch_status("dvcp_feature_propagation");
}

extern "C" int dvcp_group_rows(const float* ctr, int64_t cb, int64_t cc, int64_t cn, int Q, const float* xyz,
                               int64_t sb, int64_t sc, int64_t sn, const float* feat, int64_t fb, int64_t fn, int D,
                               const int32_t* count, const int32_t* list, int ns_list, int ns_out, double radius,
                               int B, float* rows, void* stream) {
  DVCP_REQUIRE(ctr && xyz && count && list && rows && (D == 0 || feat), "dvcp_group_rows: null pointer");
  DVCP_REQUIRE(Q >= 0 && B >= 0 && D >= 0 && ns_list >= 1 && ns_out >= 1 && radius > 0,
               "dvcp_group_rows: bad sizes Q=%d B=%d D=%d ns=%d/%d", Q, B, D, ns_list, ns_out);
  const int64_t total = static_cast<int64_t>(B) * Q * ns_out;
  if (total == 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::group_rows_kernel, dim3(dvcp::ceil_div(total, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), dvcp::PointsView<float>{ctr, cb, cc, cn}, Q,
                     dvcp::PointsView<float>{xyz, sb, sc, sn}, feat, fb, fn, D, count, list, ns_list, ns_out,
                     static_cast<float>(radius), B, rows);
  return dvcp::launch_status("dvcp_group_rows");
}

extern "C" int dvcp_cpg1d(const float* src, const float* tgt, const float* cand, int P, int Gz, const float* params,
                          float* vcp, float* weight, void* stream) {
  DVCP_REQUIRE(src && tgt && cand && params && vcp, "dvcp_cpg1d: null pointer");
  DVCP_REQUIRE(Gz >= 1 && Gz <= dvcp::kC1MaxG && P >= 0, "dvcp_cpg1d: Gz=%d unsupported (1..%d)", Gz, dvcp::kC1MaxG);
  if (P == 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::cpg1d_kernel, dim3(P), dim3(dvcp::kC1MaxG), 0, static_cast<hipStream_t>(stream), src, tgt,
                     cand, Gz, params, vcp, weight);
  return dvcp::launch_status("dvcp_cpg1d");
}

extern "C" int dvcp_cpg1d_nparams(void) { return dvcp::kCpg1dParams; }
