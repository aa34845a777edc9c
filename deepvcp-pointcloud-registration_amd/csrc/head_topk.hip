// head_topk.hip -- FE output projection + weighting layer + key-point top-k.
//   dvcp_fe_head: deep_feat_extraction.py:15 `fc` (64 -> 32, applied per REF-R R1) and
//                 weighting_layer.py:26-30 (Linear 32-16-8-1, ReLU, ReLU, Softplus).
//   dvcp_topk:    weighting_layer.py:31 torch.topk(X, K, dim=1) (sorted, descending).
#include "common.h"

namespace dvcp {

__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

// torch.nn.Softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplus(float v) { return v > 20.0f ? v : log1pf(expf(v)); }

// rows != nullptr: output row i reads input row (i / S) * Nx + rows[i] (a per-cloud gather of the
// per-point sa3 rows by the FPS order, folded into the load; indices clamped to [0, Nx)).
__global__ __launch_bounds__(256) void fe_head_kernel(const float* __restrict__ x, const int64_t* __restrict__ rows,
                                                      int S, int Nx, int P, const float* __restrict__ params,
                                                      float* __restrict__ feat, float* __restrict__ score) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float in[64];
  int64_t r = i;
  if (rows) {
    const int64_t n = rows[i];
    r = static_cast<int64_t>(i / S) * Nx + (n < 0 ? 0 : (n >= Nx ? Nx - 1 : n));
  }
  const float4* src = reinterpret_cast<const float4*>(x + r * 64);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 v = src[q];
    in[4 * q] = v.x;
    in[4 * q + 1] = v.y;
    in[4 * q + 2] = v.z;
    in[4 * q + 3] = v.w;
  }
  float f[32];
  linear_sgpr<64, 32>(in, f, params);
  float4* dst = reinterpret_cast<float4*>(feat + static_cast<int64_t>(i) * 32);
#pragma unroll
  for (int q = 0; q < 8; ++q) dst[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
  if (!score) return;
  const float* w1 = params + 64 * 32 + 32;
  const float* w2 = w1 + 32 * 16 + 16;
  const float* w3 = w2 + 16 * 8 + 8;
  float h1[16], h2[8], h3[1];
  linear_sgpr<32, 16>(f, h1, w1);
#pragma unroll
  for (int c = 0; c < 16; ++c) h1[c] = relu(h1[c]);
  linear_sgpr<16, 8>(h1, h2, w2);
#pragma unroll
  for (int c = 0; c < 8; ++c) h2[c] = relu(h2[c]);
  linear_sgpr<8, 1>(h2, h3, w3);
  score[i] = softplus(h3[0]);
}

// weighting_layer.py:27-30 alone on (P, 32) features.
__global__ __launch_bounds__(256) void weighting_kernel(const float* __restrict__ x, int P, const float* __restrict__ params,
                                                        float* __restrict__ score) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float f[32];
  const float4* src = reinterpret_cast<const float4*>(x + static_cast<int64_t>(i) * 32);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = src[q];
    f[4 * q] = v.x;
    f[4 * q + 1] = v.y;
    f[4 * q + 2] = v.z;
    f[4 * q + 3] = v.w;
  }
  const float* w2 = params + 32 * 16 + 16;
  const float* w3 = w2 + 16 * 8 + 8;
  float h1[16], h2[8], h3[1];
  linear_sgpr<32, 16>(f, h1, params);
#pragma unroll
  for (int c = 0; c < 16; ++c) h1[c] = relu(h1[c]);
  linear_sgpr<16, 8>(h1, h2, w2);
#pragma unroll
  for (int c = 0; c < 8; ++c) h2[c] = relu(h2[c]);
  linear_sgpr<8, 1>(h2, h3, w3);
  score[i] = softplus(h3[0]);
}

// Top-K of one row per workgroup: K rounds of a block argmax over the remaining elements
// (value descending, ties -> lower index), one barrier per round (double-buffered slots).
template <int PPT>
__global__ __launch_bounds__(1024) void topk_kernel(const float* __restrict__ score, int S, int K, int64_t* __restrict__ out) {
  constexpr int NT = 1024;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ uint64_t slots[2][NT / kWave];
  uint64_t key[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int n = tid + p * NT;
    key[p] = n < S ? ((static_cast<uint64_t>(float_order(score[static_cast<int64_t>(b) * S + n])) << 32) |
                      static_cast<uint64_t>(0xFFFFFFFFu - static_cast<uint32_t>(n)))
                   : 0ull;
  }
  for (int k = 0; k < K; ++k) {
    uint64_t best = 0;
#pragma unroll
    for (int p = 0; p < PPT; ++p) best = key[p] > best ? key[p] : best;
    const uint64_t w = wave_max_u64(best);
    if (lane == 0) slots[k & 1][wave] = w;
    lds_barrier();
    uint64_t m = slots[k & 1][0];
#pragma unroll
    for (int q = 1; q < NT / kWave; ++q) m = slots[k & 1][q] > m ? slots[k & 1][q] : m;
    const uint32_t win = key_index(m);
    if (tid == 0) out[static_cast<int64_t>(b) * K + k] = win;
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (key[p] == m) key[p] = 0ull;
  }
}

// Top-K by radix select (default): the K-th largest 64-bit key (float order of the score << 32 |
// ~index: value descending, ties -> lower index, exactly the argmax rounds' order) is found 8 bits
// at a time below the keys' common prefix (LDS histogram, one wave picks the digit), then the K
// keys at or above it are gathered and each one's output position is its count of larger keys.
// ~3 barriers per pass and a few passes instead of K block-argmax rounds.
constexpr int kTopkMaxK = 1024;

template <int PPT>
__global__ __launch_bounds__(1024) void topk_select_kernel(const float* __restrict__ score, int S, int K,
                                                           int64_t* __restrict__ out) {
  constexpr int NT = 1024;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ uint32_t hist[256];
  __shared__ uint64_t red[2][NT / kWave];
  __shared__ uint64_t cand[kTopkMaxK];
  __shared__ uint32_t sel[2], ncand;
  uint64_t key[PPT];
  uint64_t kmax = 0ull, kmin = ~0ull;
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int n = tid + p * NT;
    key[p] = n < S ? ((static_cast<uint64_t>(float_order(score[static_cast<int64_t>(b) * S + n])) << 32) |
                      static_cast<uint64_t>(0xFFFFFFFFu - static_cast<uint32_t>(n)))
                   : 0ull;  // padding (n >= S): excluded by index from the histograms and the gather
    if (n < S) {
      kmax = key[p] > kmax ? key[p] : kmax;
      kmin = key[p] < kmin ? key[p] : kmin;
    }
  }
  // common prefix of the real keys: the radix passes start at their first differing bit
  kmax = wave_max_u64(kmax);
  kmin = ~wave_max_u64(~kmin);
  if (lane == 0) {
    red[0][wave] = kmax;
    red[1][wave] = ~kmin;
  }
  if (tid == 0) ncand = 0u;
  lds_barrier();
  uint64_t hi = red[0][0], lo_n = red[1][0];
#pragma unroll
  for (int w = 1; w < NT / kWave; ++w) {
    hi = red[0][w] > hi ? red[0][w] : hi;
    lo_n = red[1][w] > lo_n ? red[1][w] : lo_n;
  }
  const uint64_t lo = ~lo_n;
  const int top = hi == lo ? 0 : 63 - __clzll(static_cast<long long>(hi ^ lo));  // highest differing bit
  uint64_t prefix = hi & ~((top >= 63) ? ~0ull : ((2ull << top) - 1ull));       // bits above `top`
  uint64_t pmask = (top >= 63) ? 0ull : ~((2ull << top) - 1ull);
  uint32_t need = static_cast<uint32_t>(K);
  int shift = top + 1;  // bits [shift, 64) are fixed in prefix
#pragma unroll 1
  while (shift > 0) {
    const int w = shift >= 8 ? 8 : shift;
    shift -= w;
    for (int i = tid; i < 256; i += NT) hist[i] = 0u;
    lds_barrier();
    const uint32_t dm = (1u << w) - 1u;
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (tid + p * NT < S && (key[p] & pmask) == prefix)  // padding slots never vote (any score may
        atomicAdd(&hist[static_cast<uint32_t>(key[p] >> shift) & dm], 1u);  // share their key's top bits)
    lds_barrier();
    if (wave == 0) {
      // digits from the top: the digit d where the count of larger digits is < need <= count of
      // digits >= d.  Lane l holds digits 255 - 4l .. 252 - 4l (descending).
      uint32_t c[4], run = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - (4 * lane + j)];
        run += c[j];
      }
      uint32_t incl = run;  // inclusive prefix over lanes (descending digit order)
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        const uint32_t u = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += u;
      }
      uint32_t before = incl - run;  // keys with larger digits in lower lanes
      int dsel = -1;
      uint32_t above = 0, cnt_d = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (dsel < 0 && before + c[j] >= need) {
          dsel = 255 - (4 * lane + j);
          above = before;
          cnt_d = c[j];
        }
        before += c[j];
      }
      const uint64_t hit = __ballot(dsel >= 0);
      const int src = __ffsll(static_cast<long long>(hit)) - 1;
      const int d = __shfl(dsel, src, kWave);
      const uint32_t ab = __shfl(above, src, kWave), cd = __shfl(cnt_d, src, kWave);
      if (lane == 0) {
        sel[0] = static_cast<uint32_t>(d);
        sel[1] = (need - ab) | (cd == need - ab ? 0x80000000u : 0u);  // all keys of digit d are taken
      }
    }
    lds_barrier();
    prefix |= static_cast<uint64_t>(sel[0]) << shift;
    pmask |= static_cast<uint64_t>(dm) << shift;
    const uint32_t sv = sel[1];
    need = sv & 0x7FFFFFFFu;
    if (sv & 0x80000000u) break;  // every key matching the prefix is in the top K (uniform)
  }
  // the top K: keys above the prefix range, and every key in it (count == need)
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const uint64_t km = key[p] & pmask;
    if (tid + p * NT < S && km >= prefix) {
      const uint32_t i = atomicAdd(&ncand, 1u);
      if (i < static_cast<uint32_t>(kTopkMaxK)) cand[i] = key[p];
    }
  }
  lds_barrier();
  const int nc = min(static_cast<int>(ncand), K);
  for (int i = tid; i < nc; i += NT) {
    const uint64_t ki = cand[i];
    int r = 0;
    for (int j = 0; j < nc; ++j) r += cand[j] > ki ? 1 : 0;
    out[static_cast<int64_t>(b) * K + r] = key_index(ki);
  }
}

}  // namespace dvcp

extern "C" int dvcp_fe_head(const float* x, int P, const float* params, float* feat, float* score, void* stream) {
  DVCP_REQUIRE(x && params && feat, "dvcp_fe_head: null pointer");
  if (P <= 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::fe_head_kernel, dim3(dvcp::ceil_div(P, 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     x, nullptr, 1, 1, P, params, feat, score);
  return dvcp::launch_status("dvcp_fe_head");
}

extern "C" int dvcp_fe_head_rows(const float* x, const int64_t* rows, int S, int Nx, int P, const float* params,
                                 float* feat, float* score, void* stream) {
  DVCP_REQUIRE(x && rows && params && feat, "dvcp_fe_head_rows: null pointer");
  DVCP_REQUIRE(S > 0 && Nx > 0 && P % S == 0, "dvcp_fe_head_rows: bad sizes (S=%d, Nx=%d, P=%d)", S, Nx, P);
  if (P <= 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::fe_head_kernel, dim3(dvcp::ceil_div(P, 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     x, rows, S, Nx, P, params, feat, score);
  return dvcp::launch_status("dvcp_fe_head_rows");
}

extern "C" int dvcp_weighting(const float* feat, int P, const float* params, float* score, void* stream) {
  DVCP_REQUIRE(feat && params && score, "dvcp_weighting: null pointer");
  if (P <= 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::weighting_kernel, dim3(dvcp::ceil_div(P, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), feat, P, params, score);
  return dvcp::launch_status("dvcp_weighting");
}

extern "C" int dvcp_topk(const float* score, int B, int S, int K, int64_t* idx, void* stream) {
  DVCP_REQUIRE(score && idx, "dvcp_topk: null pointer");
  DVCP_REQUIRE(K >= 0 && K <= S, "dvcp_topk: K=%d out of range for S=%d", K, S);
  if (B == 0 || K == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int ppt = dvcp::ceil_div(S, 1024);
#define DVCP_TOPK(P)                                                                                   \
  if (ppt <= P) {                                                                                      \
    if (K <= dvcp::kTopkMaxK)                                                                          \
      hipLaunchKernelGGL((dvcp::topk_select_kernel<P>), dim3(B), dim3(1024), 0, st, score, S, K, idx); \
    else                                                                                               \
      hipLaunchKernelGGL((dvcp::topk_kernel<P>), dim3(B), dim3(1024), 0, st, score, S, K, idx);        \
    return dvcp::launch_status("dvcp_topk");                                                           \
  }
  DVCP_TOPK(1)
  DVCP_TOPK(4)
  DVCP_TOPK(10)
  DVCP_TOPK(16)
#undef DVCP_TOPK
  dvcp::set_error("dvcp_topk: S=%d exceeds 16384", S);
  return DVCP_EINVAL;
}
