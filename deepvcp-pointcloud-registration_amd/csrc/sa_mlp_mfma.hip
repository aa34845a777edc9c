// sa_mlp_mfma.hip -- the two-layer set-abstraction MLPs (sa2: 35-32-64, sa3: 67-64-64;
// pointnet2_utils.py:122-132 + :195-200 with REF-R R1) on fp32 MFMA (v_mfma_f32_32x32x2_f32), and
// (sa3_mfma_kernel, further down) the three-layer sa1 table.  A centre without hits (count < 1)
// gets zeros in every kernel, like the row-per-thread kernel of sa_mlp.hip; no list entry is read.
//
// Per centre the grouped rows form a dense batched GEMM chain, rows x C0 -> C1 -> C2 then a max
// over rows, which is what the matrix cores are for.  One wave per centre; its rows go through in
// n-tiles of 32 points (padded rows repeat the first hit, exactly the reference's padding, so
// the max is unchanged).
//   layer 1, transposed:  H1^T (C1 x 32) = W1 (C1 x C0) . X^T (C0 x 32)
//        A = W1 fragment (lane: output channel, k-half), B = X^T fragment (lane: point, k-half).
//        D has channels in registers and points on lanes...
//   layer 2:              H2 (32 x C2) = H1 (32 x C1) . W2^T (C1 x C2)
//        ...so each accumulator register of layer 1 is directly a k-step of layer 2's A operand
//        (k pair = channels c, c+4 of the register), no LDS round trip;  D has points in
//        registers and channels on lanes, so the max over points is a per-lane max over
//        registers plus one exchange between lane halves.
// Input channel order per k-step s: lane half 0 takes [x, y, z, f0 .. f(D/2-1)], half 1 takes
// [0, 0, 0, f(D/2) .. f(D-1)], so each half loads one contiguous, 16-B aligned feature run.
// Bias is the accumulator's initial value; BN (eval) is y = acc * scale + shift with scale/shift
// folded on the host side of the kernel (scale, shift of dvcp_sa_group_mlp's params); ReLU.
// Layer 1 runs on the fp32 MFMA (a k-ordered fp32 fma chain).  Layer 2 (~95 % of the flops) runs
// on the bf16 matrix cores, which are 16x the fp32 MFMA rate, with fp32 accuracy kept by a three-way
// split (DVCP_SA_SPLIT3, default on): every fp32 operand is the exact sum of three bf16 pieces
// x = x0 + x1 + x2 (each residual of a round-to-nearest bf16 conversion is exact in fp32), and
//   a.b ~ a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)
// drops only the terms a1 b2, a2 b1, a2 b2 (<= 2^-24 |a||b| together, the size of one fp32
// rounding of the product); the bf16 x bf16 products are exact in the fp32 accumulator.  Six
// v_mfma_f32_32x32x16_bf16 (32 cycles each) replace eight v_mfma_f32_32x32x2_f32 (64 cycles each)
// per 16 channels of k, so layer 2 costs 3/8 of the fp32 MFMA time.  The result differs from
// the fp32 chain by summation order and the dropped terms, within the fp32 tolerances of the
// parity tests (tests/test_gpu_kernels.py: rtol = atol = 1e-5; the split's own error against an
// fp64 evaluation is checked beside the fp32 path's in test_sa_split3_accuracy).
#include "common.h"
#include "morton.h"

namespace dvcp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef DVCP_SA_SPLIT3
#define DVCP_SA_SPLIT3 1
#endif
// DVCP_SA_PACK16: the pre-pass kernel packs each centre's rows in 16-row half tiles (see the kernel)
#ifndef DVCP_SA_PACK16
#define DVCP_SA_PACK16 1
#endif

// x = x0 + x1 + x2 exactly (bf16 pieces of eight fp32 values; see the header)
struct Split3 {
  bf16x8 p0, p1, p2;
};
__device__ __forceinline__ Split3 split3(const float (&x)[8]) {
  Split3 s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 b0 = static_cast<__bf16>(x[j]);
    const float r1 = x[j] - static_cast<float>(b0);
    const __bf16 b1 = static_cast<__bf16>(r1);
    const float r2 = r1 - static_cast<float>(b1);
    s.p0[j] = b0;
    s.p1[j] = b1;
    s.p2[j] = static_cast<__bf16>(r2);
  }
  return s;
}
// acc += a.b over one 16-deep k-step, the six significant piece products, smallest first
__device__ __forceinline__ f32x16 mfma_split3(const Split3& a, const bf16x8& b0, const bf16x8& b1, const bf16x8& b2,
                                             f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p2, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b1, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b0, acc, 0, 0, 0);
}

constexpr int kMfmaWaves = 4;  // centres in flight per workgroup (one per SIMD)

template <int D, int C1, int C2>
struct SaMfmaShape {
  static constexpr int C0 = 3 + D;
  static constexpr int KS = 3 + D / 2;  // k-steps of layer 1
  static constexpr int MT = C1 / 32;    // layer-1 output tiles
  static constexpr int CT = C2 / 32;    // layer-2 output tiles
  static constexpr int K2 = MT * 16;    // k-steps of layer 2 (fp32 32x32x2)
  static constexpr int KB = MT * 2;     // k-steps of layer 2 (bf16 32x32x16, split3)
  static_assert(D % 8 == 0 && C1 % 32 == 0 && C2 % 32 == 0, "MFMA tiling");
};

// LDS image of the weights in fragment order (staged once per workgroup).
template <int D, int C1, int C2, bool PRE>
struct SaMfmaLds {
  using S = SaMfmaShape<D, C1, C2>;
  float w1[PRE ? 1 : S::MT][S::KS][64];  // A fragment of layer 1: [tile][k-step][lane] (not PRE)
  float wx[S::MT][2][64];                // decomposed layer 1: xyz columns only, k-steps (x|y), (z|0)
#if DVCP_SA_SPLIT3
  bf16x8 w2s[S::CT][S::KB][3][64];       // B fragment of layer 2 as three bf16 pieces: [tile][k-step][piece][lane]
#else
  float w2[S::CT][S::K2][64];            // B fragment of layer 2: [tile][k-step][lane]
#endif
  float b1[S::MT][2][16];       // layer-1 bias / BN scale / BN shift by [tile][lane half][register]
  float s1[S::MT][2][16];
  float t1[S::MT][2][16];
};

// channel (index into [xyz, features]) feeding k-step s of lane half h, or -1 (zero)
template <int D>
__device__ __forceinline__ int sa_in_channel(int s, int h) {
  if (s < 3) return h == 0 ? s : -1;
  return 3 + h * (D / 2) + (s - 3);
}

// output channel row of accumulator register r for lane half h (32x32 C/D map)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Decomposed layer 1 (PRE = true).  Layer 1 is linear in its input row [p - c, f]:
//   W1 [p - c; f] + b1 = W1x (p - c) + (W1f f + b1)
// and the second term depends only on the neighbour point, not on the centre.  sa_pre_mfma_kernel
// evaluates U[n] = W1f f_n + b1 once per input point (N rows instead of S x nsample), and the
// grouped kernel starts each layer-1 accumulator from the gathered U row and adds the xyz part
// with two MFMA k-steps.  Only the summation order changes (features first, then xyz); the local
// coordinates are still formed per (centre, point) pair, so no cancellation is introduced.
// The per-point pass is a plain GEMM on the fp32 matrix cores (U = F . W1f'^T + b1'): one wave
// per 32 input points, v_mfma_f32_32x32x2_f32 with k-step s taking input channels s (lane half 0)
// and s + D/2 (half 1), so each lane reads one contiguous half of its point's feature row; the
// BN-folded weights are staged once per workgroup as B fragments; bound by its 82 MB (sa3, C3).
// The accumulation is a k-ordered fp32 chain (the MFMA adds its two k-products per step).
// (Round 4 had a row-per-thread VALU form of this pass, float4 FMA chains that hipcc packed into
// v_pk_fma_f32.  With a second process on the GPU, single fp32 lanes of its accumulators came out
// different -- the round-4 two-rank test failure -- so it was removed.  The cause is not proven:
// DESIGN.md section 5 names the one distinctive sequence, a v_mov-written register broadcast into
// a packed FMA one instruction later, which no shipped kernel contains.)
template <int D, int C1>
__global__ __launch_bounds__(256) void sa_pre_mfma_kernel(const float* __restrict__ feat, int64_t fb, int64_t fn, int N,
                                                          int B, const float* __restrict__ params,
                                                          float* __restrict__ U, const int64_t* __restrict__ rows,
                                                          int Nf) {
  constexpr int C0 = 3 + D, MT = C1 / 32, KS = D / 2;
  static_assert(D % 8 == 0 && C1 % 32 == 0, "MFMA tiling");
  __shared__ float wf[MT][KS][64];  // B fragment: lane (o, h) of k-step s -> s1_o W1[o][3 + s + h D/2]
  __shared__ float bias[C1];         // folded bias (the accumulators' channel is the lane)
  const float* W1 = params;
  const float* pb1 = W1 + C1 * C0;
  const float* ps1 = pb1 + C1;
  const float* pt1 = ps1 + C1;
  for (int i = threadIdx.x; i < MT * KS * 64; i += blockDim.x) {
    const int l = i % 64, s = (i / 64) % KS, mt = i / (64 * KS), o = 32 * mt + (l & 31);
    wf[mt][s][l] = W1[o * C0 + 3 + s + (l >> 5) * (D / 2)] * ps1[o];
  }
  for (int c = threadIdx.x; c < C1; c += blockDim.x)
    bias[c] = static_cast<float>(static_cast<double>(pb1[c]) * ps1[c] + static_cast<double>(pt1[c]));
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, r32 = lane & 31;
  const int64_t total = static_cast<int64_t>(B) * N;
  const int64_t ntiles = (total + 31) / 32;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); t < ntiles;
       t += static_cast<int64_t>(gridDim.x) * 4) {
    // this lane's point (row r32 of the tile) and its half of the feature row
    const int64_t i = t * 32 + r32;
    const int64_t ic = i < total ? i : total - 1;
    const int b = static_cast<int>(ic / N), n = static_cast<int>(ic % N);
    int64_t src = n;
    if (rows) {
      const int64_t r = rows[ic];
      src = r < 0 ? 0 : (r >= Nf ? Nf - 1 : r);
    }
    const float4* fr = reinterpret_cast<const float4*>(feat + b * fb + src * fn + h * (D / 2));
    float x[KS];
#pragma unroll
    for (int v = 0; v < KS / 4; ++v) {
      const float4 q = fr[v];
      x[4 * v] = q.x;
      x[4 * v + 1] = q.y;
      x[4 * v + 2] = q.z;
      x[4 * v + 3] = q.w;
    }
    int zo = 0;  // opaque zero: the fragments are read per tile, not hoisted into registers
    asm volatile("" : "+v"(zo));
    f32x16 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const float bc = bias[32 * mt + r32 + zo];
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][r] = bc;
    }
    // H (32 points x C1): A = the feature rows (lane = point), B = the weight fragments (lane = channel)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s], wf[mt][s][lane + zo], acc[mt], 0, 0, 0);
    // D[point][channel]: lane = channel, register r = point acc_row(r, h)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t ip = t * 32 + acc_row(r, h);
      if (ip < total)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) U[ip * C1 + 32 * mt + r32] = acc[mt][r];
    }
  }
}

// Centres of each cloud in 12-bit Hilbert-cell order (one workgroup per cloud), for the MFMA
// kernel's visiting order.  The order changes only which wave computes which centre.
template <typename T>
__global__ __launch_bounds__(kBuildThreads) void sa_order_kernel(PointsView<T> ctr, int S, int32_t* __restrict__ order) {
  __shared__ uint32_t bins[kSortBins];
  __shared__ uint32_t wsum[16];
  __shared__ float red[2][3][16];
  const int b = blockIdx.x;
  auto get = [&](int i, float (&v)[3]) {
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] = static_cast<float>(ctr.at(b, a, i));
  };
  float lo[3], hi[3];
  block_bbox(S, get, lo, hi, red);
  int32_t* o = order + static_cast<int64_t>(b) * S;
  morton_sort(S, get, [&](int pos, int i, const float (&)[3]) { o[pos] = i; }, lo, hi, bins, wsum);
}

template <typename T, int D, int C1, int C2, bool PRE, bool PACK = false>
__global__ __launch_bounds__(kMfmaWaves * kWave) __attribute__((amdgpu_waves_per_eu(3))) void sa_mlp_mfma_kernel(
    PointsView<T> pts, PointsView<T> ctr, int S, int B, const float* __restrict__ feat, int64_t fb, int64_t fn,
    const int32_t* __restrict__ count, const int32_t* __restrict__ list, int nsample,
    const float* __restrict__ params, const float* __restrict__ U, int64_t ub, const int32_t* __restrict__ order,
    float* __restrict__ out, int xcd) {
  using Sh = SaMfmaShape<D, C1, C2>;
  constexpr int C0 = Sh::C0, KS = Sh::KS, MT = Sh::MT, CT = Sh::CT;
  __shared__ SaMfmaLds<D, C1, C2, PRE> L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;

  // ---- stage the weights (params: W1, b1, scale1, shift1, W2, b2, scale2, shift2) ---------
  const float* W1 = params;
  const float* pb1 = W1 + C1 * C0;
  const float* ps1 = pb1 + C1;
  const float* pt1 = ps1 + C1;
  const float* W2 = pt1 + C1;
  const float* pb2 = W2 + C2 * C1;
  const float* ps2 = pb2 + C2;
  const float* pt2 = ps2 + C2;
  if (!PRE)
    for (int i = tid; i < MT * KS * 64; i += blockDim.x) {
      const int l = i % 64, s = (i / 64) % KS, mt = i / (64 * KS);
      const int ch = sa_in_channel<D>(s, l >> 5);
      L.w1[mt][s][l] = ch < 0 ? 0.0f : W1[(32 * mt + (l & 31)) * C0 + ch];
    }
  if (PRE)
    for (int i = tid; i < MT * 2 * 64; i += blockDim.x) {
      const int l = i % 64, s = (i / 64) % 2, mt = i / 128;
      const int ch = s == 0 ? (l >> 5) : ((l >> 5) == 0 ? 2 : -1);
      L.wx[mt][s][l] = ch < 0 ? 0.0f : W1[(32 * mt + (l & 31)) * C0 + ch] * ps1[32 * mt + (l & 31)];
    }
#if DVCP_SA_SPLIT3
  // k-step s, lane half hh, element j <-> layer-1 channel 32 (s / 2) + acc_row(8 (s % 2) + j, hh): the
  // layer-1 accumulator registers 8 (s % 2) .. + 7 of tile s / 2 are the A fragment as they stand
  for (int i = tid; i < CT * Sh::KB * 64; i += blockDim.x) {
    const int l = i % 64, s = (i / 64) % Sh::KB, ct = i / (64 * Sh::KB);
    const int o = 32 * ct + (l & 31);
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      w[j] = W2[o * C1 + 32 * (s / 2) + acc_row(8 * (s % 2) + j, l >> 5)] * (PRE ? ps2[o] : 1.0f);
    const Split3 ws = split3(w);
    L.w2s[ct][s][0][l] = ws.p0;
    L.w2s[ct][s][1][l] = ws.p1;
    L.w2s[ct][s][2][l] = ws.p2;
  }
#else
  for (int i = tid; i < CT * Sh::K2 * 64; i += blockDim.x) {
    const int l = i % 64, kk = (i / 64) % Sh::K2, ct = i / (64 * Sh::K2);
    const int mt = kk / 16, r = kk % 16;
    L.w2[ct][kk][l] = W2[(32 * ct + (l & 31)) * C1 + 32 * mt + acc_row(r, l >> 5)] * (PRE ? ps2[32 * ct + (l & 31)] : 1.0f);
  }
#endif
  for (int i = tid; i < MT * 32; i += blockDim.x) {
    const int r = i % 16, hh = (i / 16) % 2, mt = i / 32;
    const int c = 32 * mt + acc_row(r, hh);
    L.b1[mt][hh][r] = pb1[c];
    L.s1[mt][hh][r] = ps1[c];
    L.t1[mt][hh][r] = pt1[c];
  }
  float b2[CT], s2[CT], t2[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    b2[ct] = pb2[32 * ct + r32];
    s2[ct] = ps2[32 * ct + r32];
    t2[ct] = pt2[32 * ct + r32];
    // PRE: BN2 folded into W2 (above) and the bias: (W h + b) s + t = (s W) h + (s b + t)
    if (PRE) b2[ct] = static_cast<float>(static_cast<double>(b2[ct]) * s2[ct] + static_cast<double>(t2[ct]));
  }
  __syncthreads();

  // ---- one centre per wave, grid-strided ------------------------------------------------
  // Centre index space.  xcd == 0: all B*S centres.  xcd != 0 (B % 8 == 0, grid a multiple of 8):
  // workgroups reach the 8 XCDs round robin (blockIdx % 8), so XCD x walks the centres of clouds
  // x, x + 8, ... and each cloud's U table and point rows are fetched into one XCD's L2.
  int64_t total, q0, qs;
  int xo = 0;
  if (xcd) {
    xo = static_cast<int>(blockIdx.x) & 7;
    total = static_cast<int64_t>((B - xo + 7) / 8) * S;
    q0 = static_cast<int64_t>(blockIdx.x >> 3) * kMfmaWaves + wave;
    qs = static_cast<int64_t>(gridDim.x >> 3) * kMfmaWaves;
  } else {
    total = static_cast<int64_t>(B) * S;
    q0 = static_cast<int64_t>(blockIdx.x) * kMfmaWaves + wave;
    qs = static_cast<int64_t>(gridDim.x) * kMfmaWaves;
  }
  // The wave's centres are ql = q0, q0 + qs, ...: their metadata (order, count, centre) is
  // loaded 64 centres at a time, one per lane, and read back by readlane, so a centre's first
  // tile waits only for its list entries (fetched one tile ahead) and its U rows.
  auto lane_bcast = [](auto v, int j) {
    if constexpr (sizeof(v) == 8) {
      const int64_t u = __builtin_bit_cast(int64_t, v);
      const int lo = __builtin_amdgcn_readlane(static_cast<int>(u & 0xFFFFFFFF), j);
      const int hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), j);
      return __builtin_bit_cast(decltype(v), (static_cast<int64_t>(hi) << 32) | static_cast<uint32_t>(lo));
    } else {
      return __builtin_bit_cast(decltype(v), __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
    }
  };
  for (int64_t qc = q0; qc < total; qc += 64 * qs) {
    const int64_t qm = qc + lane * qs;
    int m_b = 0, m_rows = 0;  // rows 0: no hit (the centre's output is 0)
    int64_t m_fc = 0;
    T m_cx = T(0), m_cy = T(0), m_cz = T(0);
    if (qm < total) {
      const int64_t q = xcd ? (xo + 8 * (qm / S)) * static_cast<int64_t>(S) + qm % S : qm;
      // centre in curve order when `order` is given: consecutive waves then gather the U / point
      // rows of one spatial neighbourhood, which stay in L2 instead of being fetched again
      m_b = static_cast<int>(q / S);
      const int c = order ? order[q] : static_cast<int>(q % S);
      m_fc = static_cast<int64_t>(m_b) * S + c;
      const int r = count[m_fc];
      m_rows = r < 1 ? 0 : (r > nsample ? nsample : r);
      ctr.load3(m_b, c, m_cx, m_cy, m_cz);
    }
    const int ncen = static_cast<int>(min<int64_t>(64, (total - qc + qs - 1) / qs));
    // list entry of this lane's point in the next tile to run (centre j, tile n0)
    auto list_entry = [&](int j, int n0) {
      const int64_t fcj = lane_bcast(m_fc, j);
      const int rj = lane_bcast(m_rows, j);
      const int row = n0 + r32;
      return rj == 0 ? 0 : list[fcj * nsample + (row < rj ? row : 0)];
    };
    constexpr bool BZ = PRE && DVCP_SA_SPLIT3;
    if constexpr (PACK) {
      static_assert(!PACK || (PRE && DVCP_SA_SPLIT3), "row packing runs on the split-3 pre-pass path");
      // Rows in 16-row half tiles: a tile takes the next two half tiles of the wave's centres in
      // order (rows 0-15 are accumulator registers 0..7 of both lane halves, rows 16-31 registers
      // 8..15), so a centre wastes at most 15 padded rows instead of 31, and the two halves' maxima
      // fold into running per-centre maxima in order.  Padded rows repeat the centre's first hit.
      int js = 0, hs = 0;  // the next half tile: centre js, half hs
      auto nh_of = [&](int jj) { return max(1, (lane_bcast(m_rows, jj) + 15) >> 4); };
      int nhj = ncen > 0 ? nh_of(0) : 0;
      int runj = -1;
      float run[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) run[ct] = 0.0f;
      auto flush = [&]() {
        const int64_t fcr = lane_bcast(m_fc, runj);
        const bool empty = lane_bcast(m_rows, runj) == 0;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          if (h == 0) out[fcr * C2 + 32 * ct + r32] = empty ? 0.0f : fmaxf(run[ct] + b2[ct], 0.0f);
      };
      auto fold = [&](int jj, const float (&m)[CT]) {
        if (jj != runj) {
          if (runj >= 0) flush();
          runj = jj;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) run[ct] = m[ct];
        } else {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) run[ct] = fmaxf(run[ct], m[ct]);
        }
      };
      while (js < ncen) {
        const int jA = js, hA = hs;
        if (++hs >= nhj) {
          hs = 0;
          if (++js < ncen) nhj = nh_of(js);
        }
        const bool hasB = js < ncen;
        const int jB = hasB ? js : jA, hB = hasB ? hs : hA;
        if (hasB && ++hs >= nhj) {
          hs = 0;
          if (++js < ncen) nhj = nh_of(js);
        }
        int zo = 0;
        asm volatile("" : "+v"(zo));
        const bool sB = r32 >= 16;  // this lane's point: row r32 of the tile
        const int b = sB ? lane_bcast(m_b, jB) : lane_bcast(m_b, jA);
        const int64_t fc = sB ? lane_bcast(m_fc, jB) : lane_bcast(m_fc, jA);
        const int rows = sB ? lane_bcast(m_rows, jB) : lane_bcast(m_rows, jA);
        const T cx = sB ? lane_bcast(m_cx, jB) : lane_bcast(m_cx, jA);
        const T cy = sB ? lane_bcast(m_cy, jB) : lane_bcast(m_cy, jA);
        const T cz = sB ? lane_bcast(m_cz, jB) : lane_bcast(m_cz, jA);
        const int row = 16 * (sB ? hB : hA) + (r32 & 15);
        const int n = rows == 0 ? 0 : list[fc * nsample + (row < rows ? row : 0)];
        f32x16 acc1[MT];
        const float4* ur = reinterpret_cast<const float4*>(U + b * ub + static_cast<int64_t>(n) * C1 + 4 * h);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 u = ur[8 * mt + 2 * i];
            acc1[mt][4 * i] = u.x;
            acc1[mt][4 * i + 1] = u.y;
            acc1[mt][4 * i + 2] = u.z;
            acc1[mt][4 * i + 3] = u.w;
          }
        // (points in packed (x, y, z, pad) rows measured no faster here -- sa2 0.298 -> 0.306, sa3
        // 0.594 -> 0.597 ms, r5ae_sa_p4_bench.log: the U rows dominate the gather -- so the FE passes
        // the (B, 3, N) layout; load3 takes either)
        T px, py, pz;
        pts.load3(b, n, px, py, pz);
        const float dx = static_cast<float>(px - cx);
        const float dy = static_cast<float>(py - cy);
        const float dz = static_cast<float>(pz - cz);
        const float x0 = h == 0 ? dx : dy, x1 = h == 0 ? dz : 0.0f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[mt][0][lane + zo], x0, acc1[mt], 0, 0, 0);
          acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[mt][1][lane + zo], x1, acc1[mt], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 16; ++r) acc1[mt][r] = acc1[mt][r] > 0.0f ? acc1[mt][r] : 0.0f;
        }
        f32x16 acc2[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc2[ct][r] = 0.0f;
#pragma unroll
        for (int st = 0; st < Sh::KB; ++st) {
          float x[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) x[jj] = acc1[st / 2][8 * (st % 2) + jj];
          const Split3 a = split3(x);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            acc2[ct] = mfma_split3(a, L.w2s[ct][st][0][lane + zo], L.w2s[ct][st][1][lane + zo],
                                   L.w2s[ct][st][2][lane + zo], acc2[ct]);
        }
        float mA[CT], mB[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          float a0 = acc2[ct][0], a1 = acc2[ct][8];
#pragma unroll
          for (int r = 1; r < 8; ++r) {
            a0 = fmaxf(a0, acc2[ct][r]);
            a1 = fmaxf(a1, acc2[ct][8 + r]);
          }
          mA[ct] = fmaxf(a0, __shfl_xor(a0, 32, kWave));
          mB[ct] = fmaxf(a1, __shfl_xor(a1, 32, kWave));
        }
        fold(jA, mA);
        if (hasB) fold(jB, mB);
      }
      if (runj >= 0) flush();
      continue;
    }
    // The first list row of the next centre is fetched one tile ahead; a centre without hits runs
    // no tile, so "next" is the next centre with hits (lane mask of the batch).
    const uint64_t live_c = __ballot(lane < ncen && m_rows > 0);
    auto next_live = [&](int j) {  // the first centre after j with hits, or 64
      const uint64_t m = j >= 63 ? 0ull : (live_c & (~0ull << (j + 1)));
      return m ? static_cast<int>(__builtin_ctzll(m)) : 64;
    };
    int n_next = 0;
    {
      const int j0 = (live_c & 1ull) ? 0 : next_live(0);
      if (j0 < ncen) n_next = list_entry(j0, 0);
    }
  for (int j = 0; j < ncen; ++j) {
    const int b = lane_bcast(m_b, j);
    const int64_t fc = lane_bcast(m_fc, j);
    const int rows = lane_bcast(m_rows, j);
    const T cx = lane_bcast(m_cx, j), cy = lane_bcast(m_cy, j), cz = lane_bcast(m_cz, j);
    // PRE with the split layer 2 (BZ): the accumulators start from zero (an inline-constant C
    // operand, no 32 register moves per tile) and the bias is added once to the maximum:
    // max_i fl(a_i + b) = fl(max_i a_i + b) (rounding is monotone), then the ReLU.
    float mx[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) mx[ct] = BZ ? -__builtin_huge_valf() : 0.0f;  // else post-ReLU values are >= +0

    for (int n0 = 0; n0 < rows; n0 += 32) {
      // An opaque zero added to every LDS weight index: the fragments are re-read per tile
      // (one ds_read per MFMA) instead of being hoisted out of the loop into ~100 registers,
      // which would cap occupancy at 2 waves per SIMD.
      int zo = 0;
      asm volatile("" : "+v"(zo));
      // B fragment of layer 1: this lane's point (r32) and its half of the input channels
      const int n = n_next;
      if (n0 + 32 < rows)
        n_next = list_entry(j, n0 + 32);
      else if (next_live(j) < ncen)
        n_next = list_entry(next_live(j), 0);
      f32x16 acc1[MT];
      if constexpr (PRE) {
        // accumulators start from U[n] (channels (r&3) + 8(r>>2) + 4h of each 32-channel tile)
        const float4* ur = reinterpret_cast<const float4*>(U + b * ub + static_cast<int64_t>(n) * C1 + 4 * h);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 u = ur[8 * mt + 2 * i];
            acc1[mt][4 * i] = u.x;
            acc1[mt][4 * i + 1] = u.y;
            acc1[mt][4 * i + 2] = u.z;
            acc1[mt][4 * i + 3] = u.w;
          }
        T px, py, pz;
        pts.load3(b, n, px, py, pz);
        const float dx = static_cast<float>(px - cx);
        const float dy = static_cast<float>(py - cy);
        const float dz = static_cast<float>(pz - cz);
        const float x0 = h == 0 ? dx : dy, x1 = h == 0 ? dz : 0.0f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[mt][0][lane + zo], x0, acc1[mt], 0, 0, 0);
          acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.wx[mt][1][lane + zo], x1, acc1[mt], 0, 0, 0);
        }
      } else {
        float x[KS];
        if (h == 0) {
          x[0] = static_cast<float>(pts.at(b, 0, n) - cx);
          x[1] = static_cast<float>(pts.at(b, 1, n) - cy);
          x[2] = static_cast<float>(pts.at(b, 2, n) - cz);
        } else {
          x[0] = x[1] = x[2] = 0.0f;
        }
        const float4* fr = reinterpret_cast<const float4*>(feat + b * fb + static_cast<int64_t>(n) * fn + h * (D / 2));
#pragma unroll
        for (int v = 0; v < D / 8; ++v) {
          const float4 f = fr[v];
          x[3 + 4 * v] = f.x;
          x[4 + 4 * v] = f.y;
          x[5 + 4 * v] = f.z;
          x[6 + 4 * v] = f.w;
        }
        // layer 1 (transposed): acc1[mt] rows = output channels, columns = points
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc1[mt][r] = L.b1[mt][h][r + zo];
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(L.w1[mt][s][lane + zo], x[s], acc1[mt], 0, 0, 0);
      }
      // BN (eval) + ReLU in place (PRE: BN already folded into U and W1x)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = PRE ? acc1[mt][r] : acc1[mt][r] * L.s1[mt][h][r + zo] + L.t1[mt][h][r + zo];
          acc1[mt][r] = v > 0.0f ? v : 0.0f;
        }
      // layer 2: A operand = the layer-1 registers, B = W2^T fragments
      f32x16 acc2[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[ct][r] = BZ ? 0.0f : b2[ct];
#if DVCP_SA_SPLIT3
#pragma unroll
      for (int s = 0; s < Sh::KB; ++s) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = acc1[s / 2][8 * (s % 2) + j];
        const Split3 a = split3(x);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          acc2[ct] = mfma_split3(a, L.w2s[ct][s][0][lane + zo], L.w2s[ct][s][1][lane + zo], L.w2s[ct][s][2][lane + zo],
                                 acc2[ct]);
      }
#else
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            acc2[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(acc1[mt][r], L.w2[ct][mt * 16 + r][lane + zo], acc2[ct], 0, 0, 0);
#endif
      // BN + ReLU, then max over this tile's points (registers).  PRE: BN is folded, and
      // max_i relu(v_i) = relu(max_i v_i), so the ReLU is the +0 the running max starts from.
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (PRE) {
            mx[ct] = fmaxf(mx[ct], acc2[ct][r]);
          } else {
            const float v = acc2[ct][r] * s2[ct] + t2[ct];
            mx[ct] = fmaxf(mx[ct], v > 0.0f ? v : 0.0f);
          }
        }
    }
    // the two lane halves hold different points of the same channel
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float m = fmaxf(mx[ct], __shfl_xor(mx[ct], 32, kWave));
      if (BZ) m = fmaxf(m + b2[ct], 0.0f);
      if (h == 0) out[fc * C2 + 32 * ct + r32] = m;
    }
  }
  }
}

// ---------------------------------------------------------------------------------------------
// The three-layer table (sa1: 3-16-16-32 on xyz, 6-16-16-32 with normals; deep_feat_extraction.py:19,
// pointnet2_utils.py:122-132 + :195-200) on the matrix cores.  The row-per-thread kernel
// (sa_mlp.hip) spends ~816 fp32 FMAs and 32 LDS atomics per grouped row; here a wave takes 32 rows
// (two 16-row half tiles, as the two-layer kernel's PACK path) through three chained MFMAs whose
// accumulators feed the next layer in place:
//   layer 1, fp32 32x32x2:       H1^T (32 ch x 32 rows) = W1 (32 x C0) . X^T, channels 16..31 zero
//        (A: lane = output channel, one input channel per lane half and k-step; B: lane = row)
//   layer 2, bf16 32x32x16 x 6:  H2^T = W2 (32 x 16) . H1^T -- the B operand (lane = row, k in
//        registers) is layer 1's accumulator registers 0..7 as they stand: k-slot 8h + r of lane
//        half h is channel acc_row(r, h); W2's A fragment is stored in that channel order
//   layer 3, bf16 32x32x16 x 6:  H3 (32 rows x 32 ch) = H2 . W3^T -- the A operand (lane = row, k
//        in registers) is again layer 2's registers 0..7, W3^T's B fragment in the same order
// Layer 3's accumulator has channels on lanes and rows in registers: rows 0-15 (the first half
// tile) are registers 0..7 of both lane halves, rows 16-31 registers 8..15, so each half tile's
// maximum is a per-lane max plus one exchange between lane halves.  BN (eval) is folded into the
// weights and biases, (W x + b) s + t = (s W) x + (s b + t); layer 3's bias and ReLU go after the
// maximum (max_i fl(a_i + b) = fl(max_i a_i + b), rounding is monotone).  Layers 2 and 3 keep fp32
// accuracy through the three-way bf16 split of the header.  A centre without hits (count < 1:
// the reference would gather index N, :104) gets zeros, as the row-per-thread kernel gives it.
struct Sa3Lds {
  float w1[3][64];   // layer-1 A fragment per k-step: lane (o, kh) -> s1_o W1[o][2 s + kh]  (o < 16)
  bf16x8 w2[3][64];  // layer-2 A fragment pieces: lane (o, kh), element r -> s2_o W2[o][acc_row(r, kh)]
  bf16x8 w3[3][64];  // layer-3 B fragment pieces: lane (o, kh), element r -> s3_o W3[o][acc_row(r, kh)]
  float b1[2][8];    // folded biases of layers 1, 2 by [lane half][accumulator register]
  float b2[2][8];
};

template <typename T, typename FT, int D>
__global__ __launch_bounds__(kMfmaWaves * kWave) void sa3_mfma_kernel(
    PointsView<T> pts, PointsView<T> ctr, int S, int B, const FT* __restrict__ feat, int64_t fb, int64_t fd, int64_t fn,
    const int32_t* __restrict__ count, const int32_t* __restrict__ list, int nsample, const float* __restrict__ params,
    float* __restrict__ out, int xcd) {
  constexpr int C0 = 3 + D, C1 = 16, C2 = 16, C3 = 32;
  constexpr int KS = (C0 + 1) / 2;  // layer-1 k-steps: input channels (2 s, 2 s + 1) on lane halves (0, 1)
  static_assert(D == 0 || D == 3, "sa1 tables");
  __shared__ Sa3Lds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const float* W1 = params;
  const float* pb1 = W1 + C1 * C0;
  const float* ps1 = pb1 + C1;
  const float* pt1 = ps1 + C1;
  const float* W2 = pt1 + C1;
  const float* pb2 = W2 + C2 * C1;
  const float* ps2 = pb2 + C2;
  const float* pt2 = ps2 + C2;
  const float* W3 = pt2 + C2;
  const float* pb3 = W3 + C3 * C2;
  const float* ps3 = pb3 + C3;
  const float* pt3 = ps3 + C3;
  auto fold_bias = [](float b, float s, float t) {
    return static_cast<float>(static_cast<double>(b) * s + static_cast<double>(t));
  };
  for (int i = tid; i < KS * 64; i += blockDim.x) {
    const int l = i % 64, s = i / 64, o = l & 31, c = 2 * s + (l >> 5);
    L.w1[s][l] = (o < C1 && c < C0) ? W1[o * C0 + c] * ps1[o] : 0.0f;
  }
  if (tid < 64) {
    const int o = tid & 31, kh = tid >> 5;
    float a[8], w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a[r] = o < C2 ? W2[o * C1 + acc_row(r, kh)] * ps2[o] : 0.0f;
      w[r] = W3[o * C2 + acc_row(r, kh)] * ps3[o];
    }
    const Split3 sa = split3(a), sw = split3(w);
    L.w2[0][tid] = sa.p0;
    L.w2[1][tid] = sa.p1;
    L.w2[2][tid] = sa.p2;
    L.w3[0][tid] = sw.p0;
    L.w3[1][tid] = sw.p1;
    L.w3[2][tid] = sw.p2;
  } else if (tid < 80) {
    const int kh = (tid - 64) >> 3, r = tid & 7, c = acc_row(r, kh);
    L.b1[kh][r] = fold_bias(pb1[c], ps1[c], pt1[c]);
    L.b2[kh][r] = fold_bias(pb2[c], ps2[c], pt2[c]);
  }
  const float b3 = fold_bias(pb3[r32], ps3[r32], pt3[r32]);
  __syncthreads();

  // centres grid-strided as in sa_mlp_mfma_kernel (xcd != 0: XCD x walks clouds x, x + 8, ...)
  int64_t total, q0, qs;
  int xo = 0;
  if (xcd) {
    xo = static_cast<int>(blockIdx.x) & 7;
    total = static_cast<int64_t>((B - xo + 7) / 8) * S;
    q0 = static_cast<int64_t>(blockIdx.x >> 3) * kMfmaWaves + wave;
    qs = static_cast<int64_t>(gridDim.x >> 3) * kMfmaWaves;
  } else {
    total = static_cast<int64_t>(B) * S;
    q0 = static_cast<int64_t>(blockIdx.x) * kMfmaWaves + wave;
    qs = static_cast<int64_t>(gridDim.x) * kMfmaWaves;
  }
  auto lane_bcast = [](auto v, int j) {
    if constexpr (sizeof(v) == 8) {
      const int64_t u = __builtin_bit_cast(int64_t, v);
      const int lo = __builtin_amdgcn_readlane(static_cast<int>(u & 0xFFFFFFFF), j);
      const int hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), j);
      return __builtin_bit_cast(decltype(v), (static_cast<int64_t>(hi) << 32) | static_cast<uint32_t>(lo));
    } else {
      return __builtin_bit_cast(decltype(v), __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
    }
  };
  for (int64_t qc = q0; qc < total; qc += 64 * qs) {
    // this lane's centre of the next 64: cloud, flat index, rows (0: no hit), coordinates
    const int64_t qm = qc + lane * qs;
    int m_b = 0, m_rows = 0;
    int64_t m_fc = 0;
    T m_cx = T(0), m_cy = T(0), m_cz = T(0);
    if (qm < total) {
      const int64_t q = xcd ? (xo + 8 * (qm / S)) * static_cast<int64_t>(S) + qm % S : qm;
      m_b = static_cast<int>(q / S);
      m_fc = q;
      const int r = count[q];
      m_rows = r < 0 ? 0 : (r > nsample ? nsample : r);
      const int c = static_cast<int>(q % S);
      ctr.load3(m_b, c, m_cx, m_cy, m_cz);
    }
    const int ncen = static_cast<int>(min<int64_t>(64, (total - qc + qs - 1) / qs));
    int js = 0, hs = 0;  // the next half tile: centre js, half hs
    auto nh_of = [&](int jj) { return max(1, (lane_bcast(m_rows, jj) + 15) >> 4); };
    int nhj = ncen > 0 ? nh_of(0) : 0;
    int runj = -1;
    float run = 0.0f;
    auto flush = [&]() {
      const int64_t fcr = lane_bcast(m_fc, runj);
      const bool empty = lane_bcast(m_rows, runj) == 0;
      if (h == 0) out[fcr * C3 + r32] = empty ? 0.0f : fmaxf(run + b3, 0.0f);
    };
    auto fold = [&](int jj, float m) {
      if (jj != runj) {
        if (runj >= 0) flush();
        runj = jj;
        run = m;
      } else {
        run = fmaxf(run, m);
      }
    };
    while (js < ncen) {
      const int jA = js, hA = hs;
      if (++hs >= nhj) {
        hs = 0;
        if (++js < ncen) nhj = nh_of(js);
      }
      const bool hasB = js < ncen;
      const int jB = hasB ? js : jA, hB = hasB ? hs : hA;
      if (hasB && ++hs >= nhj) {
        hs = 0;
        if (++js < ncen) nhj = nh_of(js);
      }
      // opaque zero on the LDS indices: fragments re-read per tile, not hoisted into registers
      int zo = 0;
      asm volatile("" : "+v"(zo));
      const bool sB = r32 >= 16;  // this lane's row r32 of the tile: first or second half tile
      const int b = sB ? lane_bcast(m_b, jB) : lane_bcast(m_b, jA);
      const int64_t fc = sB ? lane_bcast(m_fc, jB) : lane_bcast(m_fc, jA);
      const int rows = sB ? lane_bcast(m_rows, jB) : lane_bcast(m_rows, jA);
      const T cx = sB ? lane_bcast(m_cx, jB) : lane_bcast(m_cx, jA);
      const T cy = sB ? lane_bcast(m_cy, jB) : lane_bcast(m_cy, jA);
      const T cz = sB ? lane_bcast(m_cz, jB) : lane_bcast(m_cz, jA);
      const int row = 16 * (sB ? hB : hA) + (r32 & 15);
      // padded rows repeat the first hit (:104-106); a centre without hits reads point 0 (discarded)
      const int n = rows == 0 ? 0 : list[fc * nsample + (row < rows ? row : 0)];
      T px, py, pz;
      pts.load3(b, n, px, py, pz);
      const float dx = static_cast<float>(px - cx);
      const float dy = static_cast<float>(py - cy);
      const float dz = static_cast<float>(pz - cz);
      float x[KS];
      x[0] = h == 0 ? dx : dy;
      if constexpr (D == 0) {
        x[1] = h == 0 ? dz : 0.0f;
      } else {
        const FT* f = feat + b * fb + static_cast<int64_t>(n) * fn;
        x[1] = h == 0 ? dz : static_cast<float>(f[0]);
        x[2] = static_cast<float>(h == 0 ? f[fd] : f[2 * fd]);
      }
      f32x16 a1;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        a1[r] = L.b1[h][r + zo];
        a1[8 + r] = 0.0f;
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(L.w1[s][lane + zo], x[s], a1, 0, 0, 0);
      float v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = fmaxf(a1[r], 0.0f);
      const Split3 p1 = split3(v);
      f32x16 a2;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        a2[r] = L.b2[h][r + zo];
        a2[8 + r] = 0.0f;
      }
      const Split3 w2{L.w2[0][lane + zo], L.w2[1][lane + zo], L.w2[2][lane + zo]};
      a2 = mfma_split3(w2, p1.p0, p1.p1, p1.p2, a2);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = fmaxf(a2[r], 0.0f);
      const Split3 p2 = split3(v);
      f32x16 a3;
#pragma unroll
      for (int r = 0; r < 16; ++r) a3[r] = 0.0f;
      a3 = mfma_split3(p2, L.w3[0][lane + zo], L.w3[1][lane + zo], L.w3[2][lane + zo], a3);
      float mA = a3[0], mB = a3[8];
#pragma unroll
      for (int r = 1; r < 8; ++r) {
        mA = fmaxf(mA, a3[r]);
        mB = fmaxf(mB, a3[8 + r]);
      }
      mA = fmaxf(mA, __shfl_xor(mA, 32, kWave));
      mB = fmaxf(mB, __shfl_xor(mB, 32, kWave));
      fold(jA, mA);
      if (hasB) fold(jB, mB);
    }
    if (runj >= 0) flush();
  }
}

#ifndef DVCP_SA_GRID
#define DVCP_SA_GRID 4096
#endif
constexpr int kSaGrid = DVCP_SA_GRID;  // workgroups of the grid-strided centre loops (a multiple of 8)

template <typename T, typename FT, int D>
int launch_sa3_mfma(const void* xyz, int64_t sb, int64_t sc, int64_t sn, const void* c, int64_t cb, int64_t cc,
                    int64_t cn, int S, int B, const void* feat, int64_t fb, int64_t fd, int64_t fn, const int32_t* count,
                    const int32_t* list, int nsample, const float* params, float* out, hipStream_t st) {
  PointsView<T> pv{static_cast<const T*>(xyz), sb, sc, sn};
  PointsView<T> cv{static_cast<const T*>(c), cb, cc, cn};
  const int64_t centres = static_cast<int64_t>(B) * S;
  const int grid = static_cast<int>(centres < kSaGrid * kMfmaWaves ? (centres + kMfmaWaves - 1) / kMfmaWaves : kSaGrid);
  const int xcd = B % 8 == 0 && grid % 8 == 0 ? 1 : 0;
  hipLaunchKernelGGL((sa3_mfma_kernel<T, FT, D>), dim3(grid), dim3(kMfmaWaves * kWave), 0, st, pv, cv, S, B,
                     static_cast<const FT*>(feat), fb, fd, fn, count, list, nsample, params, out, xcd);
  return launch_status("dvcp_sa_group_mlp(mfma3)");
}

#define DVCP_SA3_MFMA_INST(T, FT, D)                                                                              \
  template int launch_sa3_mfma<T, FT, D>(const void*, int64_t, int64_t, int64_t, const void*, int64_t, int64_t,  \
                                         int64_t, int, int, const void*, int64_t, int64_t, int64_t, const int32_t*, \
                                         const int32_t*, int, const float*, float*, hipStream_t);
DVCP_SA3_MFMA_INST(float, float, 0)
DVCP_SA3_MFMA_INST(float, double, 0)
DVCP_SA3_MFMA_INST(double, float, 0)
DVCP_SA3_MFMA_INST(double, double, 0)
DVCP_SA3_MFMA_INST(float, float, 3)
DVCP_SA3_MFMA_INST(float, double, 3)
DVCP_SA3_MFMA_INST(double, float, 3)
DVCP_SA3_MFMA_INST(double, double, 3)
#undef DVCP_SA3_MFMA_INST

template <typename T, int D, int C1, int C2>
int launch_sa_mfma(const void* xyz, int64_t sb, int64_t sc, int64_t sn, int N, const void* c, int64_t cb, int64_t cc,
                   int64_t cn, int S, int B, const float* feat, int64_t fb, int64_t fn, const int32_t* count,
                   const int32_t* list, int nsample, const float* params, float* U, int32_t* order, float* out,
                   const int64_t* frows, int Nf, hipStream_t st) {
  PointsView<T> pv{static_cast<const T*>(xyz), sb, sc, sn};
  PointsView<T> cv{static_cast<const T*>(c), cb, cc, cn};
  const int64_t centres = static_cast<int64_t>(B) * S;
  const int grid = static_cast<int>(centres < kSaGrid * kMfmaWaves ? (centres + kMfmaWaves - 1) / kMfmaWaves : kSaGrid);
  const int xcd = B % 8 == 0 && grid % 8 == 0 ? 1 : 0;
  if (order)
    hipLaunchKernelGGL((sa_order_kernel<T>), dim3(B), dim3(kBuildThreads), 0, st, cv, S, order);
  if (U) {
    const int64_t rows = static_cast<int64_t>(B) * N;
    const int64_t wgs = (rows + 127) / 128;  // four 32-point tiles per workgroup
    hipLaunchKernelGGL((sa_pre_mfma_kernel<D, C1>), dim3(static_cast<unsigned>(wgs < 2048 ? wgs : 2048)), dim3(256), 0,
                       st, feat, fb, fn, N, B, params, U, frows, Nf);
    // 16-row half tiles for sa2 only: A/B on one box (tools/sa_bench.py, r4q) sa2 0.312 -> 0.299 ms, sa3
    // 0.626 -> 0.659 ms (its balls mostly fill whole 32-row tiles; the half-tile bookkeeping costs more)
    if constexpr (DVCP_SA_PACK16 && DVCP_SA_SPLIT3 && D == 32)
      hipLaunchKernelGGL((sa_mlp_mfma_kernel<T, D, C1, C2, true, DVCP_SA_PACK16 && DVCP_SA_SPLIT3>), dim3(grid),
                         dim3(kMfmaWaves * kWave), 0, st, pv, cv, S, B, feat, fb, fn, count, list, nsample, params, U,
                         static_cast<int64_t>(N) * C1, order, out, xcd);
    else
      hipLaunchKernelGGL((sa_mlp_mfma_kernel<T, D, C1, C2, true>), dim3(grid), dim3(kMfmaWaves * kWave), 0, st, pv, cv,
                         S, B, feat, fb, fn, count, list, nsample, params, U, static_cast<int64_t>(N) * C1, order, out, xcd);
  } else {
    hipLaunchKernelGGL((sa_mlp_mfma_kernel<T, D, C1, C2, false>), dim3(grid), dim3(kMfmaWaves * kWave), 0, st, pv,
                       cv, S, B, feat, fb, fn, count, list, nsample, params, nullptr, 0, order, out, xcd);
  }
  return launch_status("dvcp_sa_group_mlp(mfma)");
}

#define DVCP_SA_MFMA_INST(T, D, C1, C2)                                                                          \
  template int launch_sa_mfma<T, D, C1, C2>(const void*, int64_t, int64_t, int64_t, int, const void*, int64_t,  \
                                            int64_t, int64_t, int, int, const float*, int64_t, int64_t,         \
                                            const int32_t*, const int32_t*, int, const float*, float*,          \
                                            int32_t*, float*, const int64_t*, int, hipStream_t);
DVCP_SA_MFMA_INST(float, 32, 32, 64)
DVCP_SA_MFMA_INST(double, 32, 32, 64)
DVCP_SA_MFMA_INST(float, 64, 64, 64)
DVCP_SA_MFMA_INST(double, 64, 64, 64)
#undef DVCP_SA_MFMA_INST

}  // namespace dvcp
