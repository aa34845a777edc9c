// dfe_mfma.hip -- the target-side deep feature embedding (get_cat_feat_tgt.py:54-96 fused with
// deep_feat_embedding.py:47-60) on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Per candidate the 32 neighbour rows go through three 32-wide linear layers (35->32->32->32, no
// nonlinearity, Q14) and a max over the rows: a 32 x 35 -> 32 -> 32 -> 32 GEMM chain per candidate,
// one wave per candidate.  The 32x32 accumulator layout (lane l, register r holds
// D[(r&3) + 8(r>>2) + 4(l>>5)][l&31]) lets each layer feed the next without an LDS round trip:
//   layer 1, transposed: H1^T = W1 . X^T    A = W1 fragment, B = X^T (lane: row j, k-half)
//                        -> channels in registers, rows on lanes
//   layer 2, transposed: H2^T = W2 . H1^T   A = W2 fragment, B = the layer-1 registers
//                        (register r is the k-step over channels (c, c+4), c = acc_row(r, 0))
//   layer 3:             H3 = H2 . W3^T     A = the layer-2 registers, B = W3^T fragment
//                        -> rows in registers, output channels on lanes
// so the max over rows is a per-lane max over registers plus one exchange between lane halves.
// Input channel order of layer 1's k-step s: lane half 0 takes [dx, dy, dz, f0 .. f15], half 1
// [0, 0, 0, f16 .. f31] (19 k-steps; see sa_mlp_mfma.hip).
// Everything before the GEMMs is the reference's arithmetic as in dfe_tgt_kernel (dfe.hip):
// dist_sum in fp64 summed in neighbour order, w = dist / dist_sum in fp64, feature x w in fp64
// rounded to fp32, coordinates differenced in the point dtype.  The MFMA is a k-ordered fp32 fma
// chain; only the summation order differs from the row-per-thread kernel.
#include "common.h"


namespace dvcp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef DVCP_DFE_SPLIT3
#define DVCP_DFE_SPLIT3 1
#endif
// DVCP_DFE_ABL (timing experiments only, wrong results): 1 no gather, 2 no MFMA, 3 no weights,
// 4 no coordinate gather, 5 no feature-row gather.
// Round 4 at C3 (0.68 ms): 0.51, 0.47, 0.67 ms -- neither the gathers nor the matrix cores alone
// bound the kernel.  (Contiguous candidate runs per wave measured 0.71: not kept.)
#ifndef DVCP_DFE_ABL
#define DVCP_DFE_ABL 0
#endif
// DVCP_DFE_WAHEAD: a candidate's w row is formed two steps before its MFMAs instead of one, so the
// operands of candidate c + 1 need no w row of the same step (round 5 at C3, A/B on one box:
// 0.659 / 0.651 -> 0.647 / 0.651 ms, profiles/round5/r5t_dfe_ab.log)
#ifndef DVCP_DFE_WAHEAD
#define DVCP_DFE_WAHEAD 1
#endif
// DVCP_DFE_W2 (with WAHEAD): the w rows of two candidates per pass, one per lane half (the fp64
// sum, division and DPP moves run once for two candidates instead of once per candidate on
// mirrored halves); formed at every other step
#ifndef DVCP_DFE_W2
#define DVCP_DFE_W2 1
#endif
// DVCP_DFE_SCAND: the candidate's coordinates as scalar loads (its index is wave-uniform; measured
// equal to vector loads, 0.694 / 0.696 ms, profiles/round5/r5r_dfe_ab.log)
#ifndef DVCP_DFE_SCAND
#define DVCP_DFE_SCAND 1
#endif
// DVCP_DFE_PIN: the operands prepared for candidate c + 1 are pinned (an empty asm that reads
// them) before step c's exit test.  Without it the compiler sinks their computation past the
// loop's exit branch into step c + 1, in front of the MFMAs that read them, and the VALU work the
// pipeline was built to overlap with step c's MFMA chain runs in series with its own chain.
// Measured (round 5): the pinned schedule is slower, 0.647 / 0.651 -> 0.680 / 0.675 ms; three
// waves per SIMD overlap one wave's chain with another's VALU better than one wave interleaves
// both, so the default leaves the compiler's placement.
#ifndef DVCP_DFE_PIN
#define DVCP_DFE_PIN 0
#endif
// DVCP_DFE_WPE: waves per SIMD the kernel is compiled for (3: 136 VGPRs, no spills; 4: 128 VGPRs
// and 48 B of spills)
#ifndef DVCP_DFE_WPE
#define DVCP_DFE_WPE 3
#endif
// (Round 5, measured without change: the E fragments held in 26 VGPRs instead of re-read per
// candidate, 0.655 / 0.653 -> 0.664 / 0.654 ms, profiles/round5/r5aa_dfe_ereg_ab.log; the
// gathered rows three candidates ahead instead of two, 0.597 / 0.587 -> 0.599 / 0.595 ms,
// r5an_dfe_ga.log.  A build
// without packed fp32 (target attribute) ran 11x slower with wrong results: not a usable switch.)

// x = x0 + x1 + x2 exactly in three bf16 pieces; a.b from the six significant piece products
// (the fp32-accurate split of sa_mlp_mfma.hip, whose header gives the error bound)
struct DfeSplit3 {
  bf16x8 p0, p1, p2;
};
__device__ __forceinline__ DfeSplit3 dfe_split3(const float (&x)[8]) {
  DfeSplit3 s;
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
__device__ __forceinline__ f32x16 dfe_mfma_split3(const DfeSplit3& a, const bf16x8& b0, const bf16x8& b1,
                                                 const bf16x8& b2, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p2, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b1, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b0, acc, 0, 0, 0);
}

constexpr int kDfeMfmaWaves = 4;
constexpr int kDfeKS = 19;  // layer-1 k-steps: 3 + 32/2

__device__ __forceinline__ int dfe_acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct DfeMfmaLds {
  float w1[kDfeKS][64];  // A fragment of layer 1: [k-step][lane]
  float w2[16][64];      // A fragment of layer 2: [k-step][lane]
  float w3[16][64];      // B fragment of layer 3: [k-step][lane]
  float b1[2][16];       // layer 1/2 bias by [lane half][register]
  float b2[2][16];
};

template <typename T>
__global__ __launch_bounds__(kDfeMfmaWaves * kWave) void dfe_tgt_mfma_kernel(
    PointsView<T> ref, const float* __restrict__ feat, int M, const float* __restrict__ cand,
    const float* __restrict__ dist, const int32_t* __restrict__ idx, int Q, int B, const float* __restrict__ params,
    float* __restrict__ out) {
  __shared__ DfeMfmaLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  // params: W1 (32 x 35), b1, W2 (32 x 32), b2, W3 (32 x 32), b3
  const float* W1 = params;
  const float* pb1 = W1 + 32 * 35;
  const float* W2 = pb1 + 32;
  const float* pb2 = W2 + 32 * 32;
  const float* W3 = pb2 + 32;
  const float* pb3 = W3 + 32 * 32;
  for (int i = tid; i < kDfeKS * 64; i += blockDim.x) {
    const int l = i % 64, s = i / 64, hh = l >> 5;
    const int ch = s < 3 ? (hh == 0 ? s : -1) : 3 + hh * 16 + (s - 3);
    L.w1[s][l] = ch < 0 ? 0.0f : W1[(l & 31) * 35 + ch];
  }
  for (int i = tid; i < 16 * 64; i += blockDim.x) {
    const int l = i % 64, r = i / 64;
    const int in = dfe_acc_row(r, l >> 5);
    L.w2[r][l] = W2[(l & 31) * 32 + in];
    L.w3[r][l] = W3[(l & 31) * 32 + in];
  }
  for (int i = tid; i < 32; i += blockDim.x) {
    const int r = i % 16, hh = i / 16;
    L.b1[hh][r] = pb1[dfe_acc_row(r, hh)];
    L.b2[hh][r] = pb2[dfe_acc_row(r, hh)];
  }
  const float b3 = pb3[r32];
  __syncthreads();

  const int64_t total = static_cast<int64_t>(B) * Q;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * kDfeMfmaWaves + wave; g < total;
       g += static_cast<int64_t>(gridDim.x) * kDfeMfmaWaves) {
    const int b = static_cast<int>(g / Q);
    // get_cat_feat_tgt.py:57-58: dist_sum in fp64 (neighbour order), w = dist / dist_sum
    const float dj = dist[g * 32 + r32];
    double dsum = 0.0;
#pragma unroll
    for (int t = 0; t < 32; ++t)
      dsum += static_cast<double>(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(dj), t)));
    const double wj = static_cast<double>(dj) / dsum;
    int n = idx[g * 32 + r32];
    n = n < 0 ? 0 : (n >= M ? M - 1 : n);
    const float* cq = cand + g * 3;
    float x[kDfeKS];
    if (h == 0) {
      // candidates_grouped_local = tgt_pts_picked - candidate (point dtype, then .float())
      x[0] = static_cast<float>(ref.at(b, 0, n) - static_cast<T>(cq[0]));
      x[1] = static_cast<float>(ref.at(b, 1, n) - static_cast<T>(cq[1]));
      x[2] = static_cast<float>(ref.at(b, 2, n) - static_cast<T>(cq[2]));
    } else {
      x[0] = x[1] = x[2] = 0.0f;
    }
    // tgt_feat_norm[j, f] = F[idx_j, f] * w[f]   (Q10: the weight is indexed by the channel)
    const float4* fr = reinterpret_cast<const float4*>(feat + (static_cast<int64_t>(b) * M + n) * 32 + 16 * h);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float4 f = fr[v];
      const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * v + e;
        // w of channel i (half 0) or 16 + i (half 1): lanes i and 16 + i hold them
        const int2 lo = make_int2(__builtin_amdgcn_readlane(__double2loint(wj), i),
                                  __builtin_amdgcn_readlane(__double2hiint(wj), i));
        const int2 hi = make_int2(__builtin_amdgcn_readlane(__double2loint(wj), 16 + i),
                                  __builtin_amdgcn_readlane(__double2hiint(wj), 16 + i));
        const double wf = h ? __hiloint2double(hi.y, hi.x) : __hiloint2double(lo.y, lo.x);
        x[3 + i] = static_cast<float>(static_cast<double>(fv[e]) * wf);
      }
    }
    int zo = 0;  // opaque zero: weight fragments are re-read from LDS per candidate, not hoisted
    asm volatile("" : "+v"(zo));
    f32x16 a1, a2, a3;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      a1[r] = L.b1[h][r + zo];
      a2[r] = L.b2[h][r + zo];
      a3[r] = b3;
    }
#pragma unroll
    for (int s = 0; s < kDfeKS; ++s) a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(L.w1[s][lane + zo], x[s], a1, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(L.w2[r][lane + zo], a1[r], a2, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[r], L.w3[r][lane + zo], a3, 0, 0, 0);
    // MaxPool1d(32) over the rows: registers, then the other lane half
    float m = a3[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) m = fmaxf(m, a3[r]);
    m = fmaxf(m, __shfl_xor(m, 32, kWave));
    if (h == 0) out[g * 32 + r32] = m;
  }
}

// ---------------------------------------------------------------------------------------------
// Collapsed form (default).  fc1, fc2 and fc3 have no nonlinearity between them (Q14,
// deep_feat_embedding.py:48-50), so fc3(fc2(fc1 x)) = E x + e with E = W3 W2 W1 (32 x 35) and
// e = W3 (W2 b1 + b2) + b3.  Each workgroup forms E and e in fp64 from the three layers (a
// 72 kflop prologue) and rounds them once to fp32; a candidate then costs 19 MFMAs instead of 51.
// The result differs from the layer-by-layer fp32 chain only by rounding (two fewer fp32
// roundings of intermediates, one of E); tests hold it to the same 1e-5 bound.
//   H = X . E^T:  A = X (lane: row j, k-half), B = E^T fragment (lane: output channel, k-half)
//   -> output channel on lanes, rows in registers, max over rows = registers + one lane swap.
// DVCP_DFE_SPLIT3 (default): the xyz columns take two fp32 MFMA k-steps ((x|y), (z|0)) and the 32
// feature columns two 16-deep bf16 k-steps of the fp32-accurate three-way split (lane half h's
// features 16h + 8t .. + 7 in k-step t): 2 x 64 + 12 x 32 = 512 MFMA cycles per candidate instead
// of 19 x 64 = 1216.
// dist_sum: 32 fp32 distances summed in fp64 are exact whenever they span less than 2^24 (24-bit
// mantissas, 5 bits of carry, 53-bit accumulator), so a butterfly sum equals the reference's
// ordered sum; w_j = dist_j / dist_sum in fp64 is then bit-identical.
constexpr int kDfe1Waves = 4;
#ifndef DVCP_DFE_GRID
#define DVCP_DFE_GRID 512
#endif
// workgroups (a multiple of 8), every wave resident from the start (one fp64 prologue per
// workgroup, no tail of late workgroups).  Round 5: 2048 / 1536 / 1024 / 768 measured 0.703 /
// 0.674 / 0.670 / 0.666 ms and 0.682 / 0.687 / 0.665 / 0.663 (profiles/round5/r5s_dfe_grid_ab.log).
// Round 6, after the packed-row gather and the paired w rows cut the per-candidate instructions:
// 1024 / 768 / 512 / 256 workgroups 0.565 / 0.545 / 0.535 / 0.639 ms (tools/knn_bench.py --fast,
// two runs each, profiles/round6/r6aj_dfe_*.log): two workgroups per CU (two waves per SIMD) now
// keep the gathers and the matrix cores as busy as three, and leave the CU room to other kernels'
// waves
constexpr int kDfeGrid = DVCP_DFE_GRID;

// v + (v moved by the DPP pattern CTRL), fp64 (the two halves moved separately).  Every pattern
// used (quad permutes, row rotations) reads a lane of the same row for every lane, so the moves
// need no old value (mov_dpp: no zeroed destination register per move)
template <int CTRL>
__device__ __forceinline__ double dpp_add_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return v + __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}

struct Dfe1Lds {
  double p[32][35];      // W2 . W1 (fp64), prologue only
  double pb[32];         // W2 . b1 + b2
#if DVCP_DFE_SPLIT3
  float ex[2][64];          // E's xyz columns as fp32 B fragments: k-steps (x|y), (z|0)
  bf16x8 es[2][3][64];      // E's feature columns as bf16 pieces: [k-step][piece][lane]
#else
  float e[kDfeKS][64];   // E as the B fragment: [k-step][lane]
#endif
  float eb[32];          // e
  float w[kDfe1Waves][4][32];  // per-wave w rows of consecutive candidates (fp64 quotient rounded to fp32)
};

// FT: the feature table's element type -- float, or _Float16 (the C5 "fp16 features" storage:
// half the gathered bytes; each row is widened to fp32 before the weighting, which then runs in
// fp32 exactly as for a float table holding the same values).
// Target points in (x, y, z, pad) float4 rows (PointsView::rows4, dvcp_points_pack4) are gathered
// as one 16-byte load per neighbour instead of three 4-byte loads from three lines of the
// (B, 3, M) layout.  Round 5 ablation at C3: the three scattered coordinate loads alone cost
// 0.664 -> 0.513 ms, the 128-byte feature rows 0.664 -> 0.62 (profiles/round5/r5ac_dfe_abl.log);
// with packed rows the call (pack included) runs 0.54 ms (r5ad_p4.log).
// P4: the target points are (x, y, z, pad) rows (PointsView::rows4, known at launch): one
// 16-byte gather per neighbour with no per-candidate layout branch.
template <typename T, typename FT = float, bool P4 = false>
__global__ __launch_bounds__(kDfe1Waves * kWave) __attribute__((amdgpu_waves_per_eu(DVCP_DFE_WPE))) void dfe_tgt_mfma1_kernel(
    PointsView<T> ref, const FT* __restrict__ feat, int M, const float* __restrict__ cand,
    const float* __restrict__ dist, const int32_t* __restrict__ idx, int Q, int B, const float* __restrict__ params,
    float* __restrict__ out, int xcd) {
  __shared__ Dfe1Lds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const float* W1 = params;
  const float* pb1 = W1 + 32 * 35;
  const float* W2 = pb1 + 32;
  const float* pb2 = W2 + 32 * 32;
  const float* W3 = pb2 + 32;
  const float* pb3 = W3 + 32 * 32;
  // prologue: P = W2 W1, pb = W2 b1 + b2 (fp64)
  for (int i = tid; i < 32 * 36; i += blockDim.x) {
    const int o = i / 36, c = i % 36;
    double acc = 0.0;
    if (c < 35) {
      for (int a = 0; a < 32; ++a) acc = __fma_rn(static_cast<double>(W2[o * 32 + a]), static_cast<double>(W1[a * 35 + c]), acc);
      L.p[o][c] = acc;
    } else {
      for (int a = 0; a < 32; ++a) acc = __fma_rn(static_cast<double>(W2[o * 32 + a]), static_cast<double>(pb1[a]), acc);
      L.pb[o] = acc + static_cast<double>(pb2[o]);
    }
  }
  __syncthreads();
  // E = W3 P in fragment order, e = W3 pb + b3
  auto e_entry = [&](int o, int ch) {
    double acc = 0.0;
    for (int a = 0; a < 32; ++a) acc = __fma_rn(static_cast<double>(W3[o * 32 + a]), L.p[a][ch], acc);
    return static_cast<float>(acc);
  };
#if DVCP_DFE_SPLIT3
  for (int i = tid; i < 2 * 64; i += blockDim.x) {
    const int l = i % 64, s = i / 64, hh = l >> 5, o = l & 31;
    const int ch = s == 0 ? hh : (hh == 0 ? 2 : -1);
    L.ex[s][l] = ch < 0 ? 0.0f : e_entry(o, ch);
  }
  for (int i = tid; i < 2 * 64; i += blockDim.x) {
    const int l = i % 64, t = i / 64, hh = l >> 5, o = l & 31;
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = e_entry(o, 3 + 16 * hh + 8 * t + j);
    const DfeSplit3 ws = dfe_split3(w);
    L.es[t][0][l] = ws.p0;
    L.es[t][1][l] = ws.p1;
    L.es[t][2][l] = ws.p2;
  }
#else
  for (int i = tid; i < kDfeKS * 64; i += blockDim.x) {
    const int l = i % 64, s = i / 64, hh = l >> 5, o = l & 31;
    const int ch = s < 3 ? (hh == 0 ? s : -1) : 3 + hh * 16 + (s - 3);
    L.e[s][l] = ch < 0 ? 0.0f : e_entry(o, ch);
  }
#endif
  for (int o = tid; o < 32; o += blockDim.x) {
    double acc = 0.0;
    for (int a = 0; a < 32; ++a) acc = __fma_rn(static_cast<double>(W3[o * 32 + a]), L.pb[a], acc);
    L.eb[o] = static_cast<float>(acc + static_cast<double>(pb3[o]));
  }
  __syncthreads();
  const float eb = L.eb[r32];

  // Software pipeline over this wave's candidates g0, g0 + stride, ...: the kNN row (dist, idx)
  // is loaded two candidates ahead and the gathered point/feature row one ahead, so the
  // dependent idx -> gather latency overlaps the MFMAs of the candidate in hand.  Two register
  // sets (A, B) alternate, so no loaded register is ever copied (a copy would wait for its load).
  // Loads are unconditional (indices clamped to the last candidate) and a loaded index is only
  // clamped in the iteration that gathers with it.  Candidate indices are wave-uniform int32
  // (B * Q < 2^31 is checked by the launcher).
  // Candidate order.  xcd == 0: one index space over all B*Q candidates.  xcd != 0 (B >= 8, grid a
  // multiple of 8): workgroups are dispatched to the 8 XCDs round robin (blockIdx % 8), so the
  // workgroups of XCD x take the candidates of pairs x, x+8, ...; each pair's gathered feature
  // table then lives in one XCD's L2 instead of being fetched into all eight.
  int total, stride, g, xo = 0, P = 1;
  if (xcd) {
    xo = static_cast<int>(blockIdx.x) & 7;
    P = 8;
    total = ((B - xo + 7) / 8) * Q;
    stride = static_cast<int>(gridDim.x >> 3) * kDfe1Waves;
    g = static_cast<int>(blockIdx.x >> 3) * kDfe1Waves + __builtin_amdgcn_readfirstlane(wave);
  } else {
    total = B * Q;
    stride = static_cast<int>(gridDim.x) * kDfe1Waves;
    g = static_cast<int>(blockIdx.x) * kDfe1Waves + __builtin_amdgcn_readfirstlane(wave);
  }
  if (g >= total) return;
  // Local candidate index li = pl * Q + q -> pair b = xo + P * pl and global candidate b * Q + q,
  // tracked incrementally per pipeline slot (wave-uniform, no integer division per candidate);
  // indices past the end clamp to the last candidate (loads stay in bounds, results unused).
  // A tracker holds its pair bb and global candidate gc = bb Q + q as well, advanced by constant
  // steps, so a use is one select against the last candidate instead of a multiply-add chain.
  struct Cand {
    int li, q, bb, gc;
  };
  auto cand_at = [&](int li) {
    Cand c;
    c.li = li;
    const int pl = li / Q;  // once per slot at the start
    c.q = li - pl * Q;
    c.bb = xo + P * pl;
    c.gc = c.bb * Q + c.q;
    return c;
  };
  const int st_pl = stride / Q, st_q = stride - st_pl * Q;
  const int st_bb = P * st_pl, st_gc = P * st_pl * Q + st_q, wrap_gc = (P - 1) * Q;
  auto advance = [&](Cand& c) {  // branch-free (scalar selects): li += stride
    c.li += stride;
    c.q += st_q;
    c.bb += st_bb;
    c.gc += st_gc;
    const bool wrap = c.q >= Q;
    c.q = wrap ? c.q - Q : c.q;
    c.bb = wrap ? c.bb + P : c.bb;
    c.gc = wrap ? c.gc + wrap_gc : c.gc;
  };
  const Cand last = cand_at(total - 1);
  auto pair_of = [&](const Cand& c) { return c.li < total ? c.bb : last.bb; };
  auto glob_of = [&](const Cand& c) { return c.li < total ? c.gc : last.gc; };
  auto load_row = [&](const Cand& c, float& dj, int& n) {
    const int gc = glob_of(c);
    dj = dist[static_cast<int64_t>(gc) * 32 + r32];
    n = idx[static_cast<int64_t>(gc) * 32 + r32];
  };
  struct Gathered {
    float4 f[4];
    uint4 hf[2];  // fp16 table: the row's 16 halves of this lane half, widened in prep
    T px, py, pz;
    float cx, cy, cz;
  };
  auto gather = [&](const Cand& c, int nraw, Gathered& G) {
    const int bb = pair_of(c);
    const int gc = glob_of(c);
#if DVCP_DFE_ABL == 1  // (ablation builds only: every gather reads the lane's fixed row)
    const int n = r32 + 0 * nraw;
#else
    const int n = nraw < 0 ? 0 : (nraw >= M ? M - 1 : nraw);
#endif
    if constexpr (sizeof(FT) == 4) {
#if DVCP_DFE_ABL == 5  // (ablation builds only: the feature rows of the lane's fixed point)
      const float4* fr = reinterpret_cast<const float4*>(feat + (static_cast<int64_t>(bb) * M + r32) * 32 + 16 * h);
#else
      const float4* fr = reinterpret_cast<const float4*>(feat + (static_cast<int64_t>(bb) * M + n) * 32 + 16 * h);
#endif
#pragma unroll
      for (int v = 0; v < 4; ++v) G.f[v] = fr[v];
    } else {
      const uint4* fr = reinterpret_cast<const uint4*>(feat + (static_cast<int64_t>(bb) * M + n) * 32 + 16 * h);
      G.hf[0] = fr[0];
      G.hf[1] = fr[1];
    }
#if DVCP_DFE_ABL == 4  // (ablation builds only: the coordinates of the lane's fixed point)
    G.px = ref.at(bb, 0, r32);
    G.py = ref.at(bb, 1, r32);
    G.pz = ref.at(bb, 2, r32);
#else
    if constexpr (P4) {
      const float4 q = *reinterpret_cast<const float4*>(ref.p + bb * ref.sb + 4 * static_cast<int64_t>(n));
      G.px = q.x;
      G.py = q.y;
      G.pz = q.z;
    } else {
      G.px = ref.at(bb, 0, n);
      G.py = ref.at(bb, 1, n);
      G.pz = ref.at(bb, 2, n);
    }
#endif
#if DVCP_DFE_SCAND
    const float* cq = cand + static_cast<int64_t>(__builtin_amdgcn_readfirstlane(gc)) * 3;
    G.cx = cq[0];
    G.cy = cq[1];
    G.cz = cq[2];
#else
    G.cx = cand[static_cast<int64_t>(gc) * 3];
    G.cy = cand[static_cast<int64_t>(gc) * 3 + 1];
    G.cz = cand[static_cast<int64_t>(gc) * 3 + 2];
#endif
  };
  // get_cat_feat_tgt.py:57-58 (lanes 32..63 mirror lanes 0..31): the w row of a candidate, into
  // the wave's LDS row `buf` (two rows: a candidate's row is written while the previous one may
  // still be read).  w = dist / dist_sum is formed in fp64 like the reference and rounded once to
  // fp32; the feature product is then one fp32 multiply (the reference rounds the fp64 product to
  // fp32 at the DFE input: the two differ by at most one fp32 ulp of the input).
  auto weights = [&](float dj, int buf) {
    // sum of the 32 distances: quad and row rotations by DPP (no LDS round trips), then the two
    // 16-lane row totals of the lower half read back and added (the upper half mirrors it)
#if DVCP_DFE_ABL == 3  // (ablation builds only: no distance sum / division)
    L.w[wave][buf][r32] = dj;
    return;
#endif
    double v = static_cast<double>(dj);
    v = dpp_add_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v = dpp_add_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v = dpp_add_f64<0x124>(v);  // row_ror:4
    v = dpp_add_f64<0x128>(v);  // row_ror:8
    const double dsum = readlane_f64(v, 15) + readlane_f64(v, 31);
    L.w[wave][buf][r32] = static_cast<float>(static_cast<double>(dj) / dsum);  // both halves write the same value
  };
  // the same for two candidates at once: lane half 0 forms candidate A's row (dja) into slot bufa,
  // half 1 candidate B's (djb) into bufb (the DPP patterns stay inside 16-lane rows, so the halves'
  // sums do not mix: rows 0-1 are A's 32 distances, rows 2-3 B's)
  auto weights2 = [&](float dja, float djb, int bufa, int bufb) {
#if DVCP_DFE_ABL == 3  // (ablation builds only: no distance sum / division)
    L.w[wave][h ? bufb : bufa][r32] = h ? djb : dja;
    return;
#endif
    const float dj = h ? djb : dja;
    double v = static_cast<double>(dj);
    v = dpp_add_f64<0xB1>(v);
    v = dpp_add_f64<0x4E>(v);
    v = dpp_add_f64<0x124>(v);
    v = dpp_add_f64<0x128>(v);
    const double sa = readlane_f64(v, 15) + readlane_f64(v, 31);
    const double sb = readlane_f64(v, 47) + readlane_f64(v, 63);
    L.w[wave][h ? bufb : bufa][r32] = static_cast<float>(static_cast<double>(dj) / (h ? sb : sa));
  };
  // A operands of a candidate: the xyz k-steps ((dx|dy), (dz|0)) and the 32 weighted features as
  // split-3 bf16 pieces (lane half h: features 16h .. 16h + 15, k-step t: 16h + 8t ..)
  struct Prepared {
    float x0, x1;
    DfeSplit3 s[2];
  };
  auto prep = [&](const Gathered& G, int buf, Prepared& X) {
    // candidates_grouped_local = tgt_pts_picked - candidate (point dtype, then .float()); half 1: 0
    const float ddx = static_cast<float>(G.px - static_cast<T>(G.cx));
    const float ddy = static_cast<float>(G.py - static_cast<T>(G.cy));
    const float ddz = static_cast<float>(G.pz - static_cast<T>(G.cz));
    X.x0 = h == 0 ? ddx : ddy;
    X.x1 = h == 0 ? ddz : 0.0f;
    const float4* wr = reinterpret_cast<const float4*>(&L.w[wave][buf][16 * h]);
    float4 fv[4];
    if constexpr (sizeof(FT) == 4) {
#pragma unroll
      for (int v = 0; v < 4; ++v) fv[v] = G.f[v];
    } else {
      const uint32_t* hw = reinterpret_cast<const uint32_t*>(G.hf);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const uint32_t lo = hw[2 * v], hi = hw[2 * v + 1];
        fv[v].x = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(lo & 0xFFFFu)));
        fv[v].y = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(lo >> 16)));
        fv[v].z = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(hi & 0xFFFFu)));
        fv[v].w = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(hi >> 16)));
      }
    }
    float x[16];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float4 w4 = wr[v];
      x[4 * v] = fv[v].x * w4.x;
      x[4 * v + 1] = fv[v].y * w4.y;
      x[4 * v + 2] = fv[v].z * w4.z;
      x[4 * v + 3] = fv[v].w * w4.w;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float f8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) f8[j] = x[8 * t + j];
      X.s[t] = dfe_split3(f8);
    }
  };
#if DVCP_DFE_PIN
  auto pin = [&](const Prepared& X) {
    asm volatile("" ::"v"(X.x0), "v"(X.x1), "v"(X.s[0].p0), "v"(X.s[0].p1), "v"(X.s[0].p2), "v"(X.s[1].p0),
                 "v"(X.s[1].p1), "v"(X.s[1].p2));
  };
#else
  auto pin = [&](const Prepared&) {};
#endif
  // H = X E^T on the matrix cores; zero-started accumulators, e added once to the row maximum:
  // max_j fl(h_j + e) = fl(max_j h_j + e) (rounding is monotone)
  auto mfma = [&](const Prepared& X) {
    int zo = 0;  // opaque zero: E fragments are re-read from LDS per candidate, not hoisted
    asm volatile("" : "+v"(zo));
    f32x16 a;
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.0f;
#if DVCP_DFE_ABL == 2  // (ablation builds only: no MFMA, the operands still consumed)
    a[0] = X.x0 + X.x1 + static_cast<float>(X.s[0].p0[0]) + static_cast<float>(X.s[1].p2[7]) + L.ex[0][lane + zo];
#else
    a = __builtin_amdgcn_mfma_f32_32x32x2f32(X.x0, L.ex[0][lane + zo], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_32x32x2f32(X.x1, L.ex[1][lane + zo], a, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 2; ++t)
      a = dfe_mfma_split3(X.s[t], L.es[t][0][lane + zo], L.es[t][1][lane + zo], L.es[t][2][lane + zo], a);
#endif
    return a;
  };
  auto finish = [&](const Cand& cg, const f32x16& a) {
    float m = a[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) m = fmaxf(m, a[r]);
    // the other lane half's rows: v_permlane32_swap (lanes 0..31 receive lanes 32..63; only they
    // store) instead of an LDS-crossbar shuffle
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    m = fmaxf(m, __uint_as_float(sw[1]));
    m += eb;
    if (h == 0) out[static_cast<int64_t>(glob_of(cg)) * 32 + r32] = m;
  };
  // Software pipeline, one candidate per step: step c issues candidate c's MFMA chain and, in the
  // same basic block, the independent VALU work of candidate c + 1 (its w row, its operands), which
  // the scheduler places between the MFMAs; kNN rows are loaded six candidates ahead (they come
  // from HBM / the infinity cache), gathered rows two ahead of their use.  Slots: rows U & 7,
  // gathered rows and operands U & 1 (unrolled by 8, so every slot index is a constant).
  constexpr int WA = DVCP_DFE_WAHEAD;
  float dj[8];
  int nn[8];
  Gathered G[2];
  Prepared X[2];
  Cand t0 = cand_at(g), t2 = cand_at(g + 2 * stride), t6 = cand_at(g + 6 * stride);
  {
    Cand r = t0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      load_row(r, dj[i], nn[i]);
      advance(r);
    }
    Cand c1 = t0;
    advance(c1);
    gather(t0, nn[0], G[0]);
    gather(c1, nn[1], G[1]);
    if (WA && DVCP_DFE_W2) {
      weights2(dj[0], dj[1], 0, 1);
    } else {
      weights(dj[0], 0);
      if (WA) weights(dj[1], 1);
    }
    prep(G[0], 0, X[0]);
  }
#define DVCP_DFE_STEP(U)                                              \
  {                                                                   \
    const f32x16 acc = mfma(X[(U)&1]);                                \
    if (!WA) weights(dj[((U) + 1) & 7], ((U) + 1) & 3);               \
    prep(G[((U) + 1) & 1], ((U) + 1) & 3, X[((U) + 1) & 1]);          \
    if (WA && DVCP_DFE_W2 && ((U)&1) == 0)                            \
      weights2(dj[((U) + 2) & 7], dj[((U) + 3) & 7], ((U) + 2) & 3,   \
               ((U) + 3) & 3);                                        \
    if (WA && !DVCP_DFE_W2) weights(dj[((U) + 2) & 7], ((U) + 2) & 3); \
    load_row(t6, dj[((U) + 6) & 7], nn[((U) + 6) & 7]);               \
    gather(t2, nn[((U) + 2) & 7], G[(U)&1]);                          \
    pin(X[((U) + 1) & 1]);                                            \
    finish(t0, acc);                                                  \
    advance(t0);                                                      \
    advance(t2);                                                      \
    advance(t6);                                                      \
    if (t0.li >= total) break;                                        \
  }
  for (;;) {
    DVCP_DFE_STEP(0)
    DVCP_DFE_STEP(1)
    DVCP_DFE_STEP(2)
    DVCP_DFE_STEP(3)
    DVCP_DFE_STEP(4)
    DVCP_DFE_STEP(5)
    DVCP_DFE_STEP(6)
    DVCP_DFE_STEP(7)
  }
#undef DVCP_DFE_STEP
}

// (x, y, z, 0) float4 rows of B clouds of M points (the layout dfe_tgt_mfma1_kernel's P4 reads)
__global__ void points_pack4_kernel(PointsView<float> pts, int M, int B, float4* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<int64_t>(B) * M) return;
  const int b = static_cast<int>(i / M);
  const int64_t n = i - static_cast<int64_t>(b) * M;
  out[i] = make_float4(pts.at(b, 0, n), pts.at(b, 1, n), pts.at(b, 2, n), 0.0f);
}

template <typename T>
int launch_dfe_tgt_mfma(PointsView<T> ref, const float* feat, int M, const float* cand, const float* dist,
                        const int32_t* idx, int B, int Q, const float* params, float* out, bool literal,
                        hipStream_t st) {
  const int64_t total = static_cast<int64_t>(B) * Q;
  if (total >= (int64_t(1) << 31) / 32) {
    set_error("dvcp_dfe_tgt: B*Q=%lld too large", static_cast<long long>(total));
    return DVCP_EINVAL;
  }
  const int64_t need = (total + kDfeMfmaWaves - 1) / kDfeMfmaWaves;
  if (literal) {
    const int grid = static_cast<int>(need < 4096 ? need : 4096);
    hipLaunchKernelGGL((dfe_tgt_mfma_kernel<T>), dim3(grid), dim3(kDfeMfmaWaves * kWave), 0, st, ref, feat, M, cand,
                       dist, idx, Q, B, params, out);
  } else {
    // a few resident workgroups per CU amortise the fp64 prologue over many candidates
    const int xcd = B % 8 == 0 && need >= kDfeGrid ? 1 : 0;  // equal pairs per XCD
    const int grid = static_cast<int>(need < kDfeGrid ? need : kDfeGrid);
    if (sizeof(T) == 4 && ref.rows4())
      hipLaunchKernelGGL((dfe_tgt_mfma1_kernel<T, float, sizeof(T) == 4>), dim3(grid), dim3(kDfe1Waves * kWave), 0, st,
                         ref, feat, M, cand, dist, idx, Q, B, params, out, xcd);
    else
      hipLaunchKernelGGL((dfe_tgt_mfma1_kernel<T>), dim3(grid), dim3(kDfe1Waves * kWave), 0, st, ref, feat, M, cand,
                         dist, idx, Q, B, params, out, xcd);
  }
  return launch_status("dvcp_dfe_tgt(mfma)");
}

// The fp16-feature table (C5): the non-literal kernel only.
template <typename T>
int launch_dfe_tgt_mfma_f16(PointsView<T> ref, const _Float16* feat, int M, const float* cand, const float* dist,
                            const int32_t* idx, int B, int Q, const float* params, float* out, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(B) * Q;
  if (total >= (int64_t(1) << 31) / 32) {
    set_error("dvcp_dfe_tgt_f16: B*Q=%lld too large", static_cast<long long>(total));
    return DVCP_EINVAL;
  }
  const int64_t need = (total + kDfeMfmaWaves - 1) / kDfeMfmaWaves;
  const int xcd = B % 8 == 0 && need >= kDfeGrid ? 1 : 0;
  const int grid = static_cast<int>(need < kDfeGrid ? need : kDfeGrid);
  if (sizeof(T) == 4 && ref.rows4())
    hipLaunchKernelGGL((dfe_tgt_mfma1_kernel<T, _Float16, sizeof(T) == 4>), dim3(grid), dim3(kDfe1Waves * kWave), 0,
                       st, ref, feat, M, cand, dist, idx, Q, B, params, out, xcd);
  else
    hipLaunchKernelGGL((dfe_tgt_mfma1_kernel<T, _Float16>), dim3(grid), dim3(kDfe1Waves * kWave), 0, st, ref, feat, M,
                       cand, dist, idx, Q, B, params, out, xcd);
  return launch_status("dvcp_dfe_tgt_f16");
}

template int launch_dfe_tgt_mfma<float>(PointsView<float>, const float*, int, const float*, const float*,
                                        const int32_t*, int, int, const float*, float*, bool, hipStream_t);
template int launch_dfe_tgt_mfma<double>(PointsView<double>, const float*, int, const float*, const float*,
                                         const int32_t*, int, int, const float*, float*, bool, hipStream_t);

}  // namespace dvcp

extern "C" int dvcp_dfe_tgt_f16(int dtype, const void* ref_xyz, int64_t rb, int64_t rc, int64_t rn, int M,
                                const uint16_t* ref_feat, const float* cand, const float* dist, const int32_t* idx,
                                int B, int Q, const float* params, float* out, void* stream) {
  DVCP_REQUIRE(ref_xyz && ref_feat && cand && dist && idx && params && out, "dvcp_dfe_tgt_f16: null pointer");
  DVCP_REQUIRE(M > 0 && B >= 0 && B <= 65535 && Q >= 0, "dvcp_dfe_tgt_f16: bad sizes");
  if (B == 0 || Q == 0) return DVCP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const _Float16* f = reinterpret_cast<const _Float16*>(ref_feat);
  if (dtype == DVCP_F32)
    return dvcp::launch_dfe_tgt_mfma_f16<float>(dvcp::PointsView<float>{static_cast<const float*>(ref_xyz), rb, rc, rn},
                                                f, M, cand, dist, idx, B, Q, params, out, st);
  if (dtype == DVCP_F64)
    return dvcp::launch_dfe_tgt_mfma_f16<double>(
        dvcp::PointsView<double>{static_cast<const double*>(ref_xyz), rb, rc, rn}, f, M, cand, dist, idx, B, Q, params,
        out, st);
  dvcp::set_error("dvcp_dfe_tgt_f16: bad dtype %d", dtype);
  return DVCP_EINVAL;
}

extern "C" int dvcp_points_pack4(const float* xyz, int64_t sb, int64_t sc, int64_t sn, int M, int B, float* out,
                                 void* stream) {
  DVCP_REQUIRE(xyz && out, "dvcp_points_pack4: null pointer");
  DVCP_REQUIRE(M >= 0 && B >= 0, "dvcp_points_pack4: bad sizes");
  const int64_t total = static_cast<int64_t>(B) * M;
  if (total == 0) return DVCP_OK;
  DVCP_REQUIRE((reinterpret_cast<uintptr_t>(out) & 15) == 0, "dvcp_points_pack4: out must be 16-byte aligned");
  hipLaunchKernelGGL(dvcp::points_pack4_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), dvcp::PointsView<float>{xyz, sb, sc, sn}, M, B,
                     reinterpret_cast<float4*>(out));
  return dvcp::launch_status("dvcp_points_pack4");
}
