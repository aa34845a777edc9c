// morton.h -- helpers shared by the spatially tiled kernels (knn_tiled.hip, ball_query.hip):
// block-wide bounding box, 12-bit space-filling-curve (Hilbert) counting sort, and wave-uniform (scalar) loads.
#pragma once
#include "common.h"

namespace dvcp {

constexpr int kSortBins = 4096;  // 12-bit curve cells (16^3)
constexpr int kBuildThreads = 1024;

__device__ __forceinline__ float float_unorder(uint32_t u) {  // inverse of float_order
  const uint32_t flip = (u >> 31) ? 0x80000000u : 0xFFFFFFFFu;
  return __uint_as_float(u ^ flip);
}

// Wave-uniform reads through the constant address space: the compiler emits scalar loads
// (s_load_dwordx*), so tile data arrives in SGPRs and feeds the VALU as scalar operands.
typedef __attribute__((address_space(4))) const float const_float;

// A pointer known to be wave-uniform (the compiler can lose that through divergent phis).
template <typename P>
__device__ __forceinline__ P* uniform_ptr(P* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v & 0xFFFFFFFFull)));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32)));
  return reinterpret_cast<P*>((static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ uint32_t spread4b(uint32_t v) {
  v &= 0xF;
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4) | ((v & 8u) << 6);
}

// Hilbert index of a 16^3 cell (Skilling's transpose form, 4 bits per axis).  Unlike Morton
// order it has no jumps -- consecutive indices are face-adjacent cells -- so any run of
// consecutive items has a compact box (the tiled kernels' pruning depends on that).
__device__ __forceinline__ uint32_t hilbert3x4(uint32_t x, uint32_t y, uint32_t z) {
  uint32_t X[3] = {x, y, z};
#pragma unroll
  for (uint32_t Q = 8; Q > 1; Q >>= 1) {
    const uint32_t P = Q - 1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (X[i] & Q) {
        X[0] ^= P;
      } else {
        const uint32_t t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  uint32_t t = 0;
#pragma unroll
  for (uint32_t Q = 8; Q > 1; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1;
  X[0] ^= t;
  X[1] ^= t;
  X[2] ^= t;
  // bit b of X[i] lands at 3b + (2 - i)
  return spread4b(X[2]) | (spread4b(X[1]) << 1) | (spread4b(X[0]) << 2);
}

// Block-wide bounding box of n points (1024 threads).
template <typename GET>
__device__ void block_bbox(int n, GET get, float (&lo)[3], float (&hi)[3], float (*red)[3][16]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    lo[a] = __builtin_huge_valf();
    hi[a] = -__builtin_huge_valf();
  }
  for (int i = tid; i < n; i += kBuildThreads) {
    float v[3];
    get(i, v);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      lo[a] = fminf(lo[a], v[a]);
      hi[a] = fmaxf(hi[a], v[a]);
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    for (int off = 32; off > 0; off >>= 1) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off, kWave));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off, kWave));
    }
    if (lane == 0) {
      red[0][a][wave] = lo[a];
      red[1][a][wave] = hi[a];
    }
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float l = red[0][a][0], h = red[1][a][0];
    for (int w = 1; w < kBuildThreads / kWave; ++w) {
      l = fminf(l, red[0][a][w]);
      h = fmaxf(h, red[1][a][w]);
    }
    lo[a] = l;
    hi[a] = h;
  }
  __syncthreads();
}

// The 16^3 curve grid over a bounding box, and an item's 12-bit Hilbert cell in it.
struct CurveGrid {
  float lo[3], scale[3];
};
__device__ __forceinline__ CurveGrid curve_grid(const float (&lo)[3], const float (&hi)[3]) {
  CurveGrid g;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    g.lo[a] = lo[a];
    g.scale[a] = hi[a] > lo[a] ? 16.0f / (hi[a] - lo[a]) : 0.0f;
  }
  return g;
}
__device__ __forceinline__ uint32_t curve_cell(const CurveGrid& g, const float (&v)[3]) {
  uint32_t q[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    int c = static_cast<int>((v[a] - g.lo[a]) * g.scale[a]);
    q[a] = static_cast<uint32_t>(c < 0 ? 0 : (c > 15 ? 15 : c));
  }
  return hilbert3x4(q[0], q[1], q[2]);
}

// In-place exclusive scan of the kSortBins counts in bins (1024 threads).
__device__ __forceinline__ void block_scan_bins(uint32_t* bins, uint32_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int PER = kSortBins / kBuildThreads;
  uint32_t c[PER], s = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    c[k] = bins[tid * PER + k];
    s += c[k];
  }
  uint32_t incl = s;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += u;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t run = incl - s;
  for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    bins[tid * PER + k] = run;
    run += c[k];
  }
}

// Counting sort of n items by 12-bit Hilbert cell over [lo, hi]; emit(pos, i, v) for each item.
template <typename GET, typename EMIT>
__device__ void morton_sort(int n, GET get, EMIT emit, const float (&lo)[3], const float (&hi)[3], uint32_t* bins,
                            uint32_t* wsum) {
  const int tid = threadIdx.x;
  const CurveGrid g = curve_grid(lo, hi);
  for (int i = tid; i < kSortBins; i += kBuildThreads) bins[i] = 0u;
  __syncthreads();
  for (int i = tid; i < n; i += kBuildThreads) {
    float v[3];
    get(i, v);
    atomicAdd(&bins[curve_cell(g, v)], 1u);
  }
  __syncthreads();
  block_scan_bins(bins, wsum);
  __syncthreads();
  for (int i = tid; i < n; i += kBuildThreads) {
    float v[3];
    get(i, v);
    emit(static_cast<int>(atomicAdd(&bins[curve_cell(g, v)], 1u)), i, v);
  }
  __syncthreads();
}

}  // namespace dvcp
