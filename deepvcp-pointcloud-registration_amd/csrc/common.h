// common.h -- shared device helpers for libdvcp_hip.so (gfx950 / CDNA4, wave64).
//
// Build rule: every translation unit is compiled with -ffp-contract=off.  The discrete
// stages (FPS, ball query, kNN, candidate grid) must round exactly like the reference's
// torch CPU ops, so every fused multiply-add below is written out explicitly (__fma_rn)
// where the reference's BLAS uses one, and nowhere else.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dvcp.h"

namespace dvcp {

void set_error(const char* fmt, ...);
int launch_status(const char* what);

constexpr int kWave = 64;

// Strided point access: coordinate c of point n of batch b.
template <typename T>
struct PointsView {
  const T* p;
  int64_t sb, sc, sn;
  __device__ __forceinline__ T at(int b, int c, int64_t n) const {
    return p[b * sb + c * sc + n * sn];
  }
  // fp32 points in (x, y, z, pad) rows (sc == 1, sn == 4, 16-byte aligned rows: dvcp_points_pack4)
  __host__ __device__ __forceinline__ bool rows4() const {
    return sizeof(T) == 4 && sc == 1 && sn == 4 && (sb & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  }
  // the three coordinates of point n: one 16-byte load from one line for rows4() views (a gathered
  // point of the (B, 3, N) layout costs three 4-byte loads from three lines), else three loads.
  // rows4() depends on kernel arguments only: the test is wave-uniform and hoisted.
  __device__ __forceinline__ void load3(int b, int64_t n, T& x, T& y, T& z) const {
    if constexpr (sizeof(T) == 4) {
      if (rows4()) {
        const float4 q = *reinterpret_cast<const float4*>(p + b * sb + 4 * n);
        x = q.x;
        y = q.y;
        z = q.z;
        return;
      }
    }
    x = at(b, 0, n);
    y = at(b, 1, n);
    z = at(b, 2, n);
  }
};

template <typename T>
__device__ __forceinline__ T fma_rn(T a, T b, T c);
template <>
__device__ __forceinline__ float fma_rn<float>(float a, float b, float c) { return __fmaf_rn(a, b, c); }
template <>
__device__ __forceinline__ double fma_rn<double>(double a, double b, double c) { return __fma_rn(a, b, c); }

// Correctly rounded fp32 sqrt (torch's CPU sqrt is IEEE): fp64 sqrt then narrowing is exact
// for fp32 inputs (53 >= 2*24 + 2), and the fp64 sqrt is correctly rounded.
__device__ __forceinline__ float sqrt_rn(float x) { return static_cast<float>(__dsqrt_rn(static_cast<double>(x))); }
__device__ __forceinline__ double sqrt_rn(double x) { return __dsqrt_rn(x); }

// |p|^2 as torch.sum(p ** 2, -1) rounds it: ((x*x + y*y) + z*z), no fma.
template <typename T>
__device__ __forceinline__ T sumsq3(T x, T y, T z) { return (x * x + y * y) + z * z; }

// c . p as MKL's [s|d]gemm rounds a K=3 product: fma(z, z', fma(y, y', x*x')).
template <typename T>
__device__ __forceinline__ T dot3_blas(T ax, T ay, T az, T bx, T by, T bz) {
  return fma_rn<T>(az, bz, fma_rn<T>(ay, by, ax * bx));
}

// pointnet2_utils.py:37-39: ((-2 * dot) + |src|^2) + |dst|^2.
template <typename T>
__device__ __forceinline__ T expansion_d2(T dot, T ss_src, T ss_dst) {
  T d = static_cast<T>(-2) * dot;
  d = d + ss_src;
  return d + ss_dst;
}

// ---------------------------------------------------------------------------------------
// Argmax keys: larger value wins, ties go to the lower index.  Non-negative floats only
// (FPS distances); an empty slot is key 0, which every real key beats.
__device__ __forceinline__ uint64_t argmax_key(float v, uint32_t idx) {
  return (static_cast<uint64_t>(__float_as_uint(v)) << 32) | static_cast<uint64_t>(0xFFFFFFFFu - idx);
}
__device__ __forceinline__ uint32_t key_index(uint64_t k) {
  return 0xFFFFFFFFu - static_cast<uint32_t>(k & 0xFFFFFFFFull);
}
// Order-preserving map of any float to uint32 (for top-k on signed scores).
__device__ __forceinline__ uint32_t float_order(float v) {
  uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t k) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t o = __shfl_xor(k, off, kWave);
    k = o > k ? o : k;
  }
  return k;
}

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup release/acquire: it
// also waits for every outstanding global store (vmcnt(0)), which in a serial per-step loop
// that streams its outputs puts an HBM write round trip on every step.  Here only LDS traffic
// crosses the barrier, so wait for LDS (lgkmcnt) and barrier; "memory" keeps the compiler from
// moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Block-wide sum of one value per thread (blockDim multiple of 64, <= 1024).  `scratch`
// holds >= 16 T.  Every thread returns the total.  The summation order is fixed.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  T s = 0;
  for (int w = 0; w < nw; ++w) s += scratch[w];
  return s;
}

__device__ __forceinline__ float block_max_f(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max_f(v);
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  float m = scratch[0];
  for (int w = 1; w < nw; ++w) m = fmaxf(m, scratch[w]);
  return m;
}

// y = W x + b with W (COUT x CIN) row-major at p, bias right after it.  Wave-uniform
// compile-time addresses -> scalar loads (SGPR operands).
template <int CIN, int COUT>
__device__ __forceinline__ void linear_sgpr(const float (&x)[CIN], float (&y)[COUT], const float* __restrict__ p) {
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    float acc = 0.0f;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc = __fmaf_rn(p[co * CIN + ci], x[ci], acc);
    y[co] = acc + p[CIN * COUT + co];
  }
}

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace dvcp

#define DVCP_REQUIRE(cond, ...)       \
  do {                                \
    if (!(cond)) {                    \
      ::dvcp::set_error(__VA_ARGS__); \
      return DVCP_EINVAL;             \
    }                                 \
  } while (0)
