// pkfma_stress.hip -- diagnostic: the round-4 VALU per-point pass of the
// sa2 / sa3 tables (U = W1f f + b1, one thread per (point, 4-channel group), weights from LDS) run
// many times on fixed inputs and compared bit for bit with its first result.  Run two instances
// at once to share the GPU between processes.  Variant 0 is the kernel as it was (hipcc forms
// v_pk_fma_f32 from its float4 FMA chain); variant 1 is the same source with packed fp32 math
// disabled for the function (target("no-packed-fp32-ops"): plain v_fma_f32).
//
//   pkfma_stress <variant 0|1> <iterations>   -> one line: variant, launches, mismatching floats,
//                                                 how many of them were the low / high element of a pair
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

constexpr int D = 32, C1 = 32, C0 = 3 + D, CG = C1 / 4, PPB = 256 / CG;

#define PRE_BODY                                                                                               \
  __shared__ float4 w[D][CG];                                                                                  \
  __shared__ float4 bias[CG];                                                                                  \
  const float* W1 = params;                                                                                    \
  const float* pb1 = W1 + C1 * C0;                                                                             \
  const float* ps1 = pb1 + C1;                                                                                 \
  const float* pt1 = ps1 + C1;                                                                                 \
  for (int i = threadIdx.x; i < D * C1; i += 256) {                                                            \
    const int k = i / C1, c = i % C1;                                                                          \
    reinterpret_cast<float*>(&w[k][0])[c] = W1[c * C0 + 3 + k] * ps1[c];                                       \
  }                                                                                                            \
  for (int c = threadIdx.x; c < C1; c += 256)                                                                  \
    reinterpret_cast<float*>(&bias[0])[c] =                                                                    \
        static_cast<float>(static_cast<double>(pb1[c]) * ps1[c] + static_cast<double>(pt1[c]));                \
  __syncthreads();                                                                                             \
  const int g = threadIdx.x % CG;                                                                              \
  const int64_t i = static_cast<int64_t>(blockIdx.x) * PPB + threadIdx.x / CG;                                 \
  if (i >= static_cast<int64_t>(B) * N) return;                                                                \
  const int b = static_cast<int>(i / N), n = static_cast<int>(i % N);                                          \
  const float4* fr = reinterpret_cast<const float4*>(feat + b * fb + n * fn);                                  \
  float4 acc = bias[g];                                                                                        \
  _Pragma("unroll 4") for (int v = 0; v < D / 4; ++v) {                                                        \
    const float4 q = fr[v];                                                                                    \
    const float fq[4] = {q.x, q.y, q.z, q.w};                                                                  \
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                            \
      const float4 wk = w[4 * v + e][g];                                                                       \
      acc.x = __fmaf_rn(wk.x, fq[e], acc.x);                                                                   \
      acc.y = __fmaf_rn(wk.y, fq[e], acc.y);                                                                   \
      acc.z = __fmaf_rn(wk.z, fq[e], acc.z);                                                                   \
      acc.w = __fmaf_rn(wk.w, fq[e], acc.w);                                                                   \
    }                                                                                                          \
  }                                                                                                            \
  reinterpret_cast<float4*>(U + i * C1)[g] = acc;

__global__ __launch_bounds__(256) void pre_packed(const float* __restrict__ feat, int64_t fb, int64_t fn, int N, int B,
                                                  const float* __restrict__ params, float* __restrict__ U) {
  PRE_BODY
}

__global__ __launch_bounds__(256) __attribute__((target("no-packed-fp32-ops"))) void pre_plain(
    const float* __restrict__ feat, int64_t fb, int64_t fn, int N, int B, const float* __restrict__ params,
    float* __restrict__ U) {
  PRE_BODY
}

__global__ void fill(float* p, int64_t n, uint32_t seed, float lo, float hi) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = lo + (hi - lo) * static_cast<float>(h >> 8) * (1.0f / 16777216.0f);
  }
}

// counts[0] mismatching floats, [1] of them at even channels (low element of a v_pk pair), [2] odd
__global__ void compare(const float* a, const float* b, int64_t n, unsigned long long* counts) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (__float_as_uint(a[i]) != __float_as_uint(b[i])) {
      atomicAdd(&counts[0], 1ull);
      atomicAdd(&counts[(i & 1) ? 2 : 1], 1ull);
    }
  }
}

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  const int B = 12, N = 10000;   // the two-rank test's sa2 pass: 2 x 6 clouds of 10000 points
  const int64_t nf = static_cast<int64_t>(B) * N * D, nu = static_cast<int64_t>(B) * N * C1;
  const int np = C1 * C0 + 3 * C1;
  float *feat, *params, *U, *ref;
  unsigned long long* counts;
  CHECK(hipMalloc(&feat, nf * 4));
  CHECK(hipMalloc(&params, np * 4));
  CHECK(hipMalloc(&U, nu * 4));
  CHECK(hipMalloc(&ref, nu * 4));
  CHECK(hipMalloc(&counts, 3 * 8));
  CHECK(hipMemset(counts, 0, 3 * 8));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, feat, nf, 17u, 0.0f, 0.3f);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, params, static_cast<int64_t>(np), 99u, -0.3f, 0.3f);
  // BN scale near 1, shift small: (params: W1, b1, scale1, shift1)
  hipLaunchKernelGGL(fill, dim3(1), dim3(64), 0, 0, params + C1 * C0 + C1, static_cast<int64_t>(C1), 5u, 0.9f, 1.1f);
  const dim3 grid((static_cast<int64_t>(B) * N + PPB - 1) / PPB), block(256);
  auto launch = [&](float* out) {
    if (variant == 0)
      hipLaunchKernelGGL(pre_packed, grid, block, 0, 0, feat, static_cast<int64_t>(N) * D, static_cast<int64_t>(D), N, B,
                         params, out);
    else
      hipLaunchKernelGGL(pre_plain, grid, block, 0, 0, feat, static_cast<int64_t>(N) * D, static_cast<int64_t>(D), N, B,
                         params, out);
  };
  launch(ref);
  CHECK(hipDeviceSynchronize());
  for (int it = 0; it < iters; ++it) {
    launch(U);
    hipLaunchKernelGGL(compare, dim3(1024), dim3(256), 0, 0, U, ref, nu, counts);
  }
  CHECK(hipDeviceSynchronize());
  unsigned long long h[3];
  CHECK(hipMemcpy(h, counts, sizeof(h), hipMemcpyDeviceToHost));
  printf("variant %d (%s): %d launches, %llu mismatching floats (even channel %llu, odd channel %llu)\n", variant,
         variant == 0 ? "v_pk_fma_f32" : "v_fma_f32", iters, h[0], h[1], h[2]);
  return 0;
}
