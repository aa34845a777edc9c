// poison.hip -- diagnostic only (tools/diag_poison.py): fill every CU's LDS and a wave's worth of
// VGPRs with a chosen bit pattern, so a kernel launched right after that reads LDS or registers it
// never wrote sees the pattern instead of what its own previous workgroups left there.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kLdsBytes = 160 * 1024;

__global__ __launch_bounds__(1024) void poison_lds_kernel(uint32_t pattern, uint32_t* sink) {
  extern __shared__ uint32_t s[];
  for (int i = threadIdx.x; i < kLdsBytes / 4; i += blockDim.x) s[i] = pattern ^ static_cast<uint32_t>(i & 0xF);
  __syncthreads();
  if (s[(threadIdx.x * 977) % (kLdsBytes / 4)] == 0x12345678u) sink[0] = 1u;  // keeps the stores
}

// 256 threads x ~480 VGPRs of the pattern; each value is passed to an empty asm so it is
// materialised in a register and kept live to the end.
__global__ __launch_bounds__(256) void poison_vgpr_kernel(uint32_t pattern, uint32_t* sink) {
  uint32_t r[448];
#pragma unroll
  for (int j = 0; j < 448; ++j) {
    r[j] = pattern ^ static_cast<uint32_t>(j & 0xF);
    asm volatile("" : "+v"(r[j]));
  }
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 448; ++j) {
    asm volatile("" : "+v"(r[j]));
    acc ^= r[j];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int dvcp_poison(uint32_t pattern, void* sink, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  static bool init = false;
  if (!init) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(poison_lds_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes) != hipSuccess)
      return 1;
    init = true;
  }
  hipLaunchKernelGGL(poison_lds_kernel, dim3(256 * 4), dim3(1024), kLdsBytes, st, pattern,
                     static_cast<uint32_t*>(sink));
  hipLaunchKernelGGL(poison_vgpr_kernel, dim3(256 * 8), dim3(256), 0, st, pattern, static_cast<uint32_t*>(sink));
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// a single-workgroup kernel that spins for `ticks` of the 100 MHz constant clock: shifts a stream's
// next launch by a known delay (tools/diag_poison.py --delays)
__global__ void spin_kernel(uint64_t ticks, uint32_t* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (t == 0x12345678u) sink[0] = 1u;
}

extern "C" int dvcp_spin(uint64_t ticks, void* sink, void* stream) {
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), ticks,
                     static_cast<uint32_t*>(sink));
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
