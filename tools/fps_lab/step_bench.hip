// step_bench.hip -- floors of the per-step synchronisation patterns a serial argmax chain can
// use (diagnostics for the FPS design).  Each kernel runs `steps` dependent
// rounds in one workgroup per CU-sized cloud and reports clocks per round.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_max_i(int v) {
  return max(v, __builtin_amdgcn_update_dpp(static_cast<int>(0x80000000), v, CTRL, ROWS, 0xF, false));
}

// mode 0: barrier only
// mode 1: lane 0 writes a 16 B slot, barrier, every lane reads slot[lane & (W-1)], readlane 0
// mode 2: mode 1 + DPP int-max over W lanes + readlane + ballot/ffs + 3 readlanes (FPS v3 tail)
// mode 3: lane 0 ds_max_u64 into one word, barrier, every lane reads it, barrier (reset)
// mode 4: wave-wide 64-lane DPP max + readlane only (no cross-wave sync)
template <int THREADS, int MODE>
__global__ __launch_bounds__(THREADS) void step_kernel(int steps, int seed, int* out, unsigned long long* clk) {
  constexpr int W = THREADS / 64;
  __shared__ int4 slots[2][W];
  __shared__ unsigned long long key[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int v = seed ^ (threadIdx.x * 2654435761u);
  if (threadIdx.x < 2) key[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
    if constexpr (MODE == 0) {
      lds_barrier();
      v += s;
    } else if constexpr (MODE == 1 || MODE == 2) {
      int4* buf = slots[s & 1];
      if (lane == 0) buf[wave] = make_int4(v & 0x7FFFFFFF, v, v + 1, v + 2);
      lds_barrier();
      const int4 m = buf[lane & (W - 1)];
      if constexpr (MODE == 1) {
        v = __builtin_amdgcn_readlane(m.x, 0) + wave;
      } else {
        int x = m.x;
        x = dpp_max_i<0x111, 0x1>(x);
        if constexpr (W > 2) x = dpp_max_i<0x112, 0x1>(x);
        if constexpr (W > 4) x = dpp_max_i<0x114, 0x1>(x);
        if constexpr (W > 8) x = dpp_max_i<0x118, 0x1>(x);
        const int g = __builtin_amdgcn_readlane(x, W - 1);
        const uint64_t t = __ballot((lane < W) & (m.x == g));
        const int ws = __ffsll(static_cast<long long>(t)) - 1;
        v = __builtin_amdgcn_readlane(m.y, ws) + __builtin_amdgcn_readlane(m.z, ws) +
            __builtin_amdgcn_readlane(m.w, ws) + wave;
      }
    } else if constexpr (MODE == 3) {
      if (lane == 0) atomicMax(&key[s & 1], static_cast<unsigned long long>(static_cast<uint32_t>(v)) << 20);
      lds_barrier();
      const unsigned long long k = key[s & 1];
      if (threadIdx.x == 0) key[(s + 1) & 1] = 0;
      v = static_cast<int>(k >> 20) + wave;
    } else {
      int x = v & 0x7FFFFFFF;
      x = dpp_max_i<0x111, 0xF>(x);
      x = dpp_max_i<0x112, 0xF>(x);
      x = dpp_max_i<0x114, 0xF>(x);
      x = dpp_max_i<0x118, 0xF>(x);
      x = dpp_max_i<0x142, 0xA>(x);
      x = dpp_max_i<0x143, 0xC>(x);
      v = __builtin_amdgcn_readlane(x, 63) + lane;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x] = v;
    clk[blockIdx.x] = t1 - t0;
  }
}

template <int THREADS, int MODE>
static void run(const char* name, int steps, int* dout, unsigned long long* dclk) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((step_kernel<THREADS, MODE>), dim3(16), dim3(THREADS), 0, 0, steps, r, dout, dclk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  unsigned long long c;
  CK(hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost));
  printf("%-44s threads %4d: %7.1f ns/step  %7.1f clk/step (s_memtime)\n", name, THREADS, 1e6 * best / steps,
         double(c) / steps);
}

int main() {
  int* dout;
  unsigned long long* dclk;
  CK(hipMalloc(&dout, 64 * 4));
  CK(hipMalloc(&dclk, 64 * 8));
  const int steps = 100000;
  run<512, 0>("barrier only", steps, dout, dclk);
  run<1024, 0>("barrier only", steps, dout, dclk);
  run<256, 0>("barrier only", steps, dout, dclk);
  run<512, 1>("slot write + barrier + read", steps, dout, dclk);
  run<1024, 1>("slot write + barrier + read", steps, dout, dclk);
  run<512, 2>("slot + DPP reduce + readlanes (v3 tail)", steps, dout, dclk);
  run<1024, 2>("slot + DPP reduce + readlanes (v3 tail)", steps, dout, dclk);
  run<256, 2>("slot + DPP reduce + readlanes (v3 tail)", steps, dout, dclk);
  run<512, 3>("ds_max_u64 + barrier + read", steps, dout, dclk);
  run<1024, 3>("ds_max_u64 + barrier + read", steps, dout, dclk);
  run<64, 4>("wave DPP max + readlane only", steps, dout, dclk);
  run<512, 4>("wave DPP max + readlane only", steps, dout, dclk);
  return 0;
}
