// fps_lab.hip -- standalone FPS step-latency laboratory (diagnostics, not part of the product).
//
// Builds to one executable: a uniform fp32 cloud batch (B x 3 x N, channel-first like the FE
// input), a scalar CPU FPS checker, and kernel variants of the sorted/pruned FPS with optional
// per-phase s_memtime instrumentation.  Variants that win here are transplanted into
// deepvcp-pointcloud-registration_amd/csrc/fps.hip.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 fps_lab.hip -o fps_lab
//   ./fps_lab [B N npoint]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kWave = 64;

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ float dpp_maxf(float v) {
  const int o = __builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWS, 0xF, false);
  return fmaxf(v, __int_as_float(o));
}
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ int dpp_mini(int v) {
  const int o = __builtin_amdgcn_update_dpp(v, v, CTRL, ROWS, 0xF, false);
  return min(v, o);
}
__device__ __forceinline__ float wave_maxf_dpp(float v) {
  v = dpp_maxf<0x111>(v);
  v = dpp_maxf<0x112>(v);
  v = dpp_maxf<0x114>(v);
  v = dpp_maxf<0x118>(v);
  v = dpp_maxf<0x142, 0xA>(v);
  v = dpp_maxf<0x143, 0xC>(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ int wave_mini_dpp(int v) {
  v = dpp_mini<0x111>(v);
  v = dpp_mini<0x112>(v);
  v = dpp_mini<0x114>(v);
  v = dpp_mini<0x118>(v);
  v = dpp_mini<0x142, 0xA>(v);
  v = dpp_mini<0x143, 0xC>(v);
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ float rlf(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float box_lb2(float cx, float cy, float cz, const float (&bx)[6]) {
  const float ex = fmaxf(fmaxf(bx[0] - cx, cx - bx[3]), 0.f);
  const float ey = fmaxf(fmaxf(bx[1] - cy, cy - bx[4]), 0.f);
  const float ez = fmaxf(fmaxf(bx[2] - cz, cz - bx[5]), 0.f);
  return (ex * ex + ey * ey) + ez * ez;
}
__device__ __forceinline__ uint32_t spread4(uint32_t v) {
  v &= 0xF;
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4) | ((v & 8u) << 6);
}
__device__ __forceinline__ uint64_t tnow() {
  uint64_t t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

struct alignas(16) Slot {
  float v;
  int i;
  float x, y, z;
};

// Variant flags
enum : int {
  kTiming = 1,     // per-phase s_memtime sums per wave
  kReadlane = 2,   // take the winner's coordinates from registers (readlane), not a 2nd LDS read
  kGroupPrune = 4, // additionally skip 64-point groups whose box is beyond the wave's max
  kNoPrune = 8,    // no pruning at all
  kSimdRemap = 16, // assign Morton ranges to waves by hardware SIMD id
};

constexpr int kProf = 8;  // per wave: phases 0..4, active steps, hw_id, groups run

template <int THREADS, int PPT, int F>
__global__ __launch_bounds__(THREADS) void fps_lab_kernel(const float* __restrict__ xyz, int N, int npoint,
                                                          const int* __restrict__ start, int* __restrict__ out_idx,
                                                          unsigned long long* __restrict__ prof) {
  constexpr int W = THREADS / kWave;
  constexpr int kBins = 4096;
  __shared__ uint32_t bins[kBins];
  __shared__ uint16_t perm[THREADS * PPT];
  __shared__ Slot slots[2][W];
  __shared__ float red[2][3][W];
  __shared__ uint32_t wsum[W];
  __shared__ int wmap[W];

  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, hw_wave = tid >> 6;
  const float* X = xyz + static_cast<int64_t>(b) * 3 * N;
  const float* Y = X + N;
  const float* Z = Y + N;

  // SIMD-aware range assignment: range r -> the wave such that ranges r, r+1, r+2, r+3 land on
  // different SIMDs.
  int wave = hw_wave;
  const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  if constexpr ((F & kSimdRemap) != 0) {
    if (lane == 0) wmap[hw_wave] = (hwid >> 4) & 3;
    __syncthreads();
    const int my_simd = (hwid >> 4) & 3;
    int rank = 0;
    for (int w = 0; w < hw_wave; ++w) rank += (wmap[w] == my_simd);
    wave = rank * 4 + my_simd;  // assumes W/4 waves per SIMD
    __syncthreads();
  }

  float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
  for (int n = tid; n < N; n += THREADS) {
    const float v[3] = {X[n], Y[n], Z[n]};
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
      red[0][a][hw_wave] = lo[a];
      red[1][a][hw_wave] = hi[a];
    }
  }
  for (int i = tid; i < kBins; i += THREADS) bins[i] = 0u;
  __syncthreads();
  float blo[3], bsc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float l = red[0][a][0], h = red[1][a][0];
    for (int w = 1; w < W; ++w) {
      l = fminf(l, red[0][a][w]);
      h = fmaxf(h, red[1][a][w]);
    }
    blo[a] = l;
    bsc[a] = h > l ? 16.f / (h - l) : 0.f;
  }
  auto cell_of = [&](int n) -> uint32_t {
    const float v[3] = {X[n], Y[n], Z[n]};
    uint32_t c = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      int q = static_cast<int>((v[a] - blo[a]) * bsc[a]);
      q = q < 0 ? 0 : (q > 15 ? 15 : q);
      c |= spread4(static_cast<uint32_t>(q)) << a;
    }
    return c;
  };
  for (int n = tid; n < N; n += THREADS) atomicAdd(&bins[cell_of(n)], 1u);
  __syncthreads();
  {
    constexpr int PER = kBins / THREADS;
    uint32_t v[PER], s = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      v[k] = bins[tid * PER + k];
      s += v[k];
    }
    uint32_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t u = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += u;
    }
    if (lane == 63) wsum[hw_wave] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < hw_wave; ++w) base += wsum[w];
    uint32_t run = base + incl - s;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      bins[tid * PER + k] = run;
      run += v[k];
    }
  }
  __syncthreads();
  for (int n = tid; n < N; n += THREADS) perm[atomicAdd(&bins[cell_of(n)], 1u)] = static_cast<uint16_t>(n);
  __syncthreads();

  float px[PPT], py[PPT], pz[PPT], dmin[PPT];
  int pid[PPT];
  float wb[6] = {1e30f, 1e30f, 1e30f, -1e30f, -1e30f, -1e30f};
  float gb[6];  // lane p (< PPT) holds group p's box (kGroupPrune)
#pragma unroll
  for (int a = 0; a < 6; ++a) gb[a] = a < 3 ? 1e30f : -1e30f;
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int pos = wave * (kWave * PPT) + p * kWave + lane;
    float g[6];
    if (pos < N) {
      const int n = perm[pos];
      pid[p] = n;
      px[p] = X[n];
      py[p] = Y[n];
      pz[p] = Z[n];
      dmin[p] = 1e10f;
      g[0] = g[3] = px[p];
      g[1] = g[4] = py[p];
      g[2] = g[5] = pz[p];
    } else {
      pid[p] = 0x7FFFFFFF;
      px[p] = py[p] = pz[p] = 0.f;
      dmin[p] = -1.0f;
      g[0] = g[1] = g[2] = 1e30f;
      g[3] = g[4] = g[5] = -1e30f;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float l = g[a], h = g[3 + a];
      for (int off = 32; off > 0; off >>= 1) {
        l = fminf(l, __shfl_xor(l, off, kWave));
        h = fmaxf(h, __shfl_xor(h, off, kWave));
      }
      wb[a] = fminf(wb[a], l);
      wb[3 + a] = fmaxf(wb[3 + a], h);
      if (lane == p) {
        gb[a] = l;
        gb[3 + a] = h;
      }
    }
  }

  int cur = start[b];
  float cx = X[cur], cy = Y[cur], cz = Z[cur];
  int* oi = out_idx + static_cast<int64_t>(b) * npoint;
  float wv = 1e30f;
  int wi = 0x7FFFFFFF;
  float wx = 0, wy = 0, wz = 0;
  const bool empty_wave = wave * (kWave * PPT) >= N;
  uint64_t ph[5] = {0, 0, 0, 0, 0};
  uint64_t nact = 0, ngroups = 0;

  for (int step = 0; step < npoint; ++step) {
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    if constexpr ((F & kTiming) != 0) t0 = tnow();
    if (tid == 0) oi[step] = cur;
    const bool active = !empty_wave && ((F & kNoPrune) != 0 || !(box_lb2(cx, cy, cz, wb) >= wv));
    if (active) {
      float bv = -1.0f;
      int bi = 0x7FFFFFFF;
      float bx = 0, by = 0, bz = 0;
      uint64_t gmask = ~0ull;
      if constexpr ((F & kGroupPrune) != 0) gmask = __ballot(lane < PPT && !(box_lb2(cx, cy, cz, gb) >= wv));
      if constexpr ((F & kTiming) != 0) ngroups += __builtin_popcountll(gmask & ((1ull << PPT) - 1));
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        if ((gmask >> p) & 1) {
          const float dx = px[p] - cx, dy = py[p] - cy, dz = pz[p] - cz;
          const float d = (dx * dx + dy * dy) + dz * dz;
          dmin[p] = fminf(d, dmin[p]);
        }
        // still track skipped groups' cached minima (they are unchanged)
        const bool better = (dmin[p] > bv) | ((dmin[p] == bv) & (pid[p] < bi));
        bv = better ? dmin[p] : bv;
        bi = better ? pid[p] : bi;
        bx = better ? px[p] : bx;
        by = better ? py[p] : by;
        bz = better ? pz[p] : bz;
      }
      if constexpr ((F & kTiming) != 0) t1 = tnow();
      wv = wave_maxf_dpp(bv);
      const uint64_t tied = __ballot(bv == wv);
      int wl;
      if ((tied & (tied - 1)) == 0) {
        wl = __ffsll(static_cast<long long>(tied)) - 1;
      } else {
        const int mi = wave_mini_dpp(bv == wv ? bi : 0x7FFFFFFF);
        wl = __ffsll(static_cast<long long>(__ballot((bv == wv) & (bi == mi)))) - 1;
      }
      wi = __builtin_amdgcn_readlane(bi, wl);
      wx = rlf(bx, wl);
      wy = rlf(by, wl);
      wz = rlf(bz, wl);
      nact++;
    } else if constexpr ((F & kTiming) != 0) {
      t1 = tnow();
    }
    if constexpr ((F & kTiming) != 0) t2 = tnow();
    Slot* buf = slots[step & 1];
    if (lane == 0) buf[wave] = Slot{empty_wave ? -2.0f : wv, empty_wave ? 0x7FFFFFFF : wi, wx, wy, wz};
    lds_barrier();
    if constexpr ((F & kTiming) != 0) t3 = tnow();
    const Slot mine = buf[lane & (W - 1)];
    float v = mine.v;
    v = dpp_maxf<0x111, 0x1>(v);
    v = dpp_maxf<0x112, 0x1>(v);
    v = dpp_maxf<0x114, 0x1>(v);
    if constexpr (W > 8) v = dpp_maxf<0x118, 0x1>(v);
    const float gv = rlf(v, W - 1);
    const uint64_t tied = __ballot((lane < W) & (mine.v == gv));
    int ws;
    if ((tied & (tied - 1)) == 0) {
      ws = __ffsll(static_cast<long long>(tied)) - 1;
    } else {
      int ii = ((lane < W) & (mine.v == gv)) ? mine.i : 0x7FFFFFFF;
      ii = dpp_mini<0x111, 0x1>(ii);
      ii = dpp_mini<0x112, 0x1>(ii);
      ii = dpp_mini<0x114, 0x1>(ii);
      if constexpr (W > 8) ii = dpp_mini<0x118, 0x1>(ii);
      const int mi = __builtin_amdgcn_readlane(ii, W - 1);
      ws = __ffsll(static_cast<long long>(__ballot((lane < W) & (mine.v == gv) & (mine.i == mi)))) - 1;
    }
    if constexpr ((F & kReadlane) != 0) {
      cur = __builtin_amdgcn_readlane(mine.i, ws);
      cx = rlf(mine.x, ws);
      cy = rlf(mine.y, ws);
      cz = rlf(mine.z, ws);
    } else {
      cur = buf[ws].i;
      cx = buf[ws].x;
      cy = buf[ws].y;
      cz = buf[ws].z;
    }
    if constexpr ((F & kTiming) != 0) {
      const uint64_t t4 = tnow();
      ph[0] += t1 - t0;
      ph[1] += t2 - t1;
      ph[2] += t3 - t2;
      ph[3] += t4 - t3;
    }
  }
  if (prof && lane == 0) {
    unsigned long long* o = prof + (static_cast<int64_t>(b) * W + hw_wave) * kProf;
    o[0] = ph[0];
    o[1] = ph[1];
    o[2] = ph[2];
    o[3] = ph[3];
    o[4] = wave;
    o[5] = nact;
    o[6] = hwid;
    o[7] = ngroups;
  }
}

// ------------------------------------------------------------------------------------- host
static void cpu_fps(const float* X, int N, int npoint, int start, std::vector<int>& out) {
  const float* Y = X + N;
  const float* Z = Y + N;
  std::vector<float> dmin(N, 1e10f);
  int cur = start;
  out.resize(npoint);
  for (int s = 0; s < npoint; ++s) {
    out[s] = cur;
    const float cx = X[cur], cy = Y[cur], cz = Z[cur];
    float bv = -1.f;
    int bi = 0;
    for (int n = 0; n < N; ++n) {
      const float dx = X[n] - cx, dy = Y[n] - cy, dz = Z[n] - cz;
      const float d = (dx * dx + dy * dy) + dz * dz;
      if (d < dmin[n]) dmin[n] = d;
      if (dmin[n] > bv) {
        bv = dmin[n];
        bi = n;
      }
    }
    cur = bi;
  }
}

using KernelFn = void (*)(const float*, int, int, const int*, int*, unsigned long long*);

struct Variant {
  const char* name;
  KernelFn fn;
  int threads;
  int ppt;
  bool timing;
};

#define V(T, P, F, NAME) Variant{NAME, fps_lab_kernel<T, P, F>, T, P, (F & kTiming) != 0}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16;
  const int N = argc > 2 ? atoi(argv[2]) : 16384;
  const int npoint = argc > 3 ? atoi(argv[3]) : 10000;
  const int ncheck = 2;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<float> h(static_cast<size_t>(B) * 3 * N);
  for (auto& v : h) v = U(rng);
  std::vector<int> hs(B);
  for (int b = 0; b < B; ++b) hs[b] = static_cast<int>(rng() % N);
  std::vector<std::vector<int>> want(ncheck);
  for (int b = 0; b < ncheck && b < B; ++b) cpu_fps(h.data() + static_cast<size_t>(b) * 3 * N, N, npoint, hs[b], want[b]);

  float* dx;
  int *ds, *dout;
  unsigned long long* dprof;
  CK(hipMalloc(&dx, h.size() * 4));
  CK(hipMalloc(&ds, B * 4));
  CK(hipMalloc(&dout, static_cast<size_t>(B) * npoint * 4));
  CK(hipMalloc(&dprof, static_cast<size_t>(B) * 16 * kProf * 8));
  CK(hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, hs.data(), B * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  std::vector<Variant> vars = {
      V(1024, 16, 0, "base"),
      V(1024, 16, kTiming, "base+timing"),
      V(1024, 16, kReadlane, "readlane"),
      V(1024, 16, kReadlane | kNoPrune, "readlane noprune"),
      V(1024, 16, kReadlane | kGroupPrune, "readlane+groupprune"),
      V(1024, 16, kReadlane | kGroupPrune | kTiming, "readlane+groupprune+timing"),
      V(1024, 16, kReadlane | kSimdRemap, "readlane+simdremap"),
      V(1024, 16, kReadlane | kSimdRemap | kTiming, "readlane+simdremap+timing"),
      V(1024, 16, kReadlane | kSimdRemap | kGroupPrune, "readlane+simdremap+groupprune"),
      V(512, 32, kReadlane | kGroupPrune, "512thr readlane+groupprune"),
      V(512, 32, kReadlane | kGroupPrune | kTiming, "512thr readlane+groupprune+timing"),
      V(256, 64, kReadlane | kGroupPrune, "256thr readlane+groupprune"),
  };
  std::vector<int> got(static_cast<size_t>(B) * npoint);
  for (const auto& v : vars) {
    if ((N + v.threads * v.ppt - 1) / (v.threads * v.ppt) > 1) continue;
    CK(hipMemset(dprof, 0, static_cast<size_t>(B) * 16 * kProf * 8));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(v.fn, dim3(B), dim3(v.threads), 0, 0, dx, N, npoint, ds, dout, dprof);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    CK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int b = 0; b < ncheck && b < B; ++b)
      for (int s = 0; s < npoint; ++s) bad += got[static_cast<size_t>(b) * npoint + s] != want[b][s];
    printf("%-40s threads %4d ppt %3d  %8.3f ms  %6.3f us/step  mismatches %d\n", v.name, v.threads, v.ppt, best,
           1e3f * best / npoint, bad);
    if (v.timing) {
      const int W = v.threads / 64;
      std::vector<unsigned long long> pr(static_cast<size_t>(B) * 16 * kProf);
      CK(hipMemcpy(pr.data(), dprof, pr.size() * 8, hipMemcpyDeviceToHost));
      // cloud 0: per wave phases (cycles/step), active steps, SIMD id
      for (int w = 0; w < W; ++w) {
        const unsigned long long* o = &pr[(static_cast<size_t>(0) * W + w) * kProf];
        printf("   hw_wave %2d range %2llu simd %llu wave_slot %2llu: points %7.1f  wred %6.1f  barrier %7.1f  "
               "bred %6.1f cyc/step  active %5.1f%%  groups/act %.2f\n",
               w, o[4], (o[6] >> 4) & 3, o[6] & 15, double(o[0]) / npoint, double(o[1]) / npoint,
               double(o[2]) / npoint, double(o[3]) / npoint, 100.0 * o[5] / npoint,
               o[5] ? double(o[7]) / o[5] : 0.0);
      }
    }
  }
  return 0;
}
