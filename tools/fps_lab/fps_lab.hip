// fps_lab.hip -- standalone FPS step-latency laboratory (diagnostics, not part of the product).
//
// Compiles the production kernel template (csrc/fps.hip) into one executable together with a
// scalar CPU FPS checker, runs configurations of it on a uniform fp32 cloud batch
// (B x 3 x N, channel-first like the FE input) and prints us/step, mismatches against the CPU
// result, and -- for the TIMING instantiation -- per-wave step-phase clocks.
//
//   make -C tools/fps_lab            (see Makefile there)
//   ./tools/fps_lab/fps_lab [B N npoint]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../deepvcp-pointcloud-registration_amd/csrc/fps.hip"

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

using dvcp::PointsView;

static void cpu_fps(const float* X, int N, int npoint, int64_t start, std::vector<int64_t>& out) {
  const float* Y = X + N;
  const float* Z = Y + N;
  std::vector<float> dmin(N, 1e10f);
  int64_t cur = start;
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

using KernelFn = void (*)(PointsView<float>, int, int, const int64_t*, int64_t*, float*, unsigned long long*);

struct Config {
  const char* name;
  KernelFn fn;
  int threads, ppt;
  bool timing;
  bool sel = false;  // a threshold-select instantiation (its TIMING words are round statistics)
};

#define CFG(T, P, PR, TM, NAME) Config{NAME, dvcp::fps_kernel<float, T, P, PR, TM>, T, P, TM}
#define SEL(P, NAME) Config{NAME, dvcp::fps_select_kernel<float, P, false>, 512, P, false}
#define SELT(P, NAME) Config{NAME, dvcp::fps_select_kernel<float, P, true>, 512, P, true, true}
#define SEL16(P, NAME) Config{NAME, dvcp::fps_select_kernel<float, P, false, 1024>, 1024, P, false}
#define SELT16(P, NAME) Config{NAME, dvcp::fps_select_kernel<float, P, true, 1024>, 1024, P, true, true}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16;
  const int N = argc > 2 ? atoi(argv[2]) : 16384;
  const int npoint = argc > 3 ? atoi(argv[3]) : 10000;
  const int ncheck = B < 2 ? B : 2;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<float> h(static_cast<size_t>(B) * 3 * N);
  for (auto& v : h) v = U(rng);
  std::vector<int64_t> hs(B);
  for (int b = 0; b < B; ++b) hs[b] = static_cast<int64_t>(rng() % N);
  std::vector<std::vector<int64_t>> want(ncheck);
  for (int b = 0; b < ncheck; ++b) cpu_fps(h.data() + static_cast<size_t>(b) * 3 * N, N, npoint, hs[b], want[b]);

  float *dx, *dox;
  int64_t *ds, *dout;
  unsigned long long* dprof;
  const size_t prof_words = static_cast<size_t>(B) * 16 * dvcp::kFpsProf;
  CK(hipMalloc(&dx, h.size() * 4));
  CK(hipMalloc(&ds, B * 8));
  CK(hipMalloc(&dout, static_cast<size_t>(B) * npoint * 8));
  CK(hipMalloc(&dox, static_cast<size_t>(B) * 3 * npoint * 4));
  CK(hipMalloc(&dprof, prof_words * 8));
  CK(hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, hs.data(), B * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const PointsView<float> view{dx, 3LL * N, N, 1};

  const std::vector<Config> cfgs = {
      SEL(32, "select 512x32"),
      SELT(32, "select 512x32 +stats"),
      SEL16(16, "select 1024x16"),
      SELT16(16, "select 1024x16 +stats"),
      SEL(20, "select 512x20"),
      SELT(20, "select 512x20 +stats"),
      SEL16(10, "select 1024x10"),
      SELT16(10, "select 1024x10 +stats"),
      CFG(512, 32, true, false, "v3 512x32 prune"),
      CFG(512, 32, true, true, "v3 512x32 prune +timing"),
      CFG(512, 32, false, false, "v3 512x32 noprune"),
      CFG(512, 24, true, false, "v3 512x24 prune"),
      CFG(512, 16, true, false, "v3 512x16 prune"),
      CFG(1024, 16, true, false, "v3 1024x16 prune"),
      CFG(1024, 16, true, true, "v3 1024x16 prune +timing"),
      CFG(1024, 8, true, false, "v3 1024x8 prune"),
      CFG(256, 16, true, false, "v3 256x16 prune"),
  };
  std::vector<int64_t> got(static_cast<size_t>(B) * npoint);
  const std::vector<unsigned long long> pr_dummy(1);
  // split select (round 6): S workgroups per cloud; `fps_lab B N npoint parts` runs only these
  if (argc > 4) {
    struct PartCfg {
      const char* name;
      void (*fn)(PointsView<float>, int, int, const int64_t*, int64_t*, float*, dvcp::FpsPartArgs, unsigned long long*);
      int threads, ppt, S;
      bool timing;
    };
#define PART(P, NT, S, TM, NAME) PartCfg{NAME, dvcp::fps_part_kernel<P, NT, TM>, NT, P, S, TM}
    const std::vector<PartCfg> pcs = {
        PART(8, 1024, 2, false, "part 2 x 1024x8"),      PART(8, 1024, 2, true, "part 2 x 1024x8 +stats"),
        PART(4, 1024, 4, false, "part 4 x 1024x4"),      PART(4, 1024, 4, true, "part 4 x 1024x4 +stats"),
        PART(2, 1024, 8, false, "part 8 x 1024x2"),      PART(2, 1024, 8, true, "part 8 x 1024x2 +stats"),
        PART(8, 512, 4, false, "part 4 x 512x8"),        PART(8, 512, 4, true, "part 4 x 512x8 +stats"),
        PART(8, 1024, 8, false, "part 8 x 1024x8"),      PART(8, 1024, 8, true, "part 8 x 1024x8 +stats"),
        PART(16, 1024, 4, false, "part 4 x 1024x16"),    PART(16, 1024, 4, true, "part 4 x 1024x16 +stats"),
    };
    // argv[6]: 1 (default) roles by ticket, 0 by blockIdx
    const bool tickets = argc > 6 ? atoi(argv[6]) != 0 : true;
#undef PART
    uint64_t* dws;
    const size_t ws_bytes = static_cast<size_t>(dvcp::fps_workspace_bytes(B, N));
    CK(hipMalloc(&dws, ws_bytes));
    const size_t pprof_words = static_cast<size_t>(B) * 8 * 16 * dvcp::kFpsProf;
    unsigned long long* dpp;
    CK(hipMalloc(&dpp, pprof_words * 8));
    for (const auto& c : pcs) {
      const int groups = (N + 63) / 64, gpart = (groups + c.S - 1) / c.S;
      if (gpart > c.ppt * (c.threads / 64) || (c.ppt > 2 * gpart / (c.threads / 64) + 2 && c.ppt >= 8)) continue;
      const dvcp::FpsPartWs w = dvcp::fps_part_ws(B, N, c.S);
      const int capw = dvcp::kSelMax / c.S;
      char* base = reinterpret_cast<char*>(dws);
      const dvcp::FpsPartArgs qa{dws, reinterpret_cast<uint32_t*>(base + w.slot_bytes),
                                 reinterpret_cast<uint32_t*>(base + w.slot_bytes + w.flag_bytes),
                                 reinterpret_cast<int32_t*>(base + w.total - 8), c.S, B, N, dvcp::kFpsSpinCap,
                                 argc > 5 ? atoi(argv[5]) : 0,
                                 tickets ? reinterpret_cast<uint32_t*>(base + w.slot_bytes) + B : nullptr};
      (void)capw;
      CK(hipMemset(dpp, 0, pprof_words * 8));
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(dws, 0xFF, w.slot_bytes + w.flag_bytes));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(c.fn, dim3(tickets ? B * c.S : (B + 7) / 8 * 8 * c.S), dim3(c.threads), 0, 0, view, N, npoint,
                           ds, dout, dox, qa,
                           dpp);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      CK(hipMemcpy(got.data(), dout, got.size() * 8, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int b = 0; b < ncheck; ++b)
        for (int s = 0; s < npoint; ++s) bad += got[static_cast<size_t>(b) * npoint + s] != want[b][s];
      printf("%-28s B %3d N %6d npoint %6d  %8.3f ms  %6.3f us/step  mismatches %d\n", c.name, B, N, npoint, best,
             1e3f * best / npoint, bad);
      if (c.timing) {
        std::vector<unsigned long long> pr(pprof_words);
        CK(hipMemcpy(pr.data(), dpp, pr.size() * 8, hipMemcpyDeviceToHost));
        const int W = c.threads / 64;
        printf("   cloud 0: rounds %llu  scans %llu  fallbacks %llu  centres/round %.1f\n", pr[0], pr[1], pr[2],
               pr[0] ? double(npoint - 1) / pr[0] : 0.0);
        for (int part = 0; part < c.S; ++part)
          for (int wv = 0; wv < W; wv += (W > 4 ? W / 4 : 1)) {
            const unsigned long long* q = &pr[(static_cast<size_t>(part) * W + wv) * dvcp::kFpsProf];
            const double r = q[0] ? double(q[0]) : 1.0;
            printf("   part %d wave %2d clk/round: scan %.0f  decide+list %.0f  exchange %.0f  rank %.0f  prefix %.0f  "
                   "update %.0f\n", part, wv, q[3] / r, q[4] / r, q[12] / r, q[5] / r, q[6] / r, q[7] / r);
          }
      }
    }
    return 0;
  }
  for (const auto& c : cfgs) {
    if (N > c.threads * c.ppt) continue;
    CK(hipMemset(dprof, 0, prof_words * 8));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(c.fn, dim3(B), dim3(c.threads), 0, 0, view, N, npoint, ds, dout, dox, dprof);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    CK(hipMemcpy(got.data(), dout, got.size() * 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int b = 0; b < ncheck; ++b)
      for (int s = 0; s < npoint; ++s) bad += got[static_cast<size_t>(b) * npoint + s] != want[b][s];
    printf("%-28s B %3d N %6d npoint %6d  %8.3f ms  %6.3f us/step  mismatches %d\n", c.name, B, N, npoint, best,
           1e3f * best / npoint, bad);
    if (c.timing && c.sel) {
      std::vector<unsigned long long> pr(prof_words);
      CK(hipMemcpy(pr.data(), dprof, pr.size() * 8, hipMemcpyDeviceToHost));
      printf("   cloud 0: rounds %llu  scans %llu  fallbacks %llu  centres/round %.1f  rescans: none-above %llu "
             "over-cap %llu under-min %llu crowded %llu\n", pr[0], pr[1], pr[2],
             pr[0] ? double(npoint - 1) / pr[0] : 0.0, pr[8], pr[9], pr[10], pr[11]);
      for (int w = 0; w < c.threads / 64; ++w) {
        const unsigned long long* q = &pr[static_cast<size_t>(w) * dvcp::kFpsProf];
        const double r = q[0] ? double(q[0]) : 1.0;
        printf("   wave %d clk/round: scan %.0f  decide+list %.0f  rank %.0f  prefix %.0f  update %.0f\n", w,
               q[3] / r, q[4] / r, q[5] / r, q[6] / r, q[7] / r);
      }
    } else if (c.timing) {
      const int W = c.threads / 64;
      std::vector<unsigned long long> pr(prof_words);
      CK(hipMemcpy(pr.data(), dprof, pr.size() * 8, hipMemcpyDeviceToHost));
      for (int w = 0; w < W; ++w) {
        const unsigned long long* o = &pr[static_cast<size_t>(w) * dvcp::kFpsProf];  // cloud 0
        printf("   wave %2d simd %llu slot %2llu pts %5llu: update %7.1f  argmax+publish %6.1f  barrier %7.1f  "
               "reduce %6.1f clk/step  active %5.1f%%\n",
               w, (o[5] >> 4) & 3, o[5] & 15, o[6], double(o[0]) / npoint, double(o[1]) / npoint,
               double(o[2]) / npoint, double(o[3]) / npoint, 100.0 * o[4] / npoint);
      }
    }
  }
  return 0;
}
