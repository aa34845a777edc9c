// segsum.hip -- deterministic scatter-add by sorted segments (the target-feature gradient of
// get_cat_feat_tgt.py:85's gather, dvcp_dfe_tgt_backward).
//
// Every routed entry e = q * 32 + j of the target rows carries a 32-float contribution and the
// target row (b * M + n) it belongs to (the batch-statistics SA backward uses the same for its
// feature gradient, 32 or 64 floats per grouped entry, sa_bn.hip).  Instead of ~1e8 float atomics whose order (and so whose
// rounding) changes run to run, the entry ids are stably radix-sorted by target row (rocPRIM,
// keys only as wide as the row count needs), segment bounds are marked, and one wave per target
// row sums its segment in ascending entry order: the same bits every run.
//
// Workspace (entry count E, row count Rn): keys_out | vals_out (E u32 each) | lo | hi (Rn i32
// each) | rocPRIM temporary storage; the caller's keys_in / contributions live elsewhere.
#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

namespace dvcp {

namespace {

constexpr int64_t kAlign = 256;
int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

int key_bits(uint32_t nrows) {  // the sentinel key nrows must be representable
  int b = 1;
  while (b < 32 && (static_cast<uint64_t>(1) << b) <= nrows) ++b;
  return b;
}

hipError_t sort_call(void* tmp, size_t& bytes, const uint32_t* keys_in, uint32_t* keys_out, uint32_t* vals_out,
                     int64_t E, uint32_t nrows, hipStream_t st) {
  return rocprim::radix_sort_pairs(tmp, bytes, keys_in, keys_out, rocprim::counting_iterator<uint32_t>(0u), vals_out,
                                   static_cast<size_t>(E), 0u, static_cast<unsigned>(key_bits(nrows)), st);
}

// Positions p where the sorted key changes open / close that key's segment.
__global__ __launch_bounds__(256) void seg_bounds_kernel(const uint32_t* __restrict__ keys, int64_t E, uint32_t nrows,
                                                         int* __restrict__ lo, int* __restrict__ hi) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (p >= E) return;
  const uint32_t k = keys[p];
  if (k >= nrows) return;  // sentinel: entries that route nothing
  if (p == 0 || keys[p - 1] != k) lo[k] = static_cast<int>(p);
  if (p == E - 1 || keys[p + 1] != k) hi[k] = static_cast<int>(p + 1);
}

// One wave per target row, 64 entries per chunk: one coalesced load brings the chunk's entry ids
// (lane i holds entry p + i).  NC = 32: the half-waves (channel = lane & 31) take the even and
// the odd entries, all 32 of a half's contribution loads in flight before the in-order sum, the
// halves added last; NC = 64: lane = channel, 32 entries' loads in flight at a time.  (The rows
// are scattered lines: the loads, not the adds, are the cost.)
constexpr int kSegChunk = 64;
template <int NC>
__global__ __launch_bounds__(256) void seg_sum_kernel(const int* __restrict__ lo, const int* __restrict__ hi,
                                                      const uint32_t* __restrict__ vals,
                                                      const float* __restrict__ contrib, int64_t nrows,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;  // wave-uniform
  const int p0 = lo[row], p1 = hi[row];
  float s = 0.f;
  if constexpr (NC == 32) {
    const int h = lane >> 5, c = lane & 31;
    for (int p = p0; p < p1; p += kSegChunk) {
      const int n = min(kSegChunk, p1 - p);  // wave-uniform
      const uint32_t vl = lane < n ? vals[p + lane] : 0u;
      float a[kSegChunk / 2];
#pragma unroll
      for (int e = 0; e < kSegChunk / 2; ++e) {
        const uint32_t ve = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(vl), 2 * e));
        const uint32_t vo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(vl), 2 * e + 1));
        a[e] = 2 * e + h < n ? contrib[static_cast<int64_t>(h ? vo : ve) * 32 + c] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < kSegChunk / 2; ++e)
        if (2 * e + h < n) s += a[e];
    }
    const float other = __shfl_down(s, 32, kWave);
    if (h == 0) out[row * 32 + c] = s + other;
  } else {
    static_assert(NC == 64, "32 or 64 columns");
    for (int p = p0; p < p1; p += kSegChunk) {
      const int n = min(kSegChunk, p1 - p);
      const uint32_t vl = lane < n ? vals[p + lane] : 0u;
#pragma unroll
      for (int e0 = 0; e0 < kSegChunk; e0 += 32) {
        float a[32];
#pragma unroll
        for (int e = 0; e < 32; ++e) {
          const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(vl), e0 + e));
          a[e] = e0 + e < n ? contrib[static_cast<int64_t>(v) * 64 + lane] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 32; ++e)
          if (e0 + e < n) s += a[e];
      }
    }
    out[row * 64 + lane] = s;
  }
}

}  // namespace

int64_t segment_sum_workspace_bytes(int64_t E, int64_t nrows) {
  size_t tmp = 0;
  if (sort_call(nullptr, tmp, nullptr, nullptr, nullptr, E, static_cast<uint32_t>(nrows), nullptr) != hipSuccess)
    return -1;
  return 2 * align_up(E * 4) + 2 * align_up(nrows * 4) + align_up(static_cast<int64_t>(tmp));
}

// out (nrows, ncol) = per row, the sum of contrib[e] (ncol = 32 or 64 floats) over the entries e
// with keys[e] == row, in ascending e; keys[e] >= nrows: skipped.
int segment_sum(const uint32_t* keys, const float* contrib, int64_t E, int64_t nrows, int ncol, float* out, void* ws,
                hipStream_t st) {
  if (ncol != 32 && ncol != 64) {
    set_error("segment_sum: %d columns (32 or 64)", ncol);
    return DVCP_EINVAL;
  }
  char* w = static_cast<char*>(ws);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(w);
  uint32_t* vals_out = reinterpret_cast<uint32_t*>(w + align_up(E * 4));
  int* lo = reinterpret_cast<int*>(w + 2 * align_up(E * 4));
  int* hi = reinterpret_cast<int*>(w + 2 * align_up(E * 4) + align_up(nrows * 4));
  void* tmp = w + 2 * align_up(E * 4) + 2 * align_up(nrows * 4);
  size_t tmp_bytes = 0;
  const uint32_t nr = static_cast<uint32_t>(nrows);
  if (sort_call(nullptr, tmp_bytes, keys, keys_out, vals_out, E, nr, st) != hipSuccess ||
      sort_call(tmp, tmp_bytes, keys, keys_out, vals_out, E, nr, st) != hipSuccess) {
    set_error("segment_sum: radix sort failed");
    return DVCP_EHIP;
  }
  if (hipMemsetAsync(lo, 0, 2 * align_up(nrows * 4), st) != hipSuccess) {
    set_error("segment_sum: memset failed");
    return DVCP_EHIP;
  }
  hipLaunchKernelGGL(seg_bounds_kernel, dim3(ceil_div(E, 256)), dim3(256), 0, st, keys_out, E, nr, lo, hi);
  if (ncol == 32)
    hipLaunchKernelGGL(seg_sum_kernel<32>, dim3(ceil_div(nrows, 4)), dim3(256), 0, st, lo, hi, vals_out, contrib,
                       nrows, out);
  else
    hipLaunchKernelGGL(seg_sum_kernel<64>, dim3(ceil_div(nrows, 4)), dim3(256), 0, st, lo, hi, vals_out, contrib,
                       nrows, out);
  return launch_status("segment_sum");
}

}  // namespace dvcp
