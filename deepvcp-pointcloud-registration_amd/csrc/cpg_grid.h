// cpg_grid.h -- index math of the CPG candidate grid (G^3 voxels, G <= 11), shared by the
// forward (cpg.hip) and the backward (cpg_bwd.hip).
#pragma once
#include "common.h"

namespace dvcp {

// x / d for 0 <= x < 2^16 and 1 <= d <= 2^11 as one mul_hi: m = ceil(2^32 / d) overestimates
// 1/d by less than 2^-32, so x*m/2^32 exceeds x/d by less than 2^-16, while the fractional part
// of x/d is at most 1 - 1/d <= 1 - 2^-11: the floor is exact.  (Index math of an 11^3 grid: the
// generic 32-bit division costs ~25 VALU instructions and dominated this kernel's VALU count.)
struct FastDiv {
  uint32_t m, d;
  __device__ __forceinline__ explicit FastDiv(uint32_t dd)
      : m(static_cast<uint32_t>((0x100000000ull + dd - 1) / dd)), d(dd) {}
  __device__ __forceinline__ uint32_t div(uint32_t x) const { return __umulhi(x, m); }
  __device__ __forceinline__ uint32_t mod(uint32_t x) const { return x - div(x) * d; }
};

// haloed cell of voxel g = (gz*G + gy)*G + gx in the (G+2)^3 volume
__device__ __forceinline__ int cpg_halo(int g, const FastDiv& dG, const FastDiv& dGG, int PG, int PGG) {
  const uint32_t z = dGG.div(g), r = g - z * dGG.d;
  const uint32_t y = dG.div(r), x = r - y * dG.d;
  return static_cast<int>((z + 1) * PGG + (y + 1) * PG + (x + 1));
}

}  // namespace dvcp
