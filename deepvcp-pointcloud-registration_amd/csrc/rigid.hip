// rigid.hip -- pose solve (deepVCP_loss.py:13-121), one workgroup per cloud pair, fp64.
//
//   get_rigid_transform (:13-44): centroids, H = (x - cx)(y - cy)^T, torch.svd(H) = U S V^T,
//     R = V U^T with NO reflection fix (Q13), t = cy + (-R) cx.  The 3x3 SVD is a one-sided
//     Jacobi iteration in fp64; R = V U^T is invariant to the SVD's sign/order freedom.
//   svd_optimization (:57-90): R1,t1 -> y1 = R1 x + t1 -> 1-NN distance (fp32, knn_cuda
//     contract) of every y_true point against y1 -> keep the int(0.8 n) smallest (ascending,
//     ties to the lower index) -> R2,t2 = Kabsch(x1, y1[inliers]) (Q12) -> y2 = R2 x1 + t2.
//   deepVCP_loss (:105-121) needs sum|y2 - y_true1| and sum(y2 - y_true1): written per pair.
#include "common.h"

namespace dvcp {

constexpr int kRgThreads = 256;
constexpr int kRgMaxN = 1024;

struct Mat3 {
  double m[3][3];
};

// One-sided Jacobi SVD of H (3x3): H V = U diag(sig), i.e. H = U diag(sig) V^T.  Returns R = V U^T
// and U, sig (the backward needs them).
__device__ void kabsch_svd(const double (&H)[3][3], double (&R)[3][3], double (&U)[3][3], double (&sig)[3]) {
  double A[3][3], V[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      A[i][j] = H[i][j];
      V[i][j] = i == j ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 40; ++sweep) {
    bool rotated = false;
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      double alpha = 0, beta = 0, gamma = 0;
      for (int i = 0; i < 3; ++i) {
        alpha += A[i][p] * A[i][p];
        beta += A[i][q] * A[i][q];
        gamma += A[i][p] * A[i][q];
      }
      if (fabs(gamma) <= 1e-300 || fabs(gamma) <= 1e-17 * sqrt(alpha * beta)) continue;
      rotated = true;
      const double zeta = (beta - alpha) / (2.0 * gamma);
      const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
      for (int i = 0; i < 3; ++i) {
        const double ap = A[i][p], aq = A[i][q];
        A[i][p] = c * ap - s * aq;
        A[i][q] = s * ap + c * aq;
        const double vp = V[i][p], vq = V[i][q];
        V[i][p] = c * vp - s * vq;
        V[i][q] = s * vp + c * vq;
      }
    }
    if (!rotated) break;
  }
  for (int j = 0; j < 3; ++j) sig[j] = sqrt(A[0][j] * A[0][j] + A[1][j] * A[1][j] + A[2][j] * A[2][j]);
  const double smax = fmax(sig[0], fmax(sig[1], sig[2]));
  int bad = -1;
  for (int j = 0; j < 3; ++j) {
    if (sig[j] > 1e-14 * smax && sig[j] > 0) {
      for (int i = 0; i < 3; ++i) U[i][j] = A[i][j] / sig[j];
    } else {
      bad = j;
    }
  }
  if (bad >= 0) {  // rank-deficient H: complete U with the cross product of the other columns
    const int a = (bad + 1) % 3, b = (bad + 2) % 3;
    U[0][bad] = U[1][a] * U[2][b] - U[2][a] * U[1][b];
    U[1][bad] = U[2][a] * U[0][b] - U[0][a] * U[2][b];
    U[2][bad] = U[0][a] * U[1][b] - U[1][a] * U[0][b];
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = V[i][0] * U[j][0] + V[i][1] * U[j][1] + V[i][2] * U[j][2];
}

__device__ void kabsch_rotation(const double (&H)[3][3], double (&R)[3][3]) {
  double U[3][3], sig[3];
  kabsch_svd(H, R, U, sig);
}

// Kabsch on the columns listed in sel[0..m) (or 0..m-1 when sel == nullptr) of x, y (3 x n
// in LDS).  Block-wide; every thread returns R, t.
__device__ void block_kabsch(const double* x, const double* y, int n, const int* sel, int m, double (&R)[3][3],
                             double (&t)[3], double* scratch, double* shared_rt) {
  const int tid = threadIdx.x;
  double c[6];
  for (int a = 0; a < 6; ++a) c[a] = 0;
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    for (int a = 0; a < 3; ++a) {
      c[a] += x[a * n + j];
      c[3 + a] += y[a * n + j];
    }
  }
  double cen[6];
  for (int a = 0; a < 6; ++a) cen[a] = block_sum(c[a], scratch) / static_cast<double>(m);
  double h[9];
  for (int a = 0; a < 9; ++a) h[a] = 0;
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    double dx[3], dy[3];
    for (int a = 0; a < 3; ++a) {
      dx[a] = x[a * n + j] - cen[a];
      dy[a] = y[a * n + j] - cen[3 + a];
    }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) h[a * 3 + b] = fma(dx[a], dy[b], h[a * 3 + b]);
  }
  double H[3][3];
  for (int a = 0; a < 9; ++a) H[a / 3][a % 3] = block_sum(h[a], scratch);
  if (tid == 0) {
    double Rm[3][3];
    kabsch_rotation(H, Rm);
    for (int a = 0; a < 3; ++a) {
      for (int b = 0; b < 3; ++b) shared_rt[a * 3 + b] = Rm[a][b];
      // t = cy + (-R) @ cx
      shared_rt[9 + a] = cen[3 + a] + dot3_blas<double>(-Rm[a][0], -Rm[a][1], -Rm[a][2], cen[0], cen[1], cen[2]);
    }
  }
  __syncthreads();
  for (int a = 0; a < 9; ++a) R[a / 3][a % 3] = shared_rt[a];
  for (int a = 0; a < 3; ++a) t[a] = shared_rt[9 + a];
  __syncthreads();
}

__device__ __forceinline__ double affine_row(const double (&R)[3][3], const double (&t)[3], int a, double x0, double x1,
                                             double x2) {
  return dot3_blas<double>(R[a][0], R[a][1], R[a][2], x0, x1, x2) + t[a];
}

__global__ __launch_bounds__(kRgThreads) void rigid_transform_kernel(const double* __restrict__ x,
                                                                     const double* __restrict__ y, int n,
                                                                     double* __restrict__ Rout,
                                                                     double* __restrict__ tout) {
  __shared__ double scratch[16];
  __shared__ double rt[12];
  const int b = blockIdx.x;
  double R[3][3], t[3];
  block_kabsch(x + static_cast<int64_t>(b) * 3 * n, y + static_cast<int64_t>(b) * 3 * n, n, nullptr, n, R, t, scratch,
               rt);
  if (threadIdx.x == 0) {
    for (int a = 0; a < 9; ++a) Rout[b * 9 + a] = R[a / 3][a % 3];
    for (int a = 0; a < 3; ++a) tout[b * 3 + a] = t[a];
  }
}

// The forward of svd_optimization up to the second Kabsch: x, y_pred staged in xs, ys (3 x n);
// y1 = R1 x + t1; sel[0..n_in) the inliers in rank order.  Shared by the forward and the backward.
struct SvdOptLds {
  double xs[3 * kRgMaxN], ys[3 * kRgMaxN], y1[3 * kRgMaxN];
  float nn[kRgMaxN];
  int sel[kRgMaxN];
  double scratch[16];
  double rt[12];
};

__device__ void svd_opt_front(SvdOptLds& L, const double* __restrict__ xg, const double* __restrict__ yg,
                              const double (&Rt)[3][3], const double (&tt)[3], int n, int n_in, double (&R1)[3][3],
                              double (&t1)[3], double (&R2)[3][3], double (&t2)[3]) {
  const int b = blockIdx.x, tid = threadIdx.x;
  for (int e = tid; e < 3 * n; e += kRgThreads) {
    L.xs[e] = xg[static_cast<int64_t>(b) * 3 * n + e];
    L.ys[e] = yg[static_cast<int64_t>(b) * 3 * n + e];
  }
  __syncthreads();
  const double* xs = L.xs;
  block_kabsch(xs, L.ys, n, nullptr, n, R1, t1, L.scratch, L.rt);
  for (int j = tid; j < n; j += kRgThreads)
    for (int a = 0; a < 3; ++a) L.y1[a * n + j] = affine_row(R1, t1, a, xs[j], xs[n + j], xs[2 * n + j]);
  __syncthreads();
  // 1-NN (knn_cuda: both inputs .float()) of y_true_j against y1
  for (int j = tid; j < n; j += kRgThreads) {
    const float qx = static_cast<float>(affine_row(Rt, tt, 0, xs[j], xs[n + j], xs[2 * n + j]));
    const float qy = static_cast<float>(affine_row(Rt, tt, 1, xs[j], xs[n + j], xs[2 * n + j]));
    const float qz = static_cast<float>(affine_row(Rt, tt, 2, xs[j], xs[n + j], xs[2 * n + j]));
    float best = __builtin_huge_valf();
    for (int i = 0; i < n; ++i) {
      const float dx = static_cast<float>(L.y1[i]) - qx, dy = static_cast<float>(L.y1[n + i]) - qy,
                  dz = static_cast<float>(L.y1[2 * n + i]) - qz;
      const float d2 = (dx * dx + dy * dy) + dz * dz;
      best = d2 < best ? d2 : best;
    }
    L.nn[j] = sqrt_rn(best);
  }
  __syncthreads();
  // inliers: rank by (distance, index); rank < n_in lands at position rank
  for (int j = tid; j < n; j += kRgThreads) {
    const float dj = L.nn[j];
    int rank = 0;
    for (int i = 0; i < n; ++i) rank += (L.nn[i] < dj || (L.nn[i] == dj && i < j)) ? 1 : 0;
    if (rank < n_in) L.sel[rank] = j;
  }
  __syncthreads();
  block_kabsch(xs, L.y1, n, L.sel, n_in, R2, t2, L.scratch, L.rt);
}

__global__ __launch_bounds__(kRgThreads) void svd_opt_kernel(const double* __restrict__ xg, const double* __restrict__ yg,
                                                             const double* __restrict__ Rtrue,
                                                             const double* __restrict__ ttrue, int n, int n_in,
                                                             double* __restrict__ R2out, double* __restrict__ t2out,
                                                             double* __restrict__ x1out, double* __restrict__ y2out,
                                                             double* __restrict__ partial) {
  __shared__ SvdOptLds L;
  const int b = blockIdx.x, tid = threadIdx.x;
  double Rt[3][3], tt[3];
  for (int a = 0; a < 9; ++a) Rt[a / 3][a % 3] = Rtrue[b * 9 + a];
  for (int a = 0; a < 3; ++a) tt[a] = ttrue[b * 3 + a];
  double R1[3][3], t1[3], R2[3][3], t2[3];
  svd_opt_front(L, xg, yg, Rt, tt, n, n_in, R1, t1, R2, t2);
  const double* xs = L.xs;
  const int* sel = L.sel;
  double* scratch = L.scratch;
  double sabs = 0, sdif = 0;
  for (int k = tid; k < n_in; k += kRgThreads) {
    const int j = sel[k];
    for (int a = 0; a < 3; ++a) {
      const double v2 = affine_row(R2, t2, a, xs[j], xs[n + j], xs[2 * n + j]);
      const double vt = affine_row(Rt, tt, a, xs[j], xs[n + j], xs[2 * n + j]);
      if (x1out) x1out[(static_cast<int64_t>(b) * 3 + a) * n_in + k] = xs[a * n + j];
      if (y2out) y2out[(static_cast<int64_t>(b) * 3 + a) * n_in + k] = v2;
      sabs += fabs(v2 - vt);
      sdif += v2 - vt;
    }
  }
  sabs = block_sum(sabs, scratch);
  sdif = block_sum(sdif, scratch);
  if (tid == 0) {
    for (int a = 0; a < 9; ++a) R2out[b * 9 + a] = R2[a / 3][a % 3];
    for (int a = 0; a < 3; ++a) t2out[b * 3 + a] = t2[a];
    if (partial) {
      partial[b * 2] = sabs;
      partial[b * 2 + 1] = sdif;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Backward of deepVCP_loss (deepVCP_loss.py:57-121) with respect to y_pred, for loss.backward()
// in train.py:121.  The gradient follows the reference's autograd graph: loss <- y2 = R2 x1 + t2
// <- Kabsch(x1, y1[inliers]) <- y1 = R1 x + t1 <- Kabsch(x, y_pred).  The 1-NN distances and the
// top-k inlier choice carry no gradient (knn_cuda runs under no_grad; topk indices).
//
// Kabsch backward: R = V U^T is the orthogonal polar factor of H^T = R P, P = U diag(s) U^T.  For
// an incoming gR, with M = skew(R^T gR) and Y the solution of P Y + Y P = M (in U's basis:
// Y~_ij = M~_ij / (s_i + s_j)), dL/dH = -2 Y R^T.  This is the derivative torch.svd's backward
// gives for R = V U^T when the singular values are distinct, and it stays finite when they repeat.
// t = cy - R cx adds gR -= gt cx^T and d/dcy = gt.

// Adds (or writes, when `write`) dL/dy for the selected columns of y.  Block-wide.
__device__ void block_kabsch_bwd(const double* x, const double* y, int n, const int* sel, int m, const double (&gR)[3][3],
                                 const double (&gt)[3], double* gy, bool write, double* scratch, double* shared) {
  const int tid = threadIdx.x;
  double c[6];
  for (int a = 0; a < 6; ++a) c[a] = 0;
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    for (int a = 0; a < 3; ++a) {
      c[a] += x[a * n + j];
      c[3 + a] += y[a * n + j];
    }
  }
  double cen[6];
  for (int a = 0; a < 6; ++a) cen[a] = block_sum(c[a], scratch) / static_cast<double>(m);
  double h[9], sdx[3] = {0, 0, 0};
  for (int a = 0; a < 9; ++a) h[a] = 0;
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    double dx[3], dy[3];
    for (int a = 0; a < 3; ++a) {
      dx[a] = x[a * n + j] - cen[a];
      dy[a] = y[a * n + j] - cen[3 + a];
      sdx[a] += dx[a];
    }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) h[a * 3 + b] = fma(dx[a], dy[b], h[a * 3 + b]);
  }
  double H[3][3];
  for (int a = 0; a < 9; ++a) H[a / 3][a % 3] = block_sum(h[a], scratch);
  for (int a = 0; a < 3; ++a) sdx[a] = block_sum(sdx[a], scratch);
  if (tid == 0) {
    double R[3][3], U[3][3], s[3], G[3][3], M[3][3], Mt[3][3], Y[3][3], Q[3][3];
    kabsch_svd(H, R, U, s);
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) G[a][b] = gR[a][b] - gt[a] * cen[b];
    // M = (R^T G - G^T R) / 2
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double p = 0, q = 0;
        for (int k = 0; k < 3; ++k) {
          p += R[k][a] * G[k][b];
          q += G[k][a] * R[k][b];
        }
        M[a][b] = 0.5 * (p - q);
      }
    // Mt = U^T M U; Y~ = Mt / (s_i + s_j); Y = U Y~ U^T
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double v = 0;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) v += U[k][a] * M[k][l] * U[l][b];
        const double den = s[a] + s[b];
        Mt[a][b] = den > 0 ? v / den : 0.0;
      }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double v = 0;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) v += U[a][k] * Mt[k][l] * U[b][l];
        Y[a][b] = v;
      }
    // gH = -2 Y R^T
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double v = 0;
        for (int k = 0; k < 3; ++k) v += Y[a][k] * R[b][k];
        Q[a][b] = -2.0 * v;
        shared[a * 3 + b] = Q[a][b];
      }
  }
  __syncthreads();
  double gH[3][3];
  for (int a = 0; a < 9; ++a) gH[a / 3][a % 3] = shared[a];
  __syncthreads();
  // dy_k = y_k - cy: dL/dy_k = gH^T dx_k - mean_k(gH^T dx_k) + gt / m
  double mean[3];
  for (int b = 0; b < 3; ++b)
    mean[b] = (gH[0][b] * sdx[0] + gH[1][b] * sdx[1] + gH[2][b] * sdx[2]) / static_cast<double>(m);
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    double dx[3];
    for (int a = 0; a < 3; ++a) dx[a] = x[a * n + j] - cen[a];
    for (int b = 0; b < 3; ++b) {
      const double v = (gH[0][b] * dx[0] + gH[1][b] * dx[1] + gH[2][b] * dx[2]) - mean[b] + gt[b] / static_cast<double>(m);
      gy[b * n + j] = write ? v : gy[b * n + j] + v;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kRgThreads) void svd_opt_bwd_kernel(
    const double* __restrict__ xg, const double* __restrict__ yg, const double* __restrict__ Rtrue,
    const double* __restrict__ ttrue, int n, int n_in, int B, const double* __restrict__ partial,
    const double* __restrict__ gloss, double alpha, double inv_count, double* __restrict__ gy_out) {
  __shared__ SvdOptLds L;
  __shared__ double gy1[3 * kRgMaxN];
  const int b = blockIdx.x, tid = threadIdx.x;
  double Rt[3][3], tt[3];
  for (int a = 0; a < 9; ++a) Rt[a / 3][a % 3] = Rtrue[b * 9 + a];
  for (int a = 0; a < 3; ++a) tt[a] = ttrue[b * 3 + a];
  double R1[3][3], t1[3], R2[3][3], t2[3];
  svd_opt_front(L, xg, yg, Rt, tt, n, n_in, R1, t1, R2, t2);
  const double* xs = L.xs;
  // loss = alpha * mean|y_true1 - y2| + (1 - alpha) * |mean(y2 - y_true1)| over all B*3*n_in values
  double tot = 0;
  for (int bb = 0; bb < B; ++bb) tot += partial[bb * 2 + 1];
  const double sm = tot > 0 ? 1.0 : (tot < 0 ? -1.0 : 0.0);
  const double G = gloss[0] * inv_count;
  double gr[12];
  for (int a = 0; a < 12; ++a) gr[a] = 0;
  for (int k = tid; k < n_in; k += kRgThreads) {
    const int j = L.sel[k];
    for (int a = 0; a < 3; ++a) {
      const double d = affine_row(R2, t2, a, xs[j], xs[n + j], xs[2 * n + j]) -
                       affine_row(Rt, tt, a, xs[j], xs[n + j], xs[2 * n + j]);
      const double sd = d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0);
      const double g = G * (alpha * sd + (1.0 - alpha) * sm);
      for (int c = 0; c < 3; ++c) gr[a * 3 + c] += g * xs[c * n + j];
      gr[9 + a] += g;
    }
  }
  double gR[3][3], gt[3];
  for (int a = 0; a < 12; ++a) {
    const double v = block_sum(gr[a], L.scratch);
    if (a < 9) gR[a / 3][a % 3] = v; else gt[a - 9] = v;
  }
  for (int e = tid; e < 3 * n; e += kRgThreads) gy1[e] = 0;
  __syncthreads();
  block_kabsch_bwd(xs, L.y1, n, L.sel, n_in, gR, gt, gy1, false, L.scratch, L.rt);
  // y1 = R1 x + t1 over all n columns
  for (int a = 0; a < 12; ++a) gr[a] = 0;
  for (int j = tid; j < n; j += kRgThreads)
    for (int a = 0; a < 3; ++a) {
      const double g = gy1[a * n + j];
      for (int c = 0; c < 3; ++c) gr[a * 3 + c] += g * xs[c * n + j];
      gr[9 + a] += g;
    }
  for (int a = 0; a < 12; ++a) {
    const double v = block_sum(gr[a], L.scratch);
    if (a < 9) gR[a / 3][a % 3] = v; else gt[a - 9] = v;
  }
  block_kabsch_bwd(xs, L.ys, n, nullptr, n, gR, gt, gy_out + static_cast<int64_t>(b) * 3 * n, true, L.scratch, L.rt);
}

// ---------------------------------------------------------------------------------------------
// Registration error of the training harness (train.py:112-120, with C8 fixed as REF-R does):
//   rot_err   = || euler_xyz_deg(R_pred) - euler_xyz_deg(R_gt) + 1e-6 ||_2
//   trans_err = || t_pred - t_gt + 1e-6 ||_2          (nn.PairwiseDistance(p=2), eps 1e-6)
// scipy's Rotation.from_matrix(M).as_euler('xyz', degrees=True) is the extrinsic x-y-z angle
// triple (a, b, c) of M = Rz(c) Ry(b) Rx(a): a = atan2(M21, M22), b = atan2(-M20, hypot(M21, M22)),
// c = atan2(M10, M00), which agrees with scipy's quaternion route to ~1e-14 deg away from gimbal
// lock (|b| -> 90 deg, where scipy warns and zeroes the third angle).  scipy raises for a matrix
// with det <= 0 (a Kabsch reflection, Q13); the error is NaN there.
__device__ __forceinline__ bool euler_xyz_deg(const double* M, double (&e)[3]) {
  const double det = M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
                     M[2] * (M[3] * M[7] - M[4] * M[6]);
  constexpr double k = 57.29577951308232;  // 180 / pi
  e[0] = atan2(M[7], M[8]) * k;
  e[1] = atan2(-M[6], sqrt(M[7] * M[7] + M[8] * M[8])) * k;
  e[2] = atan2(M[3], M[0]) * k;
  return det > 0.0;
}

__global__ void registration_error_kernel(const double* __restrict__ Rp, const double* __restrict__ tp,
                                          const double* __restrict__ Rg, const double* __restrict__ tg, int B,
                                          int64_t rg_b, int64_t tg_b, double* __restrict__ rot,
                                          double* __restrict__ trans) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double ep[3], eg[3];
  const bool okp = euler_xyz_deg(Rp + b * 9, ep);
  const bool okg = euler_xyz_deg(Rg + b * rg_b, eg);
  const bool ok = okp && okg;
  double sr = 0.0, st = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double dr = (ep[a] - eg[a]) + 1e-6;
    const double dt = (tp[b * 3 + a] - tg[b * tg_b + a]) + 1e-6;
    sr += dr * dr;
    st += dt * dt;
  }
  rot[b] = ok ? sqrt(sr) : __builtin_nan("");
  trans[b] = sqrt(st);
}

// ---------------------------------------------------------------------------------------------
// Paper-faithful pose solve (DeepVCP paper, Sec. 3.4-3.5; SURVEY.md 8(f) rank 4 -- not reference
// parity, the reference solves unweighted with no reflection fix): weighted Kabsch with the key
// points' weights w_i, c_x = sum w x / sum w, H = sum w (x - c_x)(y - c_y)^T, and the det-sign
// correction R = V diag(1, 1, d) U^T, d = sign(det(V U^T)).  Sec. 3.5's outlier rejection: with
// inlier_ratio < 1 the int(inlier_ratio n) pairs with the smallest residual |R1 x + t1 - y| under
// the first solve (ties: the lower index) are solved again.  With the ground truth it also forms
// the paper's two loss terms per pair: sum |y_gt - y*| (the VCPs against the ground-truth
// correspondences) and sum |y_gt - (R x + t)| (the final pose applied to every key point).

struct PaperSolve {
  double R[3][3], t[3], U[3][3], sig[3], cen[6], wsum;
  int kmin;       // the singular direction the reflection fix flipped (-1: none)
};

// Block-wide weighted Kabsch over the columns sel[0..m) (all n when sel == nullptr); every thread
// returns the solve.  `rt` holds >= 32 doubles of LDS.
__device__ void weighted_kabsch(const double* x, const double* y, const double* w, int n, const int* sel, int m,
                                int reflection_fix, PaperSolve& S, double* scratch, double* rt) {
  const int tid = threadIdx.x;
  double c[7];
  for (int a = 0; a < 7; ++a) c[a] = 0;
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    const double wj = w ? w[j] : 1.0;
    for (int a = 0; a < 3; ++a) {
      c[a] = fma(wj, x[a * n + j], c[a]);
      c[3 + a] = fma(wj, y[a * n + j], c[3 + a]);
    }
    c[6] += wj;
  }
  double cen[7];
  for (int a = 0; a < 7; ++a) cen[a] = block_sum(c[a], scratch);
  const double wsum = cen[6];
  for (int a = 0; a < 6; ++a) cen[a] /= wsum;
  double h[9];
  for (int a = 0; a < 9; ++a) h[a] = 0;
  for (int k = tid; k < m; k += blockDim.x) {
    const int j = sel ? sel[k] : k;
    const double wj = w ? w[j] : 1.0;
    double dx[3], dy[3];
    for (int a = 0; a < 3; ++a) {
      dx[a] = x[a * n + j] - cen[a];
      dy[a] = y[a * n + j] - cen[3 + a];
    }
    for (int a = 0; a < 3; ++a)
      for (int bb = 0; bb < 3; ++bb) h[a * 3 + bb] = fma(wj * dx[a], dy[bb], h[a * 3 + bb]);
  }
  double H[3][3];
  for (int a = 0; a < 9; ++a) H[a / 3][a % 3] = block_sum(h[a], scratch);
  if (tid == 0) {
    double R[3][3], U[3][3], sig[3];
    kabsch_svd(H, R, U, sig);
    const double det = R[0][0] * (R[1][1] * R[2][2] - R[1][2] * R[2][1]) -
                       R[0][1] * (R[1][0] * R[2][2] - R[1][2] * R[2][0]) +
                       R[0][2] * (R[1][0] * R[2][1] - R[1][1] * R[2][0]);
    int kmin = -1;
    if (reflection_fix && det < 0) {  // V diag(1,1,-1) U^T = R - 2 v_min u_min^T, v_min = R u_min
      int k = 0;
      for (int j = 1; j < 3; ++j) k = sig[j] < sig[k] ? j : k;
      double v[3];
      for (int a = 0; a < 3; ++a) v[a] = R[a][0] * U[0][k] + R[a][1] * U[1][k] + R[a][2] * U[2][k];
      for (int a = 0; a < 3; ++a)
        for (int bb = 0; bb < 3; ++bb) R[a][bb] -= 2.0 * v[a] * U[bb][k];
      kmin = k;
    }
    for (int a = 0; a < 3; ++a) {
      for (int bb = 0; bb < 3; ++bb) {
        rt[a * 3 + bb] = R[a][bb];
        rt[12 + a * 3 + bb] = U[a][bb];
      }
      rt[9 + a] = cen[3 + a] - (R[a][0] * cen[0] + R[a][1] * cen[1] + R[a][2] * cen[2]);
      rt[21 + a] = sig[a];
    }
    rt[24] = static_cast<double>(kmin);
  }
  __syncthreads();
  for (int a = 0; a < 9; ++a) {
    S.R[a / 3][a % 3] = rt[a];
    S.U[a / 3][a % 3] = rt[12 + a];
  }
  for (int a = 0; a < 3; ++a) {
    S.t[a] = rt[9 + a];
    S.sig[a] = rt[21 + a];
  }
  S.kmin = static_cast<int>(rt[24]);
  for (int a = 0; a < 6; ++a) S.cen[a] = cen[a];
  S.wsum = wsum;
  __syncthreads();
}

// The paper's solve with rejection: the first solve, residual ranks, the kept list sel[0..m) in
// index order, the second solve.  Returns m (n when nothing is rejected, then sel is unused).
__device__ int paper_solve(const double* x, const double* y, const double* w, int n, int m_keep, int reflection_fix,
                           PaperSolve& S, double* res, int* sel, double* scratch, double* rt) {
  weighted_kabsch(x, y, w, n, nullptr, n, reflection_fix, S, scratch, rt);
  if (m_keep >= n) return n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    double d2 = 0;
    for (int a = 0; a < 3; ++a) {
      const double e = S.R[a][0] * x[j] + S.R[a][1] * x[n + j] + S.R[a][2] * x[2 * n + j] + S.t[a] - y[a * n + j];
      d2 += e * e;
    }
    res[j] = sqrt(d2);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += blockDim.x) {  // rank: strictly smaller, or equal with a lower index
    const double v = res[j];
    int r = 0;
    for (int i = 0; i < n; ++i) r += (res[i] < v || (res[i] == v && i < j)) ? 1 : 0;
    sel[kRgMaxN + j] = r < m_keep ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int k = 0;
    for (int j = 0; j < n; ++j)
      if (sel[kRgMaxN + j]) sel[k++] = j;
  }
  __syncthreads();
  weighted_kabsch(x, y, w, n, sel, m_keep, reflection_fix, S, scratch, rt);
  return m_keep;
}

__global__ __launch_bounds__(kRgThreads) void paper_pose_kernel(const double* __restrict__ xg,
                                                                const double* __restrict__ yg,
                                                                const double* __restrict__ wg, int n, int reflection_fix,
                                                                int m_keep, const double* __restrict__ Rtrue,
                                                                const double* __restrict__ ttrue,
                                                                double* __restrict__ Rout, double* __restrict__ tout,
                                                                double* __restrict__ partial) {
  __shared__ double scratch[16];
  __shared__ double rt[32];
  __shared__ double res[kRgMaxN];
  __shared__ int sel[2 * kRgMaxN];
  const int b = blockIdx.x, tid = threadIdx.x;
  const double* x = xg + static_cast<int64_t>(b) * 3 * n;
  const double* y = yg + static_cast<int64_t>(b) * 3 * n;
  const double* w = wg ? wg + static_cast<int64_t>(b) * n : nullptr;
  PaperSolve S;
  paper_solve(x, y, w, n, m_keep, reflection_fix, S, res, sel, scratch, rt);
  if (tid == 0) {
    for (int a = 0; a < 9; ++a) Rout[b * 9 + a] = S.R[a / 3][a % 3];
    for (int a = 0; a < 3; ++a) tout[b * 3 + a] = S.t[a];
  }
  if (partial) {
    double Rg[3][3], tg[3];
    for (int a = 0; a < 9; ++a) Rg[a / 3][a % 3] = Rtrue[b * 9 + a];
    for (int a = 0; a < 3; ++a) tg[a] = ttrue[b * 3 + a];
    double s1 = 0, s2 = 0;
    for (int j = tid; j < n; j += kRgThreads) {
      for (int a = 0; a < 3; ++a) {
        const double ygt = Rg[a][0] * x[j] + Rg[a][1] * x[n + j] + Rg[a][2] * x[2 * n + j] + tg[a];
        const double yp = S.R[a][0] * x[j] + S.R[a][1] * x[n + j] + S.R[a][2] * x[2 * n + j] + S.t[a];
        s1 += fabs(ygt - y[a * n + j]);
        s2 += fabs(ygt - yp);
      }
    }
    s1 = block_sum(s1, scratch);
    s2 = block_sum(s2, scratch);
    if (tid == 0) {
      partial[b * 2] = s1;
      partial[b * 2 + 1] = s2;
    }
  }
}

// Backward of the paper loss  alpha / cnt sum |y_gt - y| + (1 - alpha) / cnt sum |y_gt - (R x + t)|
// in y and w.  The rejection's selection is piecewise constant, so the gradient reaches the pose
// through the second solve only.  For that solve (sums over the kept set, W = sum w):
//   g_i = c2 sign(p_i - ygt_i) (every key point), gt = sum g_i, GR = sum g_i (x_i - c_x)^T;
//   H^T = R P' with P' = U diag(s') U^T (s' = sigma with the reflection-flipped direction
//   negated) gives dL/dH = -2 Y R^T, P' Y + Y P' = skew(R^T GR), solved in U's basis as
//   Y~_ij = M~_ij / (s'_i + s'_j) (the unweighted form is dvcp_svd_optimization_backward's);
//   dL/dy_j = w_j GH^T dx_j + (w_j / W) gt,
//   dL/dw_j = dx_j^T GH dy_j + (dy_j . gt - dx_j . R^T gt) / W   (the centroids' share),
// plus c1 sign(y_j - ygt_j) from the first term on every key point.
__global__ __launch_bounds__(kRgThreads) void paper_pose_bwd_kernel(
    const double* __restrict__ xg, const double* __restrict__ yg, const double* __restrict__ wg, int n,
    int reflection_fix, int m_keep, const double* __restrict__ Rtrue, const double* __restrict__ ttrue,
    const double* __restrict__ grad_loss, double alpha, double inv_cnt, double* __restrict__ gyg,
    double* __restrict__ gwg) {
  const double c1 = alpha * grad_loss[0] * inv_cnt, c2 = (1.0 - alpha) * grad_loss[0] * inv_cnt;
  __shared__ double scratch[16];
  __shared__ double rt[32];
  __shared__ double res[kRgMaxN];
  __shared__ int sel[2 * kRgMaxN];
  const int b = blockIdx.x, tid = threadIdx.x;
  const double* x = xg + static_cast<int64_t>(b) * 3 * n;
  const double* y = yg + static_cast<int64_t>(b) * 3 * n;
  const double* w = wg ? wg + static_cast<int64_t>(b) * n : nullptr;
  double* gy = gyg + static_cast<int64_t>(b) * 3 * n;
  double* gw = gwg ? gwg + static_cast<int64_t>(b) * n : nullptr;
  PaperSolve S;
  const int m = paper_solve(x, y, w, n, m_keep, reflection_fix, S, res, sel, scratch, rt);
  double Rg[3][3], tg[3];
  for (int a = 0; a < 9; ++a) Rg[a / 3][a % 3] = Rtrue[b * 9 + a];
  for (int a = 0; a < 3; ++a) tg[a] = ttrue[b * 3 + a];
  // the first term, and g_i of the second on every key point
  double acc[12];  // gt (3), GR (9)
  for (int a = 0; a < 12; ++a) acc[a] = 0;
  for (int j = tid; j < n; j += kRgThreads) {
    double dx[3];
    for (int a = 0; a < 3; ++a) dx[a] = x[a * n + j] - S.cen[a];
    for (int a = 0; a < 3; ++a) {
      const double ygt = Rg[a][0] * x[j] + Rg[a][1] * x[n + j] + Rg[a][2] * x[2 * n + j] + tg[a];
      const double yp = S.R[a][0] * x[j] + S.R[a][1] * x[n + j] + S.R[a][2] * x[2 * n + j] + S.t[a];
      const double e1 = y[a * n + j] - ygt, e2 = yp - ygt;
      gy[a * n + j] = c1 * (e1 > 0 ? 1.0 : (e1 < 0 ? -1.0 : 0.0));
      const double g = c2 * (e2 > 0 ? 1.0 : (e2 < 0 ? -1.0 : 0.0));
      acc[a] += g;
      for (int c = 0; c < 3; ++c) acc[3 + a * 3 + c] = fma(g, dx[c], acc[3 + a * 3 + c]);
    }
    if (gw) gw[j] = 0.0;
  }
  double gt[3], GR[3][3];
  for (int a = 0; a < 3; ++a) gt[a] = block_sum(acc[a], scratch);
  for (int a = 0; a < 9; ++a) GR[a / 3][a % 3] = block_sum(acc[3 + a], scratch);
  // dL/dH = -2 Y R^T  (every thread computes the same 3x3 algebra)
  double A[3][3];  // R^T GR
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] = S.R[0][i] * GR[0][j] + S.R[1][i] * GR[1][j] + S.R[2][i] * GR[2][j];
  double Mk[3][3], Mt[3][3], Yt[3][3], Y[3][3], T[3][3], GH[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Mk[i][j] = 0.5 * (A[i][j] - A[j][i]);
  for (int i = 0; i < 3; ++i)  // U^T Mk U
    for (int j = 0; j < 3; ++j) {
      double v = 0;
      for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) v += S.U[p][i] * Mk[p][q] * S.U[q][j];
      Mt[i][j] = v;
    }
  double sp[3];
  for (int i = 0; i < 3; ++i) sp[i] = i == S.kmin ? -S.sig[i] : S.sig[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double den = sp[i] + sp[j];
      Yt[i][j] = (i == j || den == 0.0) ? 0.0 : Mt[i][j] / den;
    }
  for (int i = 0; i < 3; ++i)  // U Yt U^T
    for (int j = 0; j < 3; ++j) {
      double v = 0;
      for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) v += S.U[i][p] * Yt[p][q] * S.U[j][q];
      Y[i][j] = v;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i][j] = Y[i][0] * S.R[j][0] + Y[i][1] * S.R[j][1] + Y[i][2] * S.R[j][2];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) GH[i][j] = -2.0 * T[i][j];
  double Rtg[3];
  for (int a = 0; a < 3; ++a) Rtg[a] = S.R[0][a] * gt[0] + S.R[1][a] * gt[1] + S.R[2][a] * gt[2];
  __syncthreads();  // gy's first-term writes are read back below by the same thread only
  for (int k = tid; k < m; k += kRgThreads) {
    const int j = m < n ? sel[k] : k;
    const double wj = w ? w[j] : 1.0;
    double dx[3], dy[3];
    for (int a = 0; a < 3; ++a) {
      dx[a] = x[a * n + j] - S.cen[a];
      dy[a] = y[a * n + j] - S.cen[3 + a];
    }
    for (int a = 0; a < 3; ++a) {
      const double ghx = GH[0][a] * dx[0] + GH[1][a] * dx[1] + GH[2][a] * dx[2];  // (GH^T dx)_a
      gy[a * n + j] += wj * ghx + (wj / S.wsum) * gt[a];
    }
    if (gw) {
      double q = 0;
      for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 3; ++c) q += dx[a] * GH[a][c] * dy[c];
      const double cy = dy[0] * gt[0] + dy[1] * gt[1] + dy[2] * gt[2];
      const double cx = dx[0] * Rtg[0] + dx[1] * Rtg[1] + dx[2] * Rtg[2];
      gw[j] = q + (cy - cx) / S.wsum;
    }
  }
}

// deepVCP_loss.py:110-119 from the per-pair partial sums: alpha * sum|.| / numel +
// (1 - alpha) * |sum(.) / numel|, summed over pairs in order (one thread; B is small).
__global__ void loss_finish_kernel(const double* __restrict__ partial, int B, double denom, double alpha,
                                   double* __restrict__ loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double sabs = 0.0, sdif = 0.0;
  for (int b = 0; b < B; ++b) {
    sabs += partial[b * 2];
    sdif += partial[b * 2 + 1];
  }
  loss[0] = alpha * (sabs / denom) + (1.0 - alpha) * fabs(sdif / denom);
}

}  // namespace dvcp

extern "C" int dvcp_registration_error(const double* R_pred, const double* t_pred, const double* R_gt, int64_t rg_b,
                                       const double* t_gt, int64_t tg_b, int B, double* rot_err, double* trans_err,
                                       void* stream) {
  DVCP_REQUIRE(R_pred && t_pred && R_gt && t_gt && rot_err && trans_err, "dvcp_registration_error: null pointer");
  DVCP_REQUIRE(B >= 0 && rg_b >= 0 && tg_b >= 0, "dvcp_registration_error: bad sizes");
  if (B == 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::registration_error_kernel, dim3(dvcp::ceil_div(B, 64)), dim3(64), 0,
                     static_cast<hipStream_t>(stream), R_pred, t_pred, R_gt, t_gt, B, rg_b, tg_b, rot_err, trans_err);
  return dvcp::launch_status("dvcp_registration_error");
}

extern "C" int dvcp_rigid_transform(const double* x, const double* y, int B, int n, double* R, double* t, void* stream) {
  DVCP_REQUIRE(n > 0 && B >= 0, "dvcp_rigid_transform: n=%d B=%d", n, B);
  if (B == 0) return DVCP_OK;  // empty tensors may carry null pointers
  DVCP_REQUIRE(x && y && R && t, "dvcp_rigid_transform: null pointer");
  hipLaunchKernelGGL(dvcp::rigid_transform_kernel, dim3(B), dim3(dvcp::kRgThreads), 0, static_cast<hipStream_t>(stream), x,
                     y, n, R, t);
  return dvcp::launch_status("dvcp_rigid_transform");
}

extern "C" int dvcp_svd_optimization(const double* x, const double* y_pred, const double* R_true, const double* t_true,
                                     int B, int n, double* R2, double* t2, double* x1, double* y2, double* partial,
                                     void* stream) {
  DVCP_REQUIRE(n > 0 && n <= dvcp::kRgMaxN, "dvcp_svd_optimization: n=%d unsupported (1..1024)", n);
  const int n_in = static_cast<int>(n * 0.8);  // deepVCP_loss.py:76 int(N*0.8)
  DVCP_REQUIRE(n_in > 0, "dvcp_svd_optimization: int(0.8 n) == 0");
  if (B == 0) return DVCP_OK;  // empty tensors may carry null pointers
  DVCP_REQUIRE(x && y_pred && R_true && t_true && R2 && t2, "dvcp_svd_optimization: null pointer");
  hipLaunchKernelGGL(dvcp::svd_opt_kernel, dim3(B), dim3(dvcp::kRgThreads), 0, static_cast<hipStream_t>(stream), x,
                     y_pred, R_true, t_true, n, n_in, R2, t2, x1, y2, partial);
  return dvcp::launch_status("dvcp_svd_optimization");
}

extern "C" int dvcp_svd_optimization_backward(const double* x, const double* y_pred, const double* R_true,
                                              const double* t_true, int B, int n, const double* partial,
                                              const double* grad_loss, double alpha, double* grad_y_pred,
                                              void* stream) {
  DVCP_REQUIRE(n > 0 && n <= dvcp::kRgMaxN, "dvcp_svd_optimization_backward: n=%d unsupported (1..1024)", n);
  const int n_in = static_cast<int>(n * 0.8);
  DVCP_REQUIRE(n_in > 0, "dvcp_svd_optimization_backward: int(0.8 n) == 0");
  if (B == 0) return DVCP_OK;  // empty tensors may carry null pointers
  DVCP_REQUIRE(x && y_pred && R_true && t_true && partial && grad_loss && grad_y_pred,
               "dvcp_svd_optimization_backward: null pointer");
  const double inv_count = 1.0 / (static_cast<double>(B) * 3.0 * n_in);
  hipLaunchKernelGGL(dvcp::svd_opt_bwd_kernel, dim3(B), dim3(dvcp::kRgThreads), 0, static_cast<hipStream_t>(stream), x,
                     y_pred, R_true, t_true, n, n_in, B, partial, grad_loss, alpha, inv_count, grad_y_pred);
  return dvcp::launch_status("dvcp_svd_optimization_backward");
}

extern "C" int dvcp_paper_pose(const double* x, const double* y, const double* w, int B, int n, int reflection_fix,
                               double inlier_ratio, const double* R_true, const double* t_true, double* R, double* t,
                               double* partial, void* stream) {
  DVCP_REQUIRE(x && y && R && t, "dvcp_paper_pose: null pointer");
  DVCP_REQUIRE(!partial || (R_true && t_true), "dvcp_paper_pose: the loss terms need R_true and t_true");
  DVCP_REQUIRE(B >= 0 && B <= 65535 && n > 0, "dvcp_paper_pose: bad sizes B=%d n=%d", B, n);
  DVCP_REQUIRE(inlier_ratio > 0 && inlier_ratio <= 1, "dvcp_paper_pose: inlier_ratio %g not in (0, 1]", inlier_ratio);
  const int m_keep = static_cast<int>(inlier_ratio * n);  // the paper's 80 %: int(0.8 n), like deepVCP_loss.py:76
  DVCP_REQUIRE(m_keep >= 1 && (m_keep >= n || n <= dvcp::kRgMaxN), "dvcp_paper_pose: rejection needs 1 <= int(ratio n) and n <= %d",
               dvcp::kRgMaxN);
  if (B == 0) return DVCP_OK;
  hipLaunchKernelGGL(dvcp::paper_pose_kernel, dim3(B), dim3(dvcp::kRgThreads), 0, static_cast<hipStream_t>(stream), x,
                     y, w, n, reflection_fix, m_keep, R_true, t_true, R, t, partial);
  return dvcp::launch_status("dvcp_paper_pose");
}

extern "C" int dvcp_paper_pose_backward(const double* x, const double* y, const double* w, int B, int n,
                                        int reflection_fix, double inlier_ratio, const double* R_true,
                                        const double* t_true, double alpha, const double* grad_loss, double* grad_y,
                                        double* grad_w, void* stream) {
  DVCP_REQUIRE(x && y && R_true && t_true && grad_loss && grad_y, "dvcp_paper_pose_backward: null pointer");
  DVCP_REQUIRE(B >= 0 && B <= 65535 && n > 0, "dvcp_paper_pose_backward: bad sizes B=%d n=%d", B, n);
  DVCP_REQUIRE(inlier_ratio > 0 && inlier_ratio <= 1, "dvcp_paper_pose_backward: inlier_ratio %g", inlier_ratio);
  const int m_keep = static_cast<int>(inlier_ratio * n);
  DVCP_REQUIRE(m_keep >= 1 && (m_keep >= n || n <= dvcp::kRgMaxN), "dvcp_paper_pose_backward: bad rejection size");
  if (B == 0) return DVCP_OK;
  const double inv_cnt = 1.0 / (static_cast<double>(B) * 3.0 * n);
  hipLaunchKernelGGL(dvcp::paper_pose_bwd_kernel, dim3(B), dim3(dvcp::kRgThreads), 0, static_cast<hipStream_t>(stream),
                     x, y, w, n, reflection_fix, m_keep, R_true, t_true, grad_loss, alpha, inv_cnt, grad_y, grad_w);
  return dvcp::launch_status("dvcp_paper_pose_backward");
}

extern "C" int dvcp_deepvcp_loss(const double* x, const double* y_pred, const double* R_true, const double* t_true,
                                 int B, int n, double alpha, double* R2, double* t2, double* partial, double* loss,
                                 void* stream) {
  DVCP_REQUIRE(partial && loss, "dvcp_deepvcp_loss: null pointer");
  const int n_in = static_cast<int>(n * 0.8);
  if (int e = dvcp_svd_optimization(x, y_pred, R_true, t_true, B, n, R2, t2, nullptr, nullptr, partial, stream)) return e;
  hipLaunchKernelGGL(dvcp::loss_finish_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), partial, B,
                     static_cast<double>(B) * 3.0 * n_in, alpha, loss);
  return dvcp::launch_status("dvcp_deepvcp_loss");
}
