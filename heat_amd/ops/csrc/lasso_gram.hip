// Lasso by covariance updates (the Gram form of the reference's cyclic coordinate descent,
// heat/regression/lasso.py:121-175). The reference's rule
//   rho_j = mean(X_j * (y - X theta + theta_j X_j)),  theta_j = rho_j (intercept) | soft(rho_j, lam)
// only needs G = X^T X / m and b = X^T y / m:  rho_j = b_j - (G theta)_j + G_jj theta_j.
// So a fit is ONE pass over the rows (lasso_gram: the upper triangle of [X | y]^T [X | y]) plus
// sweeps over an n x n matrix (lasso_cd: one wavefront, all sweeps and the convergence test on the
// device). Distributed rows need ONE all-reduce of the (n+1)^2 Gram partial per fit instead of a
// scalar all-reduce per coordinate and sweep, and no sweep touches HBM-resident data again.
#include "common.h"

namespace {

constexpr int GRAM_BLOCK = 256;

// Upper triangle of the augmented Gram [x_i | y_i]^T [x_i | y_i] over a grid-stride set of rows:
// every thread keeps NC (NC + 1) / 2 fp32 accumulators in registers (rows of <= NC - 1 features
// fit, one row = NC values loaded once), then wave shuffles + LDS reduce them to one fp64 partial
// per workgroup. Columns: 0..n-1 = x, n = y, n+1..NC-1 = 0.
template <int NC>
__global__ __launch_bounds__(GRAM_BLOCK) void lasso_gram(const float* __restrict__ x, int64_t m, int n, int64_t ldx,
                                                         const float* __restrict__ y, double* __restrict__ partial) {
  constexpr int T = NC * (NC + 1) / 2;
  float acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.f;
  const int64_t stride = (int64_t)gridDim.x * GRAM_BLOCK;
  const bool vec4 = ((ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  for (int64_t i = (int64_t)blockIdx.x * GRAM_BLOCK + threadIdx.x; i < m; i += stride) {
    const float* row = x + i * ldx;
    float v[NC];
    if (vec4) {
#pragma unroll
      for (int c = 0; c < NC; c += 4) {
        if (c + 4 <= n) {
          const floatx4 q = *reinterpret_cast<const floatx4*>(row + c);
          v[c] = q[0];
          if (c + 1 < NC) v[c + 1] = q[1];
          if (c + 2 < NC) v[c + 2] = q[2];
          if (c + 3 < NC) v[c + 3] = q[3];
        } else {
#pragma unroll
          for (int e = c; e < c + 4 && e < NC; ++e) v[e] = e < n ? row[e] : 0.f;
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c) v[c] = c < n ? row[c] : 0.f;
    }
    const float yi = y[i];
#pragma unroll
    for (int c = 0; c < NC; ++c) v[c] = c == n ? yi : v[c];
    int t = 0;
#pragma unroll
    for (int a = 0; a < NC; ++a)
#pragma unroll
      for (int b = a; b < NC; ++b, ++t) acc[t] = fmaf(v[a], v[b], acc[t]);
  }
  __shared__ double sh[GRAM_BLOCK / 64][T];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float s = ha_wave_sum(acc[t]);
    if (lane == 0) sh[wave][t] = (double)s;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += GRAM_BLOCK) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < GRAM_BLOCK / 64; ++w) s += sh[w][t];
    partial[(int64_t)blockIdx.x * T + t] = s;
  }
}

// All sweeps of cyclic coordinate descent on (G, b) for n <= 64: G staged once in LDS, lane k keeps
// theta_k in a register. Per coordinate: one LDS row read, a 64-lane fp64 butterfly sum, two lane
// broadcasts and the reference's update; the sweep's RMS change of theta (< tol stops, like the
// host loop) is accumulated uniformly so every lane leaves the loop together.
__global__ __launch_bounds__(64) void lasso_cd_small(const double* __restrict__ G, int n, int ldg,
                                                     const double* __restrict__ b, double lam, int max_iter,
                                                     double tol, double* __restrict__ theta, int* __restrict__ n_iter) {
  __shared__ double g[64][64];
  const int lane = threadIdx.x;
  for (int j = 0; j < n; ++j) g[j][lane] = lane < n ? G[(int64_t)j * ldg + lane] : 0.0;
  double th = lane < n ? theta[lane] : 0.0;
  const double bl = lane < n ? b[lane] : 0.0;
  __syncthreads();
  int it = 0;
  while (it < max_iter) {
    ++it;
    double d2 = 0.0;
    for (int j = 0; j < n; ++j) {
      const double s = __shfl(ha_wave_sum_d(g[j][lane] * th), 0, 64);
      const double old = __shfl(th, j, 64);
      const double rho = __shfl(bl, j, 64) - s + g[j][j] * old;
      const double nw = j == 0 ? rho : (rho < -lam ? rho + lam : (rho > lam ? rho - lam : 0.0));
      d2 += (nw - old) * (nw - old);
      if (lane == j) th = nw;
    }
    if (tol >= 0.0 && sqrt(d2 / n) < tol) break;
  }
  if (lane < n) theta[lane] = th;
  if (lane == 0) *n_iter = it;
}

// Wider systems (64 < n <= 2048): theta in LDS, rows of G streamed from L2 (lane k owns k + 64 q).
__global__ __launch_bounds__(64) void lasso_cd(const double* __restrict__ G, int n, int ldg,
                                               const double* __restrict__ b, double lam, int max_iter, double tol,
                                               double* __restrict__ theta, int* __restrict__ n_iter) {
  __shared__ double th[2048];
  const int lane = threadIdx.x;
  for (int k = lane; k < n; k += 64) th[k] = theta[k];
  __syncthreads();
  int it = 0;
  while (it < max_iter) {
    ++it;
    double d2 = 0.0;
    for (int j = 0; j < n; ++j) {
      const double* gj = G + (int64_t)j * ldg;
      double s = 0.0;
      for (int k = lane; k < n; k += 64) s = fma(gj[k], th[k], s);
      s = __shfl(ha_wave_sum_d(s), 0, 64);
      const double old = th[j];
      const double rho = b[j] - s + gj[j] * old;
      const double nw = j == 0 ? rho : (rho < -lam ? rho + lam : (rho > lam ? rho - lam : 0.0));
      d2 += (nw - old) * (nw - old);
      __syncthreads();  // every lane has read th[j] before it changes (one wave: a no-op barrier)
      if (lane == 0) th[j] = nw;
      __syncthreads();
    }
    if (tol >= 0.0 && sqrt(d2 / n) < tol) break;
  }
  for (int k = lane; k < n; k += 64) theta[k] = th[k];
  if (lane == 0) *n_iter = it;
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
HA_EXPORT int ha_lasso_gram_max_cols() { return 24; }

// Workgroups used for m rows (the partial buffer holds blocks * T doubles, T = NC (NC + 1) / 2 with
// NC = n + 1).
HA_EXPORT int ha_lasso_gram_blocks(int64_t m, int ncu) {
  const int64_t want = (m + GRAM_BLOCK - 1) / GRAM_BLOCK;
  const int64_t cap = 2 * (int64_t)(ncu > 0 ? ncu : 256);
  return (int)(want < 1 ? 1 : want < cap ? want : cap);
}

HA_EXPORT int ha_lasso_gram(const float* x, int64_t m, int n, int64_t ldx, const float* y, double* partial, int blocks,
                            void* stream) {
  const int nc = n + 1;
  if (n < 1 || nc > 24 || m < 1 || blocks < 1) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
#define HA_G(NC)                                                                                       \
  case NC:                                                                                             \
    hipLaunchKernelGGL(lasso_gram<NC>, dim3(blocks), dim3(GRAM_BLOCK), 0, s, x, m, n, ldx, y, partial); \
    break;
  switch (nc) {
    HA_G(2) HA_G(3) HA_G(4) HA_G(5) HA_G(6) HA_G(7) HA_G(8) HA_G(9) HA_G(10) HA_G(11) HA_G(12) HA_G(13)
    HA_G(14) HA_G(15) HA_G(16) HA_G(17) HA_G(18) HA_G(19) HA_G(20) HA_G(21) HA_G(22) HA_G(23) HA_G(24)
    default: return HA_UNSUPPORTED;
  }
#undef HA_G
  return ha_launch_status();
}

HA_EXPORT int ha_lasso_cd(const double* G, int n, int ldg, const double* b, double lam, int max_iter, double tol,
                          double* theta, int* n_iter, void* stream) {
  if (n < 1 || n > 2048 || ldg < n || max_iter < 0) return HA_BAD_ARG;
  if (n <= 64)
    hipLaunchKernelGGL(lasso_cd_small, dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol,
                       theta, n_iter);
  else
    hipLaunchKernelGGL(lasso_cd, dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol, theta,
                       n_iter);
  return ha_launch_status();
}
