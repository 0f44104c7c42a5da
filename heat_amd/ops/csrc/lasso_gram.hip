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
#define HA_GRAM_DEFAULT_UNROLL 1  // measured 1e7 x 16: U=1 0.285 ms, U=2 0.297, U=4 0.408 (2 blocks per CU)

// Upper triangle of the augmented Gram [x_i | y_i]^T [x_i | y_i] over a grid-stride set of rows:
// every thread keeps NC (NC + 1) / 2 fp32 accumulators in registers (rows of <= NC - 1 features
// fit, one row = NC values loaded once), then wave shuffles + LDS reduce them to one fp64 partial
// per workgroup. Columns: 0..n-1 = x, n = y, n+1..NC-1 = 0.
// Loads one row (n features, then y, zero-padded to NC) into v; rows >= m load zeros, which add
// nothing to any product.
template <int NC>
__device__ __forceinline__ void gram_load_row(const float* __restrict__ x, int64_t m, int n, int64_t ldx,
                                              const float* __restrict__ y, bool vec4, int64_t i, float (&v)[NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) v[c] = 0.f;
  if (i >= m) return;
  const float* row = x + i * ldx;
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
}

// Upper triangle of the augmented Gram [x_i | y_i]^T [x_i | y_i] over a grid-stride set of rows:
// every thread keeps NC (NC + 1) / 2 fp32 accumulators in registers, then wave shuffles + LDS
// reduce them to one fp64 partial per workgroup. Columns: 0..n-1 = x, n = y, n+1..NC-1 = 0.
// The accumulators cap occupancy at 1-2 waves per SIMD, so each thread issues the loads of U rows
// before the FMAs of any of them: U rows of HBM latency in flight per thread instead of one.
template <int NC, int U>
__global__ __launch_bounds__(GRAM_BLOCK) void lasso_gram(const float* __restrict__ x, int64_t m, int n, int64_t ldx,
                                                         const float* __restrict__ y, double* __restrict__ partial) {
  constexpr int T = NC * (NC + 1) / 2;
  float acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.f;
  const int64_t stride = (int64_t)gridDim.x * GRAM_BLOCK;
  const bool vec4 = ((ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  for (int64_t i = (int64_t)blockIdx.x * GRAM_BLOCK + threadIdx.x; i < m; i += U * stride) {
    float v[U][NC];
#pragma unroll
    for (int u = 0; u < U; ++u) gram_load_row<NC>(x, m, n, ldx, y, vec4, i + u * stride, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int t = 0;
#pragma unroll
      for (int a = 0; a < NC; ++a)
#pragma unroll
        for (int b = a; b < NC; ++b, ++t) acc[t] = fmaf(v[u][a], v[u][b], acc[t]);
    }
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

__device__ __forceinline__ double ha_readlane_d(double v, int lane) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// All sweeps of cyclic coordinate descent on (G, b) for n <= 64 in one wavefront. Lane k keeps
// theta_k and c_k = (G theta)_k in registers and G (symmetric) sits in LDS, so a coordinate is
//   rho = b_j - c_j + G_jj theta_j  (three lane reads),  theta_j <- update,
//   c_k += G_kj (theta_j' - theta_j) on every lane (one LDS row read that does not depend on the
//   previous coordinate) -- no cross-lane reduction on the dependency chain. The sweep's RMS change
// of theta (< tol stops, like the host loop) is wave-uniform, so all lanes leave together.
__global__ __launch_bounds__(64) void lasso_cd_small(const double* __restrict__ G, int n, int ldg,
                                                     const double* __restrict__ b, double lam, int max_iter,
                                                     double tol, double* __restrict__ theta, int* __restrict__ n_iter) {
  __shared__ double g[64][64];
  const int lane = threadIdx.x;
  for (int j = 0; j < n; ++j) g[j][lane] = lane < n ? G[(int64_t)j * ldg + lane] : 0.0;
  double th = lane < n ? theta[lane] : 0.0;
  const double bl = lane < n ? b[lane] : 0.0;
  __syncthreads();
  const double dl = g[lane][lane];
  double c = 0.0;                                   // (G theta)_lane for the start values
  for (int j = 0; j < n; ++j) c = fma(g[j][lane], ha_readlane_d(th, j), c);
  int it = 0;
  while (it < max_iter) {
    ++it;
    double d2 = 0.0;
    for (int j = 0; j < n; ++j) {
      const double old = ha_readlane_d(th, j);
      const double rho = ha_readlane_d(bl, j) - ha_readlane_d(c, j) + ha_readlane_d(dl, j) * old;
      const double nw = j == 0 ? rho : (rho < -lam ? rho + lam : (rho > lam ? rho - lam : 0.0));
      const double delta = nw - old;
      d2 = fma(delta, delta, d2);
      c = fma(g[j][lane], delta, c);  // unconditional: a uniform branch costs more than the FMA
      if (lane == j) th = nw;
    }
    if (tol >= 0.0 && sqrt(d2 / n) < tol) break;
  }
  if (lane < n) theta[lane] = th;
  if (lane == 0) *n_iter = it;
}

// Wider systems (64 < n <= 2048), same incremental form: c = G theta, theta, b and diag(G) live in
// LDS (lane k owns k + 64 q), so the per-coordinate dependency chain (c_j, b_j, G_jj, theta_j ->
// update -> c) touches LDS only. Rows of G (n doubles each; L2 / MALL resident, ~1 us away) stream
// through a register ring P rows deep: the row for coordinate t + P is requested when coordinate t
// is done with its slot, so a fetch has P coordinate chains to land (fetching only one row ahead
// measured ~1 us per coordinate: the wait for the row sat on the chain). Coordinates run over a
// padded count np = P * ceil(n / P); padded slots fetch zeros and skip their update.
// NQ = 64-lane column groups (n <= 64 NQ); P * NQ <= 64 keeps the ring within 128 VGPRs.
template <int NQ, int P>
__global__ __launch_bounds__(64) void lasso_cd(const double* __restrict__ G, int n, int ldg,
                                               const double* __restrict__ b, double lam, int max_iter, double tol,
                                               double* __restrict__ theta, int* __restrict__ n_iter) {
  __shared__ double th[64 * NQ], c[64 * NQ], bs[64 * NQ], dg[64 * NQ];
  const int lane = threadIdx.x;
  for (int k = lane; k < n; k += 64) {
    th[k] = theta[k];
    bs[k] = b[k];
    dg[k] = G[(int64_t)k * ldg + k];
  }
  __syncthreads();
  for (int k = lane; k < n; k += 64) {          // c = G theta for the start values (G symmetric)
    double s = 0.0;
    for (int j = 0; j < n; ++j) s = fma(G[(int64_t)j * ldg + k], th[j], s);
    c[k] = s;
  }
  __syncthreads();
  const int np = (n + P - 1) / P * P;
  double ring[P][NQ];
  auto fetch = [&](int j, double (&r)[NQ]) {
    const double* gj = G + (int64_t)(j < n ? j : 0) * ldg;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int k = lane + 64 * q;
      r[q] = (j < n && k < n) ? gj[k] : 0.0;
    }
  };
#pragma unroll
  for (int s = 0; s < P; ++s) fetch(s, ring[s]);
  int it = 0;
  while (it < max_iter) {
    ++it;
    double d2 = 0.0;
    for (int j0 = 0; j0 < np; j0 += P) {
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const int j = j0 + s;
        if (j < n) {                              // uniform
          const double old = th[j];
          const double rho = bs[j] - c[j] + dg[j] * old;
          const double nw = j == 0 ? rho : (rho < -lam ? rho + lam : (rho > lam ? rho - lam : 0.0));
          const double delta = nw - old;
          d2 = fma(delta, delta, d2);
          if (delta != 0.0) {                     // uniform: skipped for coordinates that stay 0
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
              const int k = lane + 64 * q;
              if (k < n) c[k] = fma(ring[s][q], delta, c[k]);
            }
            if (lane == 0) th[j] = nw;
          }
          __syncthreads();                        // one wave: orders the LDS writes (a no-op barrier)
        }
        const int jn = j + P < np ? j + P : j + P - np;   // the slot's next row (wraps into the next sweep)
        fetch(jn, ring[s]);
      }
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

// unroll = rows whose loads each thread issues before their FMAs (1, 2 or 4; 0 = default).
HA_EXPORT int ha_lasso_gram(const float* x, int64_t m, int n, int64_t ldx, const float* y, double* partial, int blocks,
                            int unroll, void* stream) {
  const int nc = n + 1;
  if (n < 1 || nc > 24 || m < 1 || blocks < 1) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (unroll <= 0) unroll = HA_GRAM_DEFAULT_UNROLL;
#define HA_G(NC)                                                                                                  \
  case NC:                                                                                                        \
    if (unroll >= 4)                                                                                              \
      hipLaunchKernelGGL((lasso_gram<NC, 4>), dim3(blocks), dim3(GRAM_BLOCK), 0, s, x, m, n, ldx, y, partial);    \
    else if (unroll == 2)                                                                                         \
      hipLaunchKernelGGL((lasso_gram<NC, 2>), dim3(blocks), dim3(GRAM_BLOCK), 0, s, x, m, n, ldx, y, partial);    \
    else                                                                                                          \
      hipLaunchKernelGGL((lasso_gram<NC, 1>), dim3(blocks), dim3(GRAM_BLOCK), 0, s, x, m, n, ldx, y, partial);    \
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
  else if (n <= 128)
    hipLaunchKernelGGL((lasso_cd<2, 8>), dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol,
                       theta, n_iter);
  else if (n <= 256)
    hipLaunchKernelGGL((lasso_cd<4, 8>), dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol,
                       theta, n_iter);
  else if (n <= 512)
    hipLaunchKernelGGL((lasso_cd<8, 8>), dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol,
                       theta, n_iter);
  else if (n <= 1024)
    hipLaunchKernelGGL((lasso_cd<16, 4>), dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol,
                       theta, n_iter);
  else
    hipLaunchKernelGGL((lasso_cd<32, 2>), dim3(1), dim3(64), 0, (hipStream_t)stream, G, n, ldg, b, lam, max_iter, tol,
                       theta, n_iter);
  return ha_launch_status();
}
