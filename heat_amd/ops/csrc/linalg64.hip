// fp64 kernels of the CholeskyQR2 factor step: blocked Cholesky G = R^T R and
// the explicit triangular inverse R^-1 of the n x n Gram matrix (n = 4096 on the north-star
// shape), built from three small kernels and one fp64 matrix-core GEMM - the library potrf /
// trsm / trtri path (rocSOLVER, rocBLAS Cijk DGEMMs) is not used.
//
//   * gemm64: C = beta C + alpha op(A) op(B) on v_mfma_f64_16x16x4_f64, 64 x 64 tiles, 4 waves of
//     32 x 32, BK = 16 staged through LDS; strided operands (row- or k-major each), a batch
//     dimension (blockIdx.z) with element strides, and an "upper tiles only" mode for the
//     symmetric trailing update;
//   * chol_diag: upper Cholesky of one nb x nb (nb <= 64) diagonal block in LDS by one workgroup
//     (pivot <= 0 or non-finite sets *info = column + 1);
//   * chol_panel: R12 = R11^-T G12 - each thread owns one column of the panel and runs the
//     forward substitution with R11 in LDS;
//   * trtri_diag: inverse of every 64 x 64 upper diagonal block (one workgroup per block; thread
//     j owns column j of the inverse).
// Numerics: every product and sum in fp64.
#include "common.h"

namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));

constexpr int G64_T = 64, G64_BK = 16;

// AK: A element (m, k) at A[k lda + m] (else A[m lda + k]); BK_: B element (k, n) at B[k ldb + n]
// (else B[n ldb + k]). UPPER: only tiles with (tile col >= tile row) are computed (and stored).
template <bool AK, bool BK_, bool UPPER>
__global__ __launch_bounds__(256) void gemm64(const double* __restrict__ A, const double* __restrict__ B,
                                              double* __restrict__ C, int64_t M, int64_t N, int64_t K, int64_t lda,
                                              int64_t ldb, int64_t ldc, int64_t sA, int64_t sB, int64_t sC,
                                              double alpha, double beta) {
  __shared__ double As[G64_BK][G64_T + 1];
  __shared__ double Bs[G64_BK][G64_T + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.y * G64_T, n0 = (int64_t)blockIdx.x * G64_T;
  if (UPPER && n0 + G64_T <= m0) return;
  A += (int64_t)blockIdx.z * sA;
  B += (int64_t)blockIdx.z * sB;
  C += (int64_t)blockIdx.z * sC;
  const int wm = wave >> 1, wn = wave & 1;
  doublex4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (doublex4)(0.0);
  for (int64_t k0 = 0; k0 < K; k0 += G64_BK) {
    // 16 x 64 elements per operand, 4 per thread
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      int kk, mm;
      if (AK) { kk = e >> 6; mm = e & 63; } else { mm = e >> 4; kk = e & 15; }
      const int64_t gk = k0 + kk, gm = m0 + mm;
      As[kk][mm] = (gk < K && gm < M) ? A[AK ? gk * lda + gm : gm * lda + gk] : 0.0;
      int kb, nn;
      if (BK_) { kb = e >> 6; nn = e & 63; } else { nn = e >> 4; kb = e & 15; }
      const int64_t gkb = k0 + kb, gn = n0 + nn;
      Bs[kb][nn] = (gkb < K && gn < N) ? B[BK_ ? gkb * ldb + gn : gn * ldb + gkb] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < G64_BK; ks += 4) {
      const int kk = ks + (lane >> 4);
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // f64 16x16x4 C/D map: column = lane & 15, row = (lane >> 4) + 4 reg
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t gn = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t gm = m0 + wm * 32 + i * 16 + (lane >> 4) + 4 * g;
        if (gm < M && gn < N && (!UPPER || gn >= gm)) {
          double* c = C + gm * ldc + gn;
          const double v = alpha * acc[i][j][g];
          *c = beta != 0.0 ? beta * *c + v : v;
        }
      }
    }
}

// upper Cholesky of the nb x nb block at G[k0, k0] (row-major, ld), in place (the strictly lower
// part of the block is zeroed); one workgroup of 256 threads.
__global__ __launch_bounds__(256) void chol_diag(double* __restrict__ G, int64_t ld, int64_t k0, int nb,
                                                 int* __restrict__ info) {
  __shared__ double S[64][65];
  const int tid = threadIdx.x;
  for (int e = tid; e < nb * nb; e += 256) {
    const int i = e / nb, j = e % nb;
    S[i][j] = G[(k0 + i) * ld + k0 + j];
  }
  __syncthreads();
  __shared__ int bad;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int p = 0; p < nb; ++p) {
    // row p: r_pp = sqrt(s_pp), r_pj = s_pj / r_pp; then the trailing update s_ij -= r_pi r_pj
    if (tid == 0) {
      const double d = S[p][p];
      if (!(d > 0.0) || !(d <= 1.79e308)) {
        bad = 1;
        if (atomicCAS(info, 0, (int)(k0 + p + 1)) != 0) {}
        S[p][p] = 1.0;
      } else {
        S[p][p] = sqrt(d);
      }
    }
    __syncthreads();
    const double rpp = S[p][p];
    for (int j = p + 1 + tid; j < nb; j += 256) S[p][j] /= rpp;
    __syncthreads();
    const int m = nb - p - 1;
    for (int e = tid; e < m * m; e += 256) {
      const int i = p + 1 + e / m, j = p + 1 + e % m;
      if (j >= i) S[i][j] -= S[p][i] * S[p][j];
    }
    __syncthreads();
  }
  for (int e = tid; e < nb * nb; e += 256) {
    const int i = e / nb, j = e % nb;
    G[(k0 + i) * ld + k0 + j] = j >= i ? S[i][j] : 0.0;
  }
}

// R12 = R11^-T G12 for the rows [k0, k0 + nb) and columns [k0 + nb, n) of G (row-major): thread
// c owns column c of the panel; forward substitution over the nb rows with R11 from LDS.
__global__ __launch_bounds__(256) void chol_panel(double* __restrict__ G, int64_t ld, int64_t n, int64_t k0, int nb) {
  __shared__ double R[64][65];
  const int tid = threadIdx.x;
  for (int e = tid; e < nb * nb; e += 256) {
    const int i = e / nb, j = e % nb;
    R[i][j] = G[(k0 + i) * ld + k0 + j];
  }
  __syncthreads();
  const int64_t c = k0 + nb + (int64_t)blockIdx.x * 256 + tid;
  if (c >= n) return;
  double x[64];
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (i < nb) x[i] = G[(k0 + i) * ld + c];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if (i < nb) {
      double s = x[i];
#pragma unroll
      for (int p = 0; p < 64; ++p)
        if (p < i) s -= R[p][i] * x[p];
      x[i] = s / R[i][i];
    }
  }
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (i < nb) G[(k0 + i) * ld + c] = x[i];
}

// inverse of every b x b upper-triangular diagonal block (b <= 64) of R (row-major, ld) into the
// same positions of X (zero below the diagonal of each block); block q covers [q b, q b + b).
__global__ __launch_bounds__(64) void trtri_diag(const double* __restrict__ R, int64_t ld, int64_t n, int b,
                                                 double* __restrict__ X, int64_t ldx) {
  __shared__ double S[64][65];
  const int j = threadIdx.x;
  const int64_t o = (int64_t)blockIdx.x * b;
  const int nb = (int)(n - o < b ? n - o : b);
  for (int i = 0; i < nb; ++i)
    if (j < nb) S[i][j] = R[(o + i) * ld + o + j];
  __syncthreads();
  if (j >= nb) return;
  // column j of the inverse: solve R x = e_j by back substitution (x_i = 0 for i > j)
  double x[64];
#pragma unroll
  for (int i = 63; i >= 0; --i) {
    if (i < nb) {
      double s = (i == j) ? 1.0 : 0.0;
      if (i <= j) {
#pragma unroll
        for (int p = 0; p < 64; ++p)
          if (p > i && p <= j && p < nb) s -= S[i][p] * x[p];
        x[i] = s / S[i][i];
      } else {
        x[i] = 0.0;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (i < nb) X[(o + i) * ldx + o + j] = x[i];
}

template <bool AK, bool BK_, bool UP>
int gemm64_launch(const double* A, const double* B, double* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                  int64_t ldb, int64_t ldc, int64_t batch, int64_t sA, int64_t sB, int64_t sC, double alpha,
                  double beta, hipStream_t s) {
  const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64), (unsigned)batch);
  hipLaunchKernelGGL((gemm64<AK, BK_, UP>), grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc, sA, sB, sC,
                     alpha, beta);
  return ha_launch_status();
}

}  // namespace

// C = beta C + alpha op(A) op(B) in fp64 (batched: blockIdx.z with element strides sA/sB/sC).
// a_kmajor: A(m, k) at A[k lda + m]; b_kmajor: B(k, n) at B[k ldb + n] (else B[n ldb + k]).
// upper: only C(i, j) with j >= i are written.
HA_EXPORT int ha_gemm64(const double* A, const double* B, double* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                        int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int upper, int64_t batch, int64_t sA,
                        int64_t sB, int64_t sC, double alpha, double beta, void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 0) return HA_BAD_ARG;
  if (M == 0 || N == 0 || batch == 0) return HA_OK;
  if ((M + 63) / 64 > 65535 || batch > 65535) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
#define HA_G64(AK, BK, UP) return gemm64_launch<AK, BK, UP>(A, B, C, M, N, K, lda, ldb, ldc, batch, sA, sB, sC, alpha, beta, s)
  if (upper) {
    if (a_kmajor) { if (b_kmajor) HA_G64(true, true, true); HA_G64(true, false, true); }
    if (b_kmajor) HA_G64(false, true, true);
    HA_G64(false, false, true);
  }
  if (a_kmajor) { if (b_kmajor) HA_G64(true, true, false); HA_G64(true, false, false); }
  if (b_kmajor) HA_G64(false, true, false);
  HA_G64(false, false, false);
#undef HA_G64
}

// Upper Cholesky G = R^T R of the n x n symmetric fp64 matrix G (row-major, ld; the upper triangle
// is read), in place: on return the upper triangle holds R.
// Blocked right-looking with 64-wide panels: chol_diag, chol_panel, then the symmetric trailing
// update G22 -= R12^T R12 (upper tiles) on gemm64. Below the diagonal blocks G keeps its input
// (the caller takes the upper triangle). *info (device int, zeroed by the caller)
// receives 1 + the first failing column (not positive definite / non-finite).
HA_EXPORT int ha_chol_upper64(double* G, int64_t n, int64_t ld, int* info, void* stream) {
  if (n < 0 || ld < n || !info) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  for (int64_t k0 = 0; k0 < n; k0 += 64) {
    const int nb = (int)(n - k0 < 64 ? n - k0 : 64);
    hipLaunchKernelGGL(chol_diag, dim3(1), dim3(256), 0, s, G, ld, k0, nb, info);
    const int64_t k1 = k0 + nb, m = n - k1;
    if (m <= 0) break;
    hipLaunchKernelGGL(chol_panel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, G, ld, n, k0, nb);
    // G22 -= R12^T R12: A = R12^T (k-major: element (i, p) at R12[p][i]), B = R12 (k-major)
    const double* R12 = G + k0 * ld + k1;
    const int rc = gemm64_launch<true, true, true>(R12, R12, G + k1 * ld + k1, m, m, nb, ld, ld, ld, 1, 0, 0, 0,
                                                   -1.0, 1.0, s);
    if (rc != HA_OK) return rc;
  }
  return ha_launch_status();  // the strictly lower part below the diagonal blocks is left as is
}

// X = R^-1 for upper-triangular R (n x n, row-major ld) into X (ldx; zero below the diagonal):
// the 64 x 64 diagonal blocks are inverted directly, then recursive doubling: for every pair of
// inverted b x b diagonal blocks, X12 = -X11 R12 X22 (two batched gemm64 calls per level).
// W: fp64 workspace of n * ldx elements.
HA_EXPORT int ha_trtri_upper64(const double* R, int64_t n, int64_t ld, double* X, int64_t ldx, double* W,
                               void* stream) {
  if (n < 0 || ld < n || ldx < n) return HA_BAD_ARG;
  if (n == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(X, 0, (size_t)(n * ldx) * sizeof(double), s);
  hipLaunchKernelGGL(trtri_diag, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, R, ld, n, 64, X, ldx);
  for (int64_t b = 64; b < n; b *= 2) {
    // pairs p: rows/cols [2 p b, 2 p b + b) and [2 p b + b, min(2 p b + 2b, n))
    const int64_t full = n / (2 * b);  // pairs whose second block is a whole b x b
    const int64_t rem = n - full * 2 * b;
    for (int pass = 0; pass < 2; ++pass) {
      int64_t batch, o, b2;
      if (pass == 0) { batch = full; o = 0; b2 = b; }
      else { if (rem <= b) break; batch = 1; o = full * 2 * b; b2 = rem - b; }
      if (batch == 0) continue;
      const int64_t st = 2 * b * (ld + 1), stx = 2 * b * (ldx + 1), stw = 2 * b * (ldx + 1);
      // W12 = X11 R12   (b x b2)
      int rc = gemm64_launch<false, true, false>(X + o * (ldx + 1), R + o * (ld + 1) + b, W + o * (ldx + 1) + b, b,
                                                 b2, b, ldx, ld, ldx, batch, stx, st, stw, 1.0, 0.0, s);
      if (rc != HA_OK) return rc;
      // X12 = -W12 X22  (b x b2)
      rc = gemm64_launch<false, true, false>(W + o * (ldx + 1) + b, X + (o + b) * (ldx + 1), X + o * (ldx + 1) + b, b,
                                             b2, b2, ldx, ldx, ldx, batch, stw, stx, stx, -1.0, 0.0, s);
      if (rc != HA_OK) return rc;
    }
  }
  return ha_launch_status();
}
