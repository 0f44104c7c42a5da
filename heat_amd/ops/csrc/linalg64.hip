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

#include <stdlib.h>

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
// part of the block is zeroed); one workgroup of 256 threads. (One-wave forms measured slower: the
// block in LDS 113 vs 89 us - LDS round trips on the dependency chain; a register-resident,
// fully unrolled form did not compile in 40 minutes.)
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
// c owns column c of the panel; forward substitution over the nb rows with R11 from LDS. FULL
// (nb == 64, every panel but a last partial one): no per-row guards, so x stays in 128 VGPRs -
// the guarded form put x in scratch (528 B per thread: 205 us per panel, 13 ms per factor).
template <bool FULL>
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
  if constexpr (FULL) {
#pragma unroll
    for (int i = 0; i < 64; ++i) x[i] = G[(k0 + i) * ld + c];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      double s = x[i];
#pragma unroll
      for (int p = 0; p < i; ++p) s -= R[p][i] * x[p];
      x[i] = s / R[i][i];
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) G[(k0 + i) * ld + c] = x[i];
  } else {
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

// ---------------------------------------------------------------------------------------------
// vtc64: W = V^T C with fp64 products and accumulation over a very long contraction (the row
// count of a tall matrix block: 1.25e6 on the north-star shape) - the "reduction over all rows"
// GEMM of the blocked Householder QR (W = V^T C of the aggregated 256-column block
// reflector, Y = V^T V for its T factor). V [m, nc], C [m, N], both row-major fp32 or fp64;
// fp32 elements are widened exactly, so every product is exact and the only rounding is the
// fp64 accumulation (what keeps ||Q^T Q - I|| at the 1e-7 level for an fp32 QR).
//   * 128 x 128 output tile per workgroup (4 waves of 64 x 64 = 4 x 4 v_mfma_f64_16x16x4_f64
//     accumulators), BK = 16 rows per stage, LDS double buffer in the input type with a row pitch
//     chosen so the 4 k-rows x 16 lanes of one MFMA operand read hit 64 distinct banks; the next
//     stage is prefetched into registers during the MFMAs (one barrier per stage);
//   * split-K over row chunks (blockIdx.z): each split writes its fp64 partial tile P[s] and
//     vtc64_sum adds the splits in index order - deterministic, no atomics.
constexpr int VT_T = 128, VT_BK = 16;

template <typename T> struct VtPitch;
template <> struct VtPitch<float> { static constexpr int P = VT_T + 16; };   // 16 k-rows apart: 16 banks
template <> struct VtPitch<double> { static constexpr int P = VT_T + 8; };   // 8 doubles = 16 banks

template <typename T, int VEC>
__global__ __launch_bounds__(256) void vtc64(const T* __restrict__ V, int64_t ldv, const T* __restrict__ C,
                                             int64_t ldc, int64_t m, int64_t nc, int64_t N, int64_t chunk,
                                             double* __restrict__ P) {
  constexpr int PP = VtPitch<T>::P;
  __shared__ T Vs[2][VT_BK][PP];
  __shared__ T Cs[2][VT_BK][PP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.y * VT_T, j0 = (int64_t)blockIdx.x * VT_T;
  const int64_t r0 = (int64_t)blockIdx.z * chunk;
  const int64_t r1 = r0 + chunk < m ? r0 + chunk : m;
  const int nst = r1 > r0 ? (int)((r1 - r0 + VT_BK - 1) / VT_BK) : 0;
  const int wm = wave >> 1, wn = wave & 1;
  // loader: each operand stage is 16 x 128 elements = 2048 / VEC vectors, LD per thread
  constexpr int LD = VT_BK * VT_T / VEC / 256;
  typedef T vec_t __attribute__((ext_vector_type(VEC)));
  vec_t rv[LD], rc[LD];
  auto load = [&](int t) {
#pragma unroll
    for (int q = 0; q < LD; ++q) {
      const int e = tid + 256 * q;
      const int kk = e / (VT_T / VEC), cc = (e % (VT_T / VEC)) * VEC;
      const int64_t g = r0 + (int64_t)t * VT_BK + kk;
      const bool rok = g < r1;
#pragma unroll
      for (int v = 0; v < VEC; ++v) { rv[q][v] = T(0); rc[q][v] = T(0); }
      if (VEC > 1) {
        if (rok && i0 + cc < nc) rv[q] = *(const vec_t*)(V + g * ldv + i0 + cc);
        if (rok && j0 + cc < N) rc[q] = *(const vec_t*)(C + g * ldc + j0 + cc);
      } else {
        if (rok && i0 + cc < nc) rv[q][0] = V[g * ldv + i0 + cc];
        if (rok && j0 + cc < N) rc[q][0] = C[g * ldc + j0 + cc];
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < LD; ++q) {
      const int e = tid + 256 * q;
      const int kk = e / (VT_T / VEC), cc = (e % (VT_T / VEC)) * VEC;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        Vs[buf][kk][cc + v] = rv[q][v];
        Cs[buf][kk][cc + v] = rc[q][v];
      }
    }
  };
  doublex4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (doublex4)(0.0);
  if (nst > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int t = 0; t < nst; ++t) {
    const int buf = t & 1;
    if (t + 1 < nst) load(t + 1);
#pragma unroll
    for (int ks = 0; ks < VT_BK; ks += 4) {
      const int kk = ks + (lane >> 4);
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = (double)Vs[buf][kk][wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (double)Cs[buf][kk][wn * 64 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nst) store(buf ^ 1);
    __syncthreads();
  }
  // partial tile (zeros for an empty chunk): P[z][i][j], f64 16x16x4 C/D map
  double* Pz = P + (int64_t)blockIdx.z * nc * N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gj = j0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t gi = i0 + wm * 64 + i * 16 + (lane >> 4) + 4 * g;
        if (gi < nc && gj < N) Pz[gi * N + gj] = acc[i][j][g];
      }
    }
}

// vtc64d: the fp32 form of vtc64 with the operands staged by LDS-DMA (global_load_lds, no
// register staging) into a 4-stage ring: one barrier per 16-row stage, the DMA of stage t + 3
// issued right after it, so three stages (~3 x 1.7 us of MFMA work) cover a load's latency - the
// register-staged kernel prefetched one stage ahead and ran at ~70 % of the fp64 MFMA rate.
// Stage image of one operand: 8 pieces of 1 KB (one DMA instruction each: lanes 0-31 k-row kk,
// lanes 32-63 k-row kk + 4, 4 columns per lane), pieces 1088 bytes apart, k-rows paired
// {0,4} {1,5} {2,6} {3,7} {8,12} ... so the 4 k-rows x 16 columns of one fragment read fall in
// 64 distinct banks. Rows past the chunk end are clamped in the DMA and zeroed in LDS.
constexpr int VD_NST = 4, VD_PIECE = 1088, VD_OP = 8 * VD_PIECE, VD_STAGE = 2 * VD_OP;

__device__ __forceinline__ int vd_off(int kk, int col) {
  return ((kk & 3) + 4 * (kk >> 3)) * VD_PIECE + ((kk >> 2) & 1) * 512 + col * 4;
}

template <int N>
__device__ __forceinline__ void vd_wait_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__global__ __launch_bounds__(256, 2) void vtc64d(const float* __restrict__ V, int64_t ldv, const float* __restrict__ C,
                                                 int64_t ldc, int64_t m, int64_t nc, int64_t N, int64_t chunk,
                                                 double* __restrict__ P) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[VD_NST * VD_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.y * VT_T, j0 = (int64_t)blockIdx.x * VT_T;
  const int64_t r0 = (int64_t)blockIdx.z * chunk;
  const int64_t r1 = r0 + chunk < m ? r0 + chunk : m;
  const int nst = r1 > r0 ? (int)((r1 - r0 + VT_BK - 1) / VT_BK) : 0;
  const int wm = wave >> 1, wn = wave & 1;
  // this lane's DMA sources: pieces p = 2 wave + e of each operand
  const int cl = (lane & 31) * 4;
  int kkp[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = 2 * wave + e;
    kkp[e] = (p & 3) + 8 * (p >> 2) + 4 * (lane >> 5);
  }
  const int64_t vcol = i0 + cl + 4 <= nc ? i0 + cl : nc - 4;  // columns past nc / N only feed
  const int64_t ccol = j0 + cl + 4 <= N ? j0 + cl : N - 4;     // outputs that are never stored
  auto issue = [&](int t) {
    unsigned char* dst = smem + (t % VD_NST) * VD_STAGE;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int p = 2 * wave + e;
      int64_t g = r0 + (int64_t)t * VT_BK + kkp[e];
      g = g < r1 ? g : r1 - 1;
      __builtin_amdgcn_global_load_lds(V + g * ldv + vcol, (__attribute__((address_space(3))) void*)(dst + p * VD_PIECE),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(C + g * ldc + ccol,
                                       (__attribute__((address_space(3))) void*)(dst + VD_OP + p * VD_PIECE), 16, 0, 0);
    }
  };
  doublex4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (doublex4)(0.0);
  for (int t = 0; t < VD_NST - 1 && t < nst; ++t) issue(t);
  for (int t = 0; t < nst; ++t) {
    const int ahead = nst - 1 - t;  // stages issued after t (at most 2)
    if (ahead >= 2) vd_wait_barrier<8>();
    else if (ahead == 1) vd_wait_barrier<4>();
    else vd_wait_barrier<0>();
    unsigned char* b = smem + (t % VD_NST) * VD_STAGE;
    if (r0 + (int64_t)(t + 1) * VT_BK > r1) {
      // tail stage: zero this wave's k-rows past the chunk end (its own DMA has landed)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int p = 2 * wave + e;
        if (r0 + (int64_t)t * VT_BK + kkp[e] >= r1) {
          *reinterpret_cast<floatx4*>(b + p * VD_PIECE + lane * 16) = (floatx4)(0.f);
          *reinterpret_cast<floatx4*>(b + VD_OP + p * VD_PIECE + lane * 16) = (floatx4)(0.f);
        }
      }
      vd_wait_barrier<0>();
    }
    if (t + VD_NST - 1 < nst) issue(t + VD_NST - 1);
#pragma unroll
    for (int ks = 0; ks < VT_BK; ks += 4) {
      const int kk = ks + (lane >> 4);
      double a[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = (double)*reinterpret_cast<const float*>(b + vd_off(kk, wm * 64 + i * 16 + (lane & 15)));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bv[j] = (double)*reinterpret_cast<const float*>(b + VD_OP + vd_off(kk, wn * 64 + j * 16 + (lane & 15)));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  double* Pz = P + (int64_t)blockIdx.z * nc * N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gj = j0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t gi = i0 + wm * 64 + i * 16 + (lane >> 4) + 4 * g;
        if (gi < nc && gj < N) Pz[gi * N + gj] = acc[i][j][g];
      }
    }
}

// vtc32: W = V^T C for a narrow V (nc <= 32: the 32-column panels of the Householder QR, whose
// inner updates were on the fp64 VALU kernel hh_vtc at ~0.5 TB/s). Tile 32 x 256 per workgroup
// (wave w: all 32 rows x columns 64 w .. 64 w + 63 = 2 x 4 v_mfma_f64_16x16x4_f64 blocks); the MFMA
// operands are loaded straight from global memory (lane (k = lane >> 4, c = lane & 15): V[g][16 i + c]
// and C[g][j0 + 16 j + c], rows g = r + k), 8 k-steps (32 rows) per batch so 48 loads are in flight
// per lane, two waves per SIMD. Split-K partials as vtc64.
__global__ __launch_bounds__(256, 2) void vtc32(const float* __restrict__ V, int64_t ldv, const float* __restrict__ C,
                                             int64_t ldc, int64_t m, int64_t nc, int64_t N, int64_t chunk,
                                             double* __restrict__ P) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kr = lane >> 4, cc = lane & 15;
  const int64_t j0 = (int64_t)blockIdx.x * 256 + wave * 64;
  const int64_t r0 = (int64_t)blockIdx.z * chunk;
  const int64_t r1 = r0 + chunk < m ? r0 + chunk : m;
  bool vok[2], cok[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) vok[i] = 16 * i + cc < nc;
#pragma unroll
  for (int j = 0; j < 4; ++j) cok[j] = j0 + 16 * j + cc < N;
  doublex4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (doublex4)(0.0);
  // out-of-range rows / columns: clamped addresses, the loaded value replaced by 0
  int vcol[2];
  int64_t ccol[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) vcol[i] = vok[i] ? 16 * i + cc : 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) ccol[j] = cok[j] ? j0 + 16 * j + cc : 0;
  for (int64_t r = r0; r < r1; r += 32) {
    float va[8][2], cv[8][4];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int64_t g0 = r + 4 * s + kr;
      const bool ok = g0 < r1;
      const int64_t g = ok ? g0 : r1 - 1;
      const float* vr = V + g * ldv;
      const float* cr = C + g * ldc;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float x = vr[vcol[i]];
        va[s][i] = ok && vok[i] ? x : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = cr[ccol[j]];
        cv[s][j] = ok && cok[j] ? x : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)va[s][i], (double)cv[s][j], acc[i][j], 0, 0, 0);
  }
  double* Pz = P + (int64_t)blockIdx.z * nc * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gj = j0 + 16 * j + cc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t gi = 16 * i + kr + 4 * g;
        if (gi < nc && gj < N) Pz[gi * N + gj] = acc[i][j][g];
      }
    }
}

// W[e] (+)= sum over z = 0, 1, ... < count of P[z stride + e], in z order (8 loads in flight).
__global__ __launch_bounds__(256) void vtc64_sum(const double* __restrict__ P, int64_t count, int64_t stride,
                                                 int64_t plane, double* __restrict__ W, int accumulate) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < plane; e += (int64_t)gridDim.x * 256) {
    double s = accumulate ? W[e] : 0.0;
    int64_t z = 0;
    for (; z + 8 <= count; z += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = P[(z + u) * stride + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; z < count; ++z) s += P[z * stride + e];
    W[e] = s;
  }
}

// First level of a two-level fixed-order split sum (many splits, small plane): P[q G][e] =
// sum of P[z][e] for z in [q G, q G + G), in z order - every element is read and written by one
// thread, so the group's first slot is overwritten in place.
__global__ __launch_bounds__(256) void vtc64_group_sum(double* __restrict__ P, int64_t splits, int64_t plane, int G) {
  const int64_t ngroups = (splits + G - 1) / G;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < ngroups * plane;
       idx += (int64_t)gridDim.x * 256) {
    const int64_t q = idx / plane, e = idx % plane;
    const int64_t z0 = q * G, z1 = z0 + G < splits ? z0 + G : splits;
    double s = 0.0;
    int64_t z = z0;
    for (; z + 8 <= z1; z += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = P[(z + u) * plane + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; z < z1; ++z) s += P[z * plane + e];
    P[z0 * plane + e] = s;
  }
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

// Row-chunk split count of ha_vtc64 for (m, nc, N): enough workgroups to fill the chip (>= ~1024)
// with >= 32 stages per split; the caller sizes the partial buffer as splits * nc * N doubles.
HA_EXPORT int64_t ha_vtc64_splits(int64_t m, int64_t nc, int64_t N) {
  if (m <= 0 || nc <= 0 || N <= 0) return 1;
  if (nc <= 32) {  // vtc32: 32 x 256 tiles, >= ~512 workgroups, >= 64 rows per split
    const int64_t tiles = (N + 255) / 256;
    int64_t s = (512 + tiles - 1) / tiles;
    const int64_t maxs = (m + 63) / 64;
    if (s > maxs) s = maxs;
    if (s > 65535) s = 65535;
    return s < 1 ? 1 : s;
  }
  const int64_t tiles = ((nc + VT_T - 1) / VT_T) * ((N + VT_T - 1) / VT_T);
  int64_t s = (1024 + tiles - 1) / tiles;
  const int64_t maxs = (m + 32 * VT_BK - 1) / (32 * VT_BK);
  if (s > maxs) s = maxs;
  if (s > 65535) s = 65535;
  return s < 1 ? 1 : s;
}

// W [nc, N] (row-major fp64, contiguous) = V^T C (+ W when accumulate), V [m, nc] (ldv) and
// C [m, N] (ldc) row-major, dtype 0 = fp32 / 1 = fp64; P: ha_vtc64_splits(m, nc, N) * nc * N
// doubles of scratch. Deterministic (fixed split order).
HA_EXPORT int ha_vtc64(const void* V, int64_t ldv, const void* C, int64_t ldc, int dtype, int64_t m, int64_t nc,
                       int64_t N, double* W, double* P, int accumulate, void* stream) {
  if (m < 0 || nc < 0 || N < 0 || (dtype != 0 && dtype != 1)) return HA_BAD_ARG;
  if (nc == 0 || N == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  if (m == 0) {
    if (!accumulate) hipMemsetAsync(W, 0, (size_t)(nc * N) * sizeof(double), s);
    return ha_launch_status();
  }
  if ((nc + VT_T - 1) / VT_T > 65535) return HA_UNSUPPORTED;
  const int64_t splits = ha_vtc64_splits(m, nc, N);
  const int64_t chunk = ((m + splits - 1) / splits + VT_BK - 1) / VT_BK * VT_BK;
  const dim3 grid((unsigned)((N + VT_T - 1) / VT_T), (unsigned)((nc + VT_T - 1) / VT_T), (unsigned)splits);
  if (dtype == 0 && nc <= 32) {
    const int64_t chunk32 = ((m + splits - 1) / splits + 31) / 32 * 32;
    hipLaunchKernelGGL(vtc32, dim3((unsigned)((N + 255) / 256), 1, (unsigned)splits), dim3(256), 0, s,
                       (const float*)V, ldv, (const float*)C, ldc, m, nc, N, chunk32, P);
  } else if (dtype == 0) {
    const bool v4 = nc % 4 == 0 && N % 4 == 0 && ldv % 4 == 0 && ldc % 4 == 0 && ((uintptr_t)V & 15) == 0 &&
                    ((uintptr_t)C & 15) == 0;
    static const bool v1 = getenv("HEAT_VTC64_V1") && atoi(getenv("HEAT_VTC64_V1"));  // A/B: register staging
    if (v4 && !v1)
      hipLaunchKernelGGL(vtc64d, grid, dim3(256), 0, s, (const float*)V, ldv, (const float*)C, ldc, m, nc, N, chunk,
                         P);
    else if (v4)
      hipLaunchKernelGGL((vtc64<float, 4>), grid, dim3(256), 0, s, (const float*)V, ldv, (const float*)C, ldc, m, nc,
                         N, chunk, P);
    else
      hipLaunchKernelGGL((vtc64<float, 1>), grid, dim3(256), 0, s, (const float*)V, ldv, (const float*)C, ldc, m, nc,
                         N, chunk, P);
  } else {
    const bool v2 = nc % 2 == 0 && N % 2 == 0 && ldv % 2 == 0 && ldc % 2 == 0 && ((uintptr_t)V & 15) == 0 &&
                    ((uintptr_t)C & 15) == 0;
    if (v2)
      hipLaunchKernelGGL((vtc64<double, 2>), grid, dim3(256), 0, s, (const double*)V, ldv, (const double*)C, ldc, m,
                         nc, N, chunk, P);
    else
      hipLaunchKernelGGL((vtc64<double, 1>), grid, dim3(256), 0, s, (const double*)V, ldv, (const double*)C, ldc, m,
                         nc, N, chunk, P);
  }
  const int64_t plane = nc * N;
  const int64_t g = (plane + 255) / 256;
  if (splits > 64 && g < 256) {
    // few output elements, many splits: sum groups of 32 splits in parallel first
    constexpr int G = 32;
    const int64_t ng = (splits + G - 1) / G;
    const int64_t g1 = (ng * plane + 255) / 256;
    hipLaunchKernelGGL(vtc64_group_sum, dim3((unsigned)(g1 < 8192 ? g1 : 8192)), dim3(256), 0, s, P, splits, plane, G);
    hipLaunchKernelGGL(vtc64_sum, dim3((unsigned)g), dim3(256), 0, s, P, ng, G * plane, plane, W, accumulate);
  } else {
    hipLaunchKernelGGL(vtc64_sum, dim3((unsigned)(g < 8192 ? g : 8192)), dim3(256), 0, s, P, splits, plane, plane, W,
                       accumulate);
  }
  return ha_launch_status();
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
    if (nb == 64)
      hipLaunchKernelGGL(chol_panel<true>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, G, ld, n, k0, nb);
    else
      hipLaunchKernelGGL(chol_panel<false>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, G, ld, n, k0, nb);
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

namespace {
// y[r] = sum_k M[r][k] x[k] (fp64, row-major M with leading dimension ld): one 256-thread block per
// row, a fixed-order tree reduction (deterministic). The condition estimate of CholeskyQR2 runs
// 48 of these on 4096 x 4096 factors; on gemm64 (64 x 64 tiles, one output column) each took
// 0.44 ms - 21 ms per QR - against ~30 us at HBM speed here.
__global__ __launch_bounds__(256) void gemv64_rows(const double* __restrict__ M, int64_t ld, int64_t cols,
                                                   const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double red[4];
  const int64_t r = blockIdx.x;
  const double* row = M + r * ld;
  double s = 0.0;
  for (int64_t k = threadIdx.x; k < cols; k += 256) s = fma(row[k], x[k], s);
  s = ha_wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) y[r] = (red[0] + red[1]) + (red[2] + red[3]);
}
}  // namespace

// y = M x for a row-major fp64 M [rows, cols] (leading dimension ld), x [cols], y [rows].
HA_EXPORT int ha_gemv64(const double* M, int64_t rows, int64_t cols, int64_t ld, const double* x, double* y,
                        void* stream) {
  if (rows < 0 || cols < 0 || ld < cols || !M || !x || !y) return HA_BAD_ARG;
  if (rows == 0) return HA_OK;
  if (rows > 0x7fffffffLL) return HA_UNSUPPORTED;
  hipLaunchKernelGGL(gemv64_rows, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, M, ld, cols, x, y);
  return ha_launch_status();
}
