// Blocked Householder QR building blocks (SURVEY K8 geqrf panel / K9 larfb trailing update) for
// tall row-distributed matrices: the panel is factorised column by column with ONE kernel per
// column, the trailing matrix is updated by GEMMs (compact WY: C -= V (T^T (V^T C))).
//
// Panel column j (global column k0 + j, diagonal row d = k0 + j) needs, over all rows >= d,
//   S[c] = sum_{g >= d} A[g][j] A[g][c]   (c >= j)   and   rowd[c] = A[d][c]
// - one small vector (2 NB doubles) that is summed over the row blocks of all ranks (an RCCL
// all-reduce between the column kernels when the rows are distributed; every rank's contribution
// to rowd is zero except the owner's). From it EVERY block computes the reflector redundantly:
//   alpha = rowd[j], |x| = sqrt(S[j]), beta = -sign(alpha) |x|, tau = (beta - alpha) / beta,
//   v = x / (alpha - beta) (v_d = 1), w_c = v^T A[:, c] = rowd[c] + (S[c] - alpha rowd[c]) / (alpha - beta)
// and applies A[g][c] -= tau v_g w_c to its rows g > d, stores v_g in A[g][j] and (owner of d) the
// R row (beta, rowd[c] - tau w_c) in row d. The same kernel then accumulates the S / rowd vector of
// column j + 1 from the rows it has just updated - so a panel of NB columns is NB launches, each one
// pass over the panel's rows, with fp64 accumulation of every dot product.
//
// The step also writes column j of Y = V^T V (for larft) from the same sums, so the panel needs no
// separate V^T V pass. The host factors each panel in a compact m x NB copy (row pitch NB: the 32
// passes stream contiguous rows instead of one 128-byte segment per 16 KB matrix row) - `coff` is
// the panel's first column within a row of A, k0 its global column.
//
// Layout: A row-major (lda), rows of this rank = global rows [g0, g0 + m). 8 lanes own one row (4
// consecutive panel columns each: 16- or 32-byte accesses, a row segment per 8 lanes), 32 rows per
// 256-thread block, grid-stride over the rows; block partial sums go through LDS, then a
// fixed-order two-level sum (hh_block_sum) - no float atomics, bit-reproducible.
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int HH_NB = 32;     // panel width (8 lanes x 4 columns)
constexpr int HH_COPIES = 32; // S accumulator copies: copy g = the fixed-order sum of block group g
constexpr int HH_SLEN = 2 * HH_NB;  // one copy: S[NB] | rowd[NB]

template <typename T>
struct Vec4 {
  T v[4];
};

template <typename T>
__device__ __forceinline__ Vec4<T> hh_load4(const T* p, int ncols_here) {
  Vec4<T> r;
  if (ncols_here >= 4 && ((uintptr_t)p % (4 * sizeof(T))) == 0) {
    if constexpr (sizeof(T) == 4) {
      const floatx4 q = *reinterpret_cast<const floatx4*>(p);
#pragma unroll
      for (int i = 0; i < 4; ++i) r.v[i] = q[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) r.v[i] = p[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = i < ncols_here ? p[i] : T(0);
  }
  return r;
}

template <typename T>
__device__ __forceinline__ void hh_store4(T* p, const Vec4<T>& r, int ncols_here) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < ncols_here) p[i] = r.v[i];
}

// Block-reduce the per-lane partials acc[4] (columns 4 q .. 4 q + 3, q = lane % 8) over the 32
// row groups of the block, then a FIXED-ORDER tree instead of float atomics (whose arrival order
// made the factorization differ run to run in the last bits): the block's column sums go to its
// own slot of `part` (write-through), the blocks form HH_COPIES groups of consecutive blocks, and
// the last-arriving block of each group (ticket on cnt[group], reset by it) adds its group's slots
// in a fixed order (8 strided partial sums + a pairwise tree) into accumulator copy `group` of
// out; hh_gather_s then adds the copies in a fixed order.
__device__ __forceinline__ void hh_block_sum(const double (&acc)[4], double* __restrict__ out, double* red,
                                             double* __restrict__ part, unsigned* __restrict__ cnt) {
  __shared__ bool last;
  const int tid = threadIdx.x, q = tid & 7, grp = tid >> 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) red[grp * HH_NB + 4 * q + i] = acc[i];
  __syncthreads();
  if (tid < HH_NB) {
    double s = 0.0;
    for (int g = 0; g < 32; ++g) s += red[g * HH_NB + tid];
    ha_store_wt(part + (int64_t)blockIdx.x * HH_NB + tid, s);
  }
  const int gb = (gridDim.x + HH_COPIES - 1) / HH_COPIES;  // blocks per group
  const int group = blockIdx.x / gb;
  const int b0 = group * gb, b1 = b0 + gb < (int)gridDim.x ? b0 + gb : (int)gridDim.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add((ha_gu32*)(cnt + group), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    last = t == (unsigned)(b1 - b0 - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store((ha_gu32*)(cnt + group), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (last) {
    // the group's partials over all 256 threads: thread (sub = tid / 32, column tid % 32) sums
    // blocks b0 + sub, b0 + sub + 8, ... (independent loads in flight), then a fixed pairwise tree
    // over the 8 subs. One thread walking the ~64 partials of its column was a chain of dependent
    // L2 round trips: ~30 us of the ~50 us fixed cost per launch (tools/microbench/hh_step_scan.py)
    const int col = tid & (HH_NB - 1), sub = tid >> 5;
    double s = 0.0;
#pragma unroll 4
    for (int b = b0 + sub; b < b1; b += 8) s += part[(int64_t)b * HH_NB + col];
    red[sub * HH_NB + col] = s;
    __syncthreads();
    if (tid < HH_NB)
      out[group * HH_SLEN + tid] = ((red[tid] + red[HH_NB + tid]) + (red[2 * HH_NB + tid] + red[3 * HH_NB + tid])) +
                                   ((red[4 * HH_NB + tid] + red[5 * HH_NB + tid]) +
                                    (red[6 * HH_NB + tid] + red[7 * HH_NB + tid]));
  }
  __syncthreads();
}

// Sum of the HH_COPIES replicated accumulators of one S buffer into LDS (every block): thread
// (quarter q = tid / 64, element e = tid % 64) adds copies q, q + 4, ... (8 independent loads),
// then a fixed-order sum of the 4 quarters. `scratch`: 256 doubles of LDS.
__device__ __forceinline__ void hh_gather_s(const double* __restrict__ S, double* __restrict__ out,
                                            double* __restrict__ scratch) {
  static_assert(HH_SLEN == 64 && HH_COPIES % 4 == 0, "one element per lane of a quarter");
  const int e = threadIdx.x & 63, q = threadIdx.x >> 6;
  double v = 0.0;
#pragma unroll
  for (int c = q; c < HH_COPIES; c += 4) v += S[c * HH_SLEN + e];
  scratch[q * 64 + e] = v;
  __syncthreads();
  if (threadIdx.x < 64) out[e] = (scratch[e] + scratch[64 + e]) + (scratch[128 + e] + scratch[192 + e]);
  __syncthreads();
}

// S / rowd of the first column of a panel: S[c] = sum_{g >= d} A[g][0] A[g][c], rowd = row d.
template <typename T>
__global__ __launch_bounds__(256) void hh_colsums(const T* __restrict__ A, int64_t m, int64_t lda, int64_t g0,
                                                  int64_t k0, int ncols, int64_t d, double* __restrict__ S,
                                                  double* __restrict__ part, unsigned* __restrict__ cnt) {
  __shared__ double red[32 * HH_NB];
  const int q = threadIdx.x & 7;
  const int nh = ncols - 4 * q < 4 ? (ncols - 4 * q > 0 ? ncols - 4 * q : 0) : 4;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t i = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3); i < m; i += (int64_t)gridDim.x * 32) {
    const int64_t g = g0 + i;
    if (g < d) continue;
    const Vec4<T> a = hh_load4(A + i * lda + k0 + 4 * q, nh);
    const double x0 = (double)__shfl(a.v[0], threadIdx.x & ~7, 64);  // column 0 lives on lane 0 of the group
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += x0 * (double)a.v[c];
    if (g == d) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nh) S[HH_NB + 4 * q + c] = (double)a.v[c];  // row d: exactly one writer
    }
  }
  hh_block_sum(acc, S, red, part, cnt);
}

// ROWS: rows per thread and sweep in hh_step, loads issued before the first use (with the serial
// block-sum tail, 4 measured SLOWER: 4.34 vs 2.74 ms per 32-column panel at 1.25e6 rows, r4t).
// A/B switches (read once): HEAT_HH_ROWS (1 | 2 | 4), HEAT_HH_BLOCKS_PER_CU (grid cap, default 4).
// Measured per launch at 1.25e6 rows with the parallel tails (r4y, tools/microbench/hh_step_scan.py):
// rows 1 / 4 blocks per CU 66 us, rows 2 / 4 66 us, rows 1 / 8 68-79 us, rows 4 / 8 102 us.
static int hh_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

// hh_step's work on one row g >= d (a: the row's 4 panel values of this lane, already loaded)
template <typename T>
__device__ __forceinline__ void hh_step_row(Vec4<T>& a, T* row, int64_t g, int64_t d, int j, int jl, int jq, int j1l,
                                            int j1q, int q, int ncols, int nh, bool wr, double beta, double tauv,
                                            double scale, const double (&w)[4], double* __restrict__ Sout,
                                            double (&acc)[4]) {
  if (g == d) {
    // the owner writes the R row: beta on the diagonal, rowd[c] - tau w_c right of it
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int col = 4 * q + c;
      if (col == j) a.v[c] = (T)beta;
      else if (col > j && col < ncols) a.v[c] = (T)((double)a.v[c] - tauv * w[c]);
    }
    if (wr) hh_store4(row, a, nh);
    return;
  }
  // g > d: v_g = x_g / (alpha - beta), A[g][c] -= tau v_g w_c
  const T xj = __shfl(a.v[jl], (threadIdx.x & ~7) + jq, 64);
  const double v = (double)xj * scale;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int col = 4 * q + c;
    if (col == j) a.v[c] = (T)v;
    else if (col > j && col < ncols) a.v[c] = (T)((double)a.v[c] - tauv * v * w[c]);
  }
  if (wr) hh_store4(row, a, nh);
  if (Sout) {
    // next column's sums over rows g >= d + 1 (all rows handled here), row d + 1's values
    const double x1 = (double)__shfl(a.v[j1l], (threadIdx.x & ~7) + j1q, 64);
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += x1 * (double)a.v[c];
    if (g == d + 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nh) Sout[HH_NB + 4 * q + c] = (double)a.v[c];  // row d + 1: one writer
    }
  }
}

// One panel column: apply reflector j (from Sin) to this rank's rows, store v / R, accumulate the
// next column's S / rowd into Sout (nullptr for the panel's last column).
template <typename T, int HH_ROWS>
__global__ __launch_bounds__(256) void hh_step(T* __restrict__ A, int64_t m, int64_t lda, int64_t g0, int64_t k0,
                                               int64_t coff, int ncols, int j, const double* __restrict__ Sin,
                                               double* __restrict__ Sout, T* __restrict__ tau,
                                               double* __restrict__ Y, double* __restrict__ part,
                                               unsigned* __restrict__ cnt) {
  __shared__ double red[32 * HH_NB];
  __shared__ double sin_[HH_SLEN];
  hh_gather_s(Sin, sin_, red);
  const int64_t d = k0 + j;
  const int q = threadIdx.x & 7;
  const int nh = ncols - 4 * q < 4 ? (ncols - 4 * q > 0 ? ncols - 4 * q : 0) : 4;
  // reflector scalars (identical in every thread of every block)
  const double alpha = sin_[HH_NB + j];
  const double nrm2 = sin_[j];
  const double sig = nrm2 - alpha * alpha;  // sum of squares strictly below the diagonal
  double beta = alpha, tauv = 0.0, scale = 0.0;
  if (sig > 0.0 && nrm2 > 0.0) {
    const double nx = sqrt(nrm2);
    beta = alpha >= 0.0 ? -nx : nx;
    tauv = (beta - alpha) / beta;
    scale = 1.0 / (alpha - beta);
  }
  double w[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int col = 4 * q + c;
    const double rd = sin_[HH_NB + col];
    w[c] = (col > j && col < ncols) ? rd + scale * (sin_[col] - alpha * rd) : 0.0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) tau[j] = (T)tauv;
  if (Y && blockIdx.x == 0 && threadIdx.x <= j) {
    // column j of Y = V^T V (the larft input) from the same global sums: v_j = e_d + scale x below
    // row d, so for c < j  Y[c][j] = v_c[d] + scale (S[c] - alpha v_c[d])  (v_c[d] = rowd[c]) -
    // the same expression as w_c; Y[j][j] = 1 + scale^2 sig
    const int c = threadIdx.x;
    const double rd = sin_[HH_NB + c];
    Y[c * ncols + j] = c < j ? rd + scale * (sin_[c] - alpha * rd) : 1.0 + scale * scale * sig;
  }
  const int jl = j & 3, jq = j >> 2;              // lane group slot holding column j
  const bool wr = 4 * q + 3 >= j;  // columns < j are read (sums), never changed: no store
  // Y null: the caller forms V^T V itself (one GEMM after the panel), so the finished columns
  // (all 4 of this lane's < j) are not even loaded - the column steps stream only the part of the
  // panel still changing (their S / rowd entries are left zero and unused)
  const bool skip = Y == nullptr && !wr;
  const int j1 = j + 1, j1l = j1 & 3, j1q = j1 >> 2;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * 32;
  for (int64_t i0 = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3); i0 < m; i0 += HH_ROWS * stride) {
    Vec4<T> a[HH_ROWS];
#pragma unroll
    for (int u = 0; u < HH_ROWS; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < m && g0 + i >= d) {
        if (skip) {
#pragma unroll
          for (int c = 0; c < 4; ++c) a[u].v[c] = (T)0;
        } else {
          a[u] = hh_load4(A + i * lda + coff + 4 * q, nh);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < HH_ROWS; ++u) {
      const int64_t i = i0 + u * stride;
      const int64_t g = g0 + i;
      // rows above the diagonal: untouched (the group is uniform in g)
      if (i >= m || g < d) continue;
      T* row = A + i * lda + coff + 4 * q;
      hh_step_row(a[u], row, g, d, j, jl, jq, j1l, j1q, q, ncols, nh, wr, beta, tauv, scale, w, Sout, acc);
    }
  }
  if (Sout) hh_block_sum(acc, Sout, red, part, cnt);
}

// larft: T (nb x nb, upper triangular, row-major, ldt = nb) of the compact WY form
// H_0 ... H_{nb-1} = I - V T V^T from tau and Y = V^T V (fp64, summed over all rows):
// T[j][j] = tau_j, T[0:j, j] = -tau_j T[0:j, 0:j] Y[0:j, j]. One workgroup; column by column.
template <typename T>
__global__ __launch_bounds__(64) void hh_larft(const double* __restrict__ Y, const T* __restrict__ tau, int nb,
                                               T* __restrict__ Tm) {
  __shared__ double t[HH_NB * HH_NB];
  __shared__ double z[HH_NB];
  const int i = threadIdx.x;
  for (int e = i; e < HH_NB * HH_NB; e += 64) t[e] = 0.0;
  __syncthreads();
  for (int j = 0; j < nb; ++j) {
    const double tj = (double)tau[j];
    if (i < j) {
      double s = 0.0;
      for (int k = i; k < j; ++k) s += t[i * HH_NB + k] * Y[k * nb + j];
      z[i] = -tj * s;
    }
    __syncthreads();
    if (i < j) t[i * HH_NB + j] = z[i];
    if (i == 0) t[j * HH_NB + j] = tj;
    __syncthreads();
  }
  for (int e = i; e < nb * nb; e += 64) Tm[e] = (T)t[(e / nb) * HH_NB + e % nb];
}

// W[c][j] += sum_i V[i][c] C[i][j] (c < nc <= 32, j < N) over rows [0, m) with FP64 accumulation:
// the V^T C products of the trailing update / Q accumulation (and V^T V) reduce over ALL rows of
// the matrix (1e6+), where an fp32 GEMM's accumulation error (~sqrt(m) u) would cost
// orthogonality - and rocBLAS's fp64 GEMM is slow on these tall-skinny shapes. Block = 256
// columns of C x a row slice (split-K over blockIdx.y); thread (jl = t % 64, c-group = t / 64)
// owns W rows 8 cg .. 8 cg + 7 of columns jl + 64 u (u < 4): every V value read from LDS feeds 4
// fp64 FMAs. V rows are staged through LDS 64 at a time (broadcast reads); per-split partials are
// summed in split order by hh_vtc_sum.
template <typename T>
__global__ __launch_bounds__(256) void hh_vtc(const T* __restrict__ V, int64_t ldv, const T* __restrict__ C,
                                              int64_t ldc, int64_t m, int64_t N, int nc, int64_t rows_per_split,
                                              double* __restrict__ W, int64_t ldw) {
  // W here is the partial buffer [splits][nc][ldw]
  __shared__ T vs[64 * HH_NB];
  const int t = threadIdx.x, jl = t & 63, cg = t >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * 256 + jl;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < m ? r0 + rows_per_split : m;
  double acc[8][4];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[c][u] = 0.0;
  for (int64_t rb = r0; rb < r1; rb += 64) {
    const int nr = r1 - rb < 64 ? (int)(r1 - rb) : 64;
    __syncthreads();
    for (int e = t; e < 64 * HH_NB; e += 256) {
      const int rr = e / HH_NB, cc = e % HH_NB;
      vs[e] = (rr < nr && cc < nc) ? V[(rb + rr) * ldv + cc] : T(0);
    }
    __syncthreads();
    for (int rr = 0; rr < nr; ++rr) {
      double x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t j = j0 + 64 * u;
        x[u] = j < N ? (double)C[(rb + rr) * ldc + j] : 0.0;
      }
      const T* vr = vs + rr * HH_NB + 8 * cg;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const double v = (double)vr[c];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[c][u] = fma(v, x[u], acc[c][u]);
      }
    }
  }
  // this split's partial block of W (no atomics: a W element would otherwise take one atomic add
  // per split - millions per call); hh_vtc_sum adds the splits
  double* P = W + (int64_t)blockIdx.y * nc * ldw;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t j = j0 + 64 * u;
    if (j >= N) continue;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (8 * cg + c < nc) P[(int64_t)(8 * cg + c) * ldw + j] = acc[c][u];
  }
}

// W[c][j] += sum over splits of P[s][c][j] (coalesced over j)
__global__ __launch_bounds__(256) void hh_vtc_sum(const double* __restrict__ P, int splits, int64_t plane,
                                                  double* __restrict__ W, int64_t total) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    double s = 0.0;
    for (int k = 0; k < splits; ++k) s += P[k * plane + e];
    W[e] += s;
  }
}

int hh_grid(int64_t m) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const int64_t need = (m + 31) / 32;
  static const int per_cu = hh_env("HEAT_HH_BLOCKS_PER_CU", 4);
  const int64_t cap = (int64_t)per_cu * ncu;  // enough waves in flight; tickets spread over HH_COPIES groups
  return (int)(need < cap ? (need > 0 ? need : 1) : cap);
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
HA_EXPORT int ha_hh_nb() { return HH_NB; }
// doubles per S buffer (HH_COPIES replicated accumulators of S[NB] | rowd[NB])
HA_EXPORT int ha_hh_slen() { return HH_COPIES * HH_SLEN; }
// doubles of the per-block partial slots of ha_hh_colsums / ha_hh_step for m local rows, and the
// number of (zeroed, self-resetting) group counters
HA_EXPORT int64_t ha_hh_part_len(int64_t m) { return (int64_t)hh_grid(m) * HH_NB; }
HA_EXPORT int ha_hh_counters() { return HH_COPIES; }

// S (2 NB doubles, zeroed by the caller) += column-0 sums of the panel at column k0 (ncols <= NB
// columns) over this rank's rows g >= d, and row d's values if this rank owns it.
HA_EXPORT int ha_hh_colsums(const void* A, int dtype, int64_t m, int64_t lda, int64_t g0, int64_t k0, int ncols,
                            int64_t d, double* S, double* part, unsigned* cnt, void* stream) {
  if (ncols <= 0 || ncols > HH_NB || m < 0) return HA_BAD_ARG;
  if (m == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(hh_colsums<float>, dim3(hh_grid(m)), dim3(256), 0, s, (const float*)A, m, lda, g0, k0, ncols,
                       d, S, part, cnt);
  else
    hipLaunchKernelGGL(hh_colsums<double>, dim3(hh_grid(m)), dim3(256), 0, s, (const double*)A, m, lda, g0, k0, ncols,
                       d, S, part, cnt);
  return ha_launch_status();
}

// Reflector j of the panel (see the header); Sout (zeroed, 2 NB doubles) receives column j + 1's
// partial sums unless it is null.
// coff: the panel's first column within a row of A (k0 for the matrix itself, 0 for a compact
// panel copy); Y (nullable, ncols x ncols fp64 row-major): receives column j of V^T V. Y null:
// the finished columns (< j) are not loaded and their S entries stay zero (the caller computes
// V^T V after the panel).
HA_EXPORT int ha_hh_step(void* A, int dtype, int64_t m, int64_t lda, int64_t g0, int64_t k0, int64_t coff, int ncols,
                         int j, const double* Sin, double* Sout, void* tau, double* Y, double* part, unsigned* cnt,
                         void* stream) {
  if (ncols <= 0 || ncols > HH_NB || j < 0 || j >= ncols || m < 0 || coff < 0) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int grid = hh_grid(m);
  static const int rows = hh_env("HEAT_HH_ROWS", 1);
#define HA_HH_STEP(T, R)                                                                                    \
  hipLaunchKernelGGL((hh_step<T, R>), dim3(grid), dim3(256), 0, s, (T*)A, m, lda, g0, k0, coff, ncols, j, Sin, Sout, \
                     (T*)tau, Y, part, cnt)
  if (dtype == 0) {
    if (rows >= 4) HA_HH_STEP(float, 4);
    else if (rows == 2) HA_HH_STEP(float, 2);
    else HA_HH_STEP(float, 1);
  } else {
    HA_HH_STEP(double, 1);
  }
#undef HA_HH_STEP
  return ha_launch_status();
}

HA_EXPORT int ha_hh_larft(const double* Y, const void* tau, int nb, int dtype, void* Tm, void* stream) {
  if (nb <= 0 || nb > HH_NB) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(hh_larft<float>, dim3(1), dim3(64), 0, s, Y, (const float*)tau, nb, (float*)Tm);
  else
    hipLaunchKernelGGL(hh_larft<double>, dim3(1), dim3(64), 0, s, Y, (const double*)tau, nb, (double*)Tm);
  return ha_launch_status();
}

// Number of row splits ha_hh_vtc uses for (m, N) (the caller sizes the partial buffer:
// splits * nc * N doubles).
HA_EXPORT int64_t ha_hh_vtc_splits(int64_t m, int64_t N) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const int64_t bx = (N + 255) / 256;
  int64_t splits = (4LL * ncu + bx - 1) / bx;  // ~4 blocks per CU overall
  const int64_t maxs = (m + 255) / 256;        // >= 256 rows per split
  splits = splits < maxs ? splits : maxs;
  splits = splits < 1 ? 1 : splits > 65535 ? 65535 : splits;
  const int64_t rps = ((m + splits - 1) / splits + 63) / 64 * 64;
  return (m + rps - 1) / rps;
}

// W (fp64 [nc][N], contiguous) += V[:, :nc]^T C[:, :N] over m rows, fp64 accumulation.
// P: scratch of ha_hh_vtc_splits(m, N) * nc * N doubles.
HA_EXPORT int ha_hh_vtc(const void* V, int64_t ldv, const void* C, int64_t ldc, int dtype, int64_t m, int64_t N,
                        int nc, double* W, double* P, void* stream) {
  if (nc <= 0 || nc > HH_NB || m < 0 || N < 0 || !P) return HA_BAD_ARG;
  if (m == 0 || N == 0) return HA_OK;
  const int64_t bx = (N + 255) / 256;
  const int64_t splits = ha_hh_vtc_splits(m, N);
  const int64_t rps = ((m + splits - 1) / splits + 63) / 64 * 64;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(hh_vtc<float>, dim3((unsigned)bx, (unsigned)splits), dim3(256), 0, s, (const float*)V, ldv,
                       (const float*)C, ldc, m, N, nc, rps, P, N);
  else
    hipLaunchKernelGGL(hh_vtc<double>, dim3((unsigned)bx, (unsigned)splits), dim3(256), 0, s, (const double*)V, ldv,
                       (const double*)C, ldc, m, N, nc, rps, P, N);
  const int64_t total = (int64_t)nc * N;
  const int64_t g = (total + 255) / 256;
  hipLaunchKernelGGL(hh_vtc_sum, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, s, P, (int)splits, total, W,
                     total);
  return ha_launch_status();
}
