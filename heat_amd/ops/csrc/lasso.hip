// Lasso cyclic coordinate descent on CDNA4 (reference heat/regression/lasso.py:121-175).
//
// The reference recomputes the full prediction x @ theta for EVERY coordinate (O(m n^2) per
// sweep) and syncs the host ~3 times per coordinate.  Here the residual r = y - X theta is kept
// on the device and the features are stored transposed (one contiguous row per feature), so one
// coordinate step is ONE fused pass:  r -= delta_{j-1} * X_{j-1}  and  partial += X_j . r
// (coalesced 16-byte loads), then a one-thread update applies the (reference-identical) rule
//   rho = <X_j, r>/m + theta_j * <X_j, X_j>/m ;  theta_j = rho (intercept) | soft(rho, lambda)
// without any host round trip.  Distributed rows add ONE scalar all-reduce between the two.
#include "common.h"

namespace {

constexpr int LASSO_SLOTS = 4;  // partial[0] result, [1] arrival counter, then one slot per block

__global__ __launch_bounds__(256) void lasso_pass(const float* __restrict__ xt, int64_t m, int64_t ldxt, int jprev,
                                                  int jnext, const float* __restrict__ delta, float* __restrict__ r,
                                                  float* __restrict__ partial) {
  const float d = (jprev >= 0) ? *delta : 0.f;
  const float* xp = jprev >= 0 ? xt + (int64_t)jprev * ldxt : nullptr;
  const float* xn = jnext >= 0 ? xt + (int64_t)jnext * ldxt : nullptr;
  float acc = 0.f;
  const int64_t nv = m / 4;
  const bool vec = ((ldxt & 3) == 0) && ((reinterpret_cast<uintptr_t>(r) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(xt) & 15) == 0);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t tail0 = 0;
  if (vec) {
    floatx4* r4 = reinterpret_cast<floatx4*>(r);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nv; q += stride) {
      floatx4 rv = r4[q];
      if (xp) {
        const floatx4 a = reinterpret_cast<const floatx4*>(xp)[q];
        rv = rv - d * a;
        r4[q] = rv;
      }
      if (xn) {
        const floatx4 b = reinterpret_cast<const floatx4*>(xn)[q];
        acc = fmaf(b[0], rv[0], acc);
        acc = fmaf(b[1], rv[1], acc);
        acc = fmaf(b[2], rv[2], acc);
        acc = fmaf(b[3], rv[3], acc);
      }
    }
    tail0 = nv * 4;
  }
  for (int64_t i = tail0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    float rv = r[i];
    if (xp) {
      rv -= d * xp[i];
      r[i] = rv;
    }
    if (xn) acc = fmaf(xn[i], rv, acc);
  }
  if (xn) {
    // deterministic dot product: the block's sum goes to its own slot (written through, sc1) and
    // the last-arriving block adds the slots in block order (a float atomicAdd made theta depend
    // on the arrival order of the blocks); partial[0] = result, partial[1] = arrival counter
    acc = ha_wave_sum(acc);
    __shared__ float sh[4];
    __shared__ bool last;
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float b = (sh[0] + sh[1]) + (sh[2] + sh[3]);
      __hip_atomic_store((ha_gu32*)(partial + LASSO_SLOTS + blockIdx.x), __float_as_uint(b), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add((ha_gu32*)(partial + 1), 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      last = t == gridDim.x - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store((ha_gu32*)(partial + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    if (!last) return;
    float t = 0.f;
    for (unsigned q = threadIdx.x; q < gridDim.x; q += blockDim.x) t += partial[LASSO_SLOTS + q];
    t = ha_wave_sum(t);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) partial[0] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  }
}

__global__ void lasso_update(float* __restrict__ theta, int j, float* __restrict__ partial,
                             const float* __restrict__ colsq, float lam, float inv_m, float* __restrict__ delta,
                             int intercept) {
  const float old = theta[j];
  const float rho = partial[0] * inv_m + old * colsq[j];
  float nw;
  if (intercept) nw = rho;
  else nw = rho < -lam ? rho + lam : (rho > lam ? rho - lam : 0.f);
  theta[j] = nw;
  *delta = nw - old;
}

// Fit preparation in one pass over X (row-major [m][n]): XT = X^T (feature-major, the layout of
// lasso_pass) and the per-workgroup column sums of squares.  64 x 64 tiles through LDS (+1
// padding), workgroups striding over 64-row bands; lasso_colsq adds the partials in order.
// Replaces torch's transpose copy + (XT*XT).sum(1), which took 4 ms of a 5 ms sweep at 1e7 x 16.
__global__ __launch_bounds__(256) void lasso_prepare(const float* __restrict__ x, int64_t m, int n, int64_t ldx,
                                                     float* __restrict__ xt, int64_t ldxt,
                                                     float* __restrict__ colpart) {
  __shared__ float tile[64][65];
  const int c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  float sq = 0.f;                                          // column c0 + tx (thread rows ty = 0 only)
  // grid-stride over 64-row bands (bounded grid: the column partials are gridDim.x x n floats)
  for (int64_t band = blockIdx.x; band * 64 < m; band += gridDim.x) {
    const int64_t r0 = band * 64;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = ty * 16 + i;
      const int64_t r = r0 + rr;
      const int c = c0 + tx;
      const float v = (r < m && c < n) ? x[r * ldx + c] : 0.f;
      tile[rr][tx] = v;
    }
    __syncthreads();
    // write transposed: thread (tx, ty) writes rows c0 + ty*16 + i, columns r0 + tx
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int cc = ty * 16 + i;
      const int c = c0 + cc;
      const int64_t r = r0 + tx;
      const float v = tile[tx][cc];
      if (c < n && r < m) xt[(int64_t)c * ldxt + r] = v;
    }
    // column sums of squares: thread tx of wave 0 sums column tx over the 64 rows
    if (ty == 0) {
#pragma unroll 8
      for (int rr = 0; rr < 64; ++rr) {
        const float v = tile[rr][tx];
        sq = fmaf(v, v, sq);
      }
    }
    __syncthreads();
  }
  if (ty == 0 && c0 + tx < n) colpart[(int64_t)blockIdx.x * n + c0 + tx] = sq;
}

// Narrow X (n <= 64 features, e.g. 16): one row per thread. A thread loads its whole row (16-byte
// pieces when aligned, all issued before use) and writes feature j to xt[j][row]: consecutive
// threads write consecutive rows, so every store instruction is 256 contiguous bytes. Column sums
// of squares stay in registers over a grid-stride loop and leave with one atomic per (workgroup,
// column). (The 64 x 64 tile kernel above keeps 3/4 of its lanes idle at n = 16: 1.03 ms at 1e7 x 16.)
template <int NC, bool VEC>
__global__ __launch_bounds__(256) void lasso_prepare_rows(const float* __restrict__ x, int64_t m, int n, int64_t ldx,
                                                          float* __restrict__ xt, int64_t ldxt,
                                                          float* __restrict__ colpart) {
  __shared__ float red[4][NC];
  float sq[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) sq[j] = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256) {
    float v[NC];
    const float* xr = x + r * ldx;
    if (VEC) {
#pragma unroll
      for (int q = 0; q < NC / 4; ++q) {
        floatx4 p = {0.f, 0.f, 0.f, 0.f};
        if (4 * q < n) p = *reinterpret_cast<const floatx4*>(xr + 4 * q);
        v[4 * q] = p[0];
        v[4 * q + 1] = p[1];
        v[4 * q + 2] = p[2];
        v[4 * q + 3] = p[3];
      }
    } else {
#pragma unroll
      for (int j = 0; j < NC; ++j) v[j] = j < n ? xr[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j < n) xt[(int64_t)j * ldxt + r] = v[j];
      sq[j] = fmaf(v[j], v[j], sq[j]);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const float s = ha_wave_sum(sq[j]);
    if (lane == 0) red[wave][j] = s;
  }
  __syncthreads();
  if (threadIdx.x < n) {
    const int j = threadIdx.x;
    colpart[(int64_t)blockIdx.x * n + j] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
  }
}

// colsq[j] = sum over the B workgroup partials colpart[b][j] in a fixed order (one workgroup per
// column: strided per-thread sums, then wave butterflies and the 4 wave sums in order)
__global__ __launch_bounds__(256) void lasso_colsq(const float* __restrict__ colpart, int64_t B, int n,
                                                   float* __restrict__ colsq) {
  __shared__ float sh[4];
  const int j = blockIdx.x;
  float t = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 256) t += colpart[b * n + j];
  t = ha_wave_sum(t);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) colsq[j] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

}  // namespace

// Workgroups of ha_lasso_prepare for (m, n): its colpart scratch holds blocks * n floats.
static int64_t lasso_prepare_blocks(int64_t m, int n) {
  if (n <= 64) {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
    int64_t blocks = (m + 255) / 256;
    if (blocks > 8LL * ncu) blocks = 8LL * ncu;
    return blocks < 1 ? 1 : blocks;
  }
  const int64_t bands = (m + 63) / 64;
  return bands < 2048 ? bands : 2048;
}

HA_EXPORT int64_t ha_lasso_prepare_scratch(int64_t m, int n) {
  return m <= 0 || n <= 0 ? 1 : lasso_prepare_blocks(m, n) * (int64_t)n;
}

// XT = X^T and colsq[j] = sum_i X[i][j]^2 (fixed-order, bit-reproducible); colpart: scratch of
// ha_lasso_prepare_scratch(m, n) floats.
HA_EXPORT int ha_lasso_prepare(const float* x, int64_t m, int n, int64_t ldx, float* xt, int64_t ldxt, float* colsq,
                               float* colpart, void* stream) {
  if (m <= 0 || n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t blocks = lasso_prepare_blocks(m, n);
  if (n <= 64) {
    const bool vec = n % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
#define HA_LP(NC)                                                                                           \
  if (vec)                                                                                                  \
    hipLaunchKernelGGL((lasso_prepare_rows<NC, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, m, n, ldx, xt, \
                       ldxt, colpart);                                                                      \
  else                                                                                                      \
    hipLaunchKernelGGL((lasso_prepare_rows<NC, false>), dim3((unsigned)blocks), dim3(256), 0, s, x, m, n, ldx, xt, \
                       ldxt, colpart);
    if (n <= 16) {
      HA_LP(16)
    } else if (n <= 32) {
      HA_LP(32)
    } else {
      HA_LP(64)
    }
#undef HA_LP
  } else {
    if ((n + 63) / 64 > 65535) return HA_UNSUPPORTED;
    hipLaunchKernelGGL(lasso_prepare, dim3((unsigned)blocks, (unsigned)((n + 63) / 64)), dim3(256), 0, s, x, m, n,
                       ldx, xt, ldxt, colpart);
  }
  hipLaunchKernelGGL(lasso_colsq, dim3((unsigned)n), dim3(256), 0, s, colpart, blocks, n, colsq);
  return ha_launch_status();
}

// Floats of ha_lasso_pass's partial buffer: result, arrival counter (zero before the first pass,
// reset by every pass), padding, one slot per workgroup.
HA_EXPORT int64_t ha_lasso_partial_floats(int num_cus) { return LASSO_SLOTS + (int64_t)num_cus * 4; }

HA_EXPORT int ha_lasso_pass(const float* xt, int64_t m, int64_t ldxt, int jprev, int jnext, const float* delta,
                            float* r, float* partial, int num_cus, void* stream) {
  if (m <= 0 && jnext < 0) return HA_OK;
  int64_t blocks = (m / 4 + 255) / 256;
  const int64_t cap = (int64_t)num_cus * 4;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(lasso_pass, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, xt, m, ldxt, jprev, jnext,
                     delta, r, partial);
  return ha_launch_status();
}

HA_EXPORT int ha_lasso_update(float* theta, int j, float* partial, const float* colsq, float lam, float inv_m,
                              float* delta, int intercept, void* stream) {
  hipLaunchKernelGGL(lasso_update, dim3(1), dim3(1), 0, (hipStream_t)stream, theta, j, partial, colsq, lam, inv_m,
                     delta, intercept);
  return ha_launch_status();
}
