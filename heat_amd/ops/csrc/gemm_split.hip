// fp32 GEMM emulated on the FP16 matrix cores ("fp16x3" split GEMM).
//
// MI355X runs fp16 MFMA at 16x the fp32 MFMA rate (2.5 PFLOP/s vs 157 TFLOP/s dense), and the
// library fp32 GEMM (hipBLASLt) sits at ~150 TFLOP/s. Splitting each fp32 operand into two fp16
// planes, x = s^-1 (hi + lo), and contracting
//     A B ~= s_A^-1 s_B^-1 (hi_A hi_B + hi_A lo_B + lo_A hi_B)
// recovers fp32-GEMM accuracy (the dropped lo_A lo_B term and the fp16 rounding of lo are both
// <= 2^-22 relative to |a||b| per product; products are exact in fp32 and accumulate in fp32 like
// a plain fp32 GEMM) at one third of the fp16 rate. The three products are ONE library GEMM with a
// tripled contraction dimension: [hi_A | hi_A | lo_A] (M x 3K) times [hi_B ; lo_B ; hi_B] (3K x N),
// fp16 in, fp32 accumulate and out (measured 1.24 PFLOP/s raw = ~410 TFLOP/s fp32-equivalent,
// 2.7x the fp32 GEMM; tools/microbench/mm_f16_probe.py).
//
// The power-of-two scales s are per row of A and per column of B (the non-contracted dims), so
// they factor out of the dot products exactly; they put each row's (column's) largest magnitude
// in [2^14, 2^15): far from fp16 overflow (65504) and with the smallest kept magnitudes 2^-38
// below the largest before fp16's subnormal range. This file holds the memory-bound parts: the
// per-row/column absmax (with a non-finite flag: the caller falls back to the fp32 GEMM on
// inf/nan, whose propagation the split cannot reproduce), the split into the K-tripled layout,
// and the exact ldexp unscaling epilogue of the product.
#include "common.h"

#include <float.h>

namespace {

typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));

// e such that m * 2^e in [2^14, 2^15); 0 for zero / non-finite maxima
__device__ __forceinline__ int sp_exp(float m) {
  return (m > 0.f && m <= FLT_MAX) ? 14 - ilogbf(m) : 0;
}

__device__ __forceinline__ bool sp_bad(float v) { return !(fabsf(v) <= FLT_MAX); }

// max |x| of every physical row; one wave per row. VEC: 16-byte loads (C % 4 == 0, ld % 4 == 0,
// aligned base).
template <bool VEC>
__global__ __launch_bounds__(256) void sp_rowmax(const float* __restrict__ X, int64_t R, int64_t C, int64_t ld,
                                                 float* __restrict__ mx, int* __restrict__ flag) {
  const int lane = threadIdx.x & 63;
  bool bad = false;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += (int64_t)gridDim.x * 4) {
    const float* p = X + r * ld;
    float m = 0.f;
    if (VEC) {
      for (int64_t c = 4 * lane; c < C; c += 256) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(p + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bad |= sp_bad(v[q]);
          m = fmaxf(m, fabsf(v[q]));
        }
      }
    } else {
      for (int64_t c = lane; c < C; c += 64) {
        const float v = p[c];
        bad |= sp_bad(v);
        m = fmaxf(m, fabsf(v));
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) mx[r] = m;
  }
  if (__ballot(bad) != 0ull && lane == 0) atomicOr(flag, 1);
}

// max |x| of every physical column (mx zeroed by the caller; non-negative floats order like their
// bit patterns, so the merge is an unsigned atomicMax). Thread = 4 consecutive columns over a band
// of rows.
__global__ __launch_bounds__(256) void sp_colmax(const float* __restrict__ X, int64_t R, int64_t C, int64_t ld,
                                                 int rows_per_blk, unsigned* __restrict__ mx, int* __restrict__ flag) {
  const int64_t c0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t r1 = r0 + rows_per_blk < R ? r0 + rows_per_blk : R;
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  bool bad = false;
  if (c0 < C) {
    const int nq = C - c0 >= 4 ? 4 : (int)(C - c0);
    for (int64_t r = r0; r < r1; ++r) {
      const float* p = X + r * ld + c0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < nq) {
          const float v = p[q];
          bad |= sp_bad(v);
          m[q] = fmaxf(m[q], fabsf(v));
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < nq && m[q] > 0.f) atomicMax(mx + c0 + q, __float_as_uint(m[q]));
  }
  if (__ballot(bad) != 0ull && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// hi/lo planes of the scaled matrix. axis 0: scale per physical row, 1: per physical column.
// hi goes to hi0 (and hi1, hi2 when given), lo to lo; all outputs [R, C] with leading dimension
// ldo. Three hi copies serve the Gram product X^T X from one buffer [h; h; l; h]: its rows
// [R, 4R) are the left operand [h; l; h], rows [0, 3R) the right one [h; h; l].
// ex[] receives the exponents (written by the first column / row of threads).
template <bool VEC>
__global__ __launch_bounds__(256) void sp_split3(const float* __restrict__ X, int64_t R, int64_t C, int64_t ld, int axis,
                                                 const float* __restrict__ mx, _Float16* __restrict__ hi0,
                                                 _Float16* __restrict__ hi1, _Float16* __restrict__ hi2,
                                                 _Float16* __restrict__ lo, int64_t ldo, int* __restrict__ ex) {
  constexpr int W = VEC ? 4 : 1;
  const int64_t cw = (C + W - 1) / W;
  const int64_t total = R * cw;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / cw;
    const int64_t c = (t - r * cw) * W;
    float v[W];
    if (VEC) {
      const floatx4 q = *reinterpret_cast<const floatx4*>(X + r * ld + c);
#pragma unroll
      for (int i = 0; i < W; ++i) v[i] = q[i];
    } else {
      v[0] = X[r * ld + c];
    }
    int e[W];
    if (axis == 0) {
      const int er = sp_exp(mx[r]);
#pragma unroll
      for (int i = 0; i < W; ++i) e[i] = er;
      if (c == 0) ex[r] = er;
    } else {
#pragma unroll
      for (int i = 0; i < W; ++i) e[i] = sp_exp(mx[c + i]);
      if (r == 0) {
#pragma unroll
        for (int i = 0; i < W; ++i) ex[c + i] = e[i];
      }
    }
    _Float16 h[W], l[W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const float s = ldexpf(v[i], e[i]);
      h[i] = (_Float16)s;
      l[i] = (_Float16)(s - (float)h[i]);
    }
    const int64_t o = r * ldo + c;
    if (VEC) {
      const halfx4 hv = {h[0], h[1], h[2], h[3]};
      const halfx4 lv = {l[0], l[1], l[2], l[3]};
      *reinterpret_cast<halfx4*>(hi0 + o) = hv;
      if (hi1) *reinterpret_cast<halfx4*>(hi1 + o) = hv;
      if (hi2) *reinterpret_cast<halfx4*>(hi2 + o) = hv;
      *reinterpret_cast<halfx4*>(lo + o) = lv;
    } else {
      hi0[o] = h[0];
      if (hi1) hi1[o] = h[0];
      if (hi2) hi2[o] = h[0];
      lo[o] = l[0];
    }
  }
}

// Row-scaled split in one pass over the matrix: a wave owns a row, finds its absmax, then re-reads
// the row (L2-resident: 16 KB at 4096 columns) and writes the planes. Saves the separate absmax
// kernel's full read of X for the row-scaled (left, row-major) operand.
__global__ __launch_bounds__(256) void sp_split3_rows(const float* __restrict__ X, int64_t R, int64_t C, int64_t ld,
                                                      _Float16* __restrict__ hi0, _Float16* __restrict__ hi1,
                                                      _Float16* __restrict__ lo, int64_t ldo, int* __restrict__ ex,
                                                      int* __restrict__ flag) {
  const int lane = threadIdx.x & 63;
  bool bad = false;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += (int64_t)gridDim.x * 4) {
    const float* p = X + r * ld;
    float m = 0.f;
    for (int64_t c = 4 * lane; c < C; c += 256) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(p + c);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bad |= sp_bad(v[q]);
        m = fmaxf(m, fabsf(v[q]));
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const int e = sp_exp(m);
    if (lane == 0) ex[r] = e;
    const int64_t ro = r * ldo;
    for (int64_t c = 4 * lane; c < C; c += 256) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(p + c);
      halfx4 hv, lv;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float s = ldexpf(v[q], e);
        hv[q] = (_Float16)s;
        lv[q] = (_Float16)(s - (float)hv[q]);
      }
      *reinterpret_cast<halfx4*>(hi0 + ro + c) = hv;
      if (hi1) *reinterpret_cast<halfx4*>(hi1 + ro + c) = hv;
      *reinterpret_cast<halfx4*>(lo + ro + c) = lv;
    }
  }
  if (__ballot(bad) != 0ull && lane == 0) atomicOr(flag, 1);
}

// C[i, j] = 2^-(ea[i] + eb[j]) C[i, j]  (exact: a power-of-two rescale of the fp32 product)
template <bool VEC>
__global__ __launch_bounds__(256) void sp_unscale(float* __restrict__ Cm, int64_t M, int64_t N, int64_t ldc,
                                                  const int* __restrict__ ea, const int* __restrict__ eb) {
  constexpr int W = VEC ? 4 : 1;
  const int64_t nw = (N + W - 1) / W;
  const int64_t total = M * nw;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / nw;
    const int64_t j = (t - i * nw) * W;
    const int a = ea[i];
    float* p = Cm + i * ldc + j;
    if (VEC) {
      floatx4 v = *reinterpret_cast<floatx4*>(p);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ldexpf(v[q], -(a + eb[j + q]));
      __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p));
    } else {
      *p = ldexpf(*p, -(a + eb[j]));
    }
  }
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline bool aligned8(const void* p) { return ((uintptr_t)p & 7) == 0; }

unsigned grid_for(int64_t work, int64_t per_block) {
  int64_t b = (work + per_block - 1) / per_block;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

// absmax per physical row (axis 0) or column (axis 1) of X [R, C] (leading dimension ld) into
// mx (float[R] or float[C]); *flag |= 1 if X holds inf/nan (flag zeroed by the caller).
HA_EXPORT int ha_split_absmax(const float* X, int64_t R, int64_t C, int64_t ld, int axis, float* mx, int* flag,
                              void* stream) {
  if (R < 0 || C < 0 || ld < C || (axis != 0 && axis != 1)) return HA_BAD_ARG;
  if (R == 0 || C == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  if (axis == 0) {
    const unsigned g = grid_for(R, 4);
    if (C % 4 == 0 && ld % 4 == 0 && aligned16(X))
      hipLaunchKernelGGL(sp_rowmax<true>, dim3(g), dim3(256), 0, s, X, R, C, ld, mx, flag);
    else
      hipLaunchKernelGGL(sp_rowmax<false>, dim3(g), dim3(256), 0, s, X, R, C, ld, mx, flag);
  } else {
    hipMemsetAsync(mx, 0, (size_t)C * sizeof(float), s);
    const unsigned gx = (unsigned)((C + 1023) / 1024);
    // >= ~2048 workgroups in total, bands of at least 64 rows
    int64_t rows = R * gx / 2048;
    rows = rows < 64 ? 64 : rows;
    const int64_t gy = (R + rows - 1) / rows;
    if (gy > 65535) return HA_UNSUPPORTED;
    hipLaunchKernelGGL(sp_colmax, dim3(gx, (unsigned)gy), dim3(256), 0, s, X, R, C, ld, (int)rows,
                       reinterpret_cast<unsigned*>(mx), flag);
  }
  return ha_launch_status();
}

// fp16 hi/lo planes of X scaled per row (axis 0) or column (axis 1) by the maxima of
// ha_split_absmax; see sp_split3. ex: int32[R] or int32[C].
HA_EXPORT int ha_split3(const float* X, int64_t R, int64_t C, int64_t ld, int axis, const float* mx, void* hi0,
                        void* hi1, void* hi2, void* lo, int64_t ldo, int* ex, void* stream) {
  if (R < 0 || C < 0 || ld < C || ldo < C || (axis != 0 && axis != 1) || !hi0 || !lo) return HA_BAD_ARG;
  if (R == 0 || C == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  _Float16 *h0 = (_Float16*)hi0, *h1 = (_Float16*)hi1, *h2 = (_Float16*)hi2, *l = (_Float16*)lo;
  const bool vec = C % 4 == 0 && ld % 4 == 0 && ldo % 4 == 0 && aligned16(X) && aligned8(h0) && aligned8(l) &&
                   (!h1 || aligned8(h1)) && (!h2 || aligned8(h2));
  if (vec)
    hipLaunchKernelGGL(sp_split3<true>, dim3(grid_for(R * (C / 4), 256)), dim3(256), 0, s, X, R, C, ld, axis, mx,
                       h0, h1, h2, l, ldo, ex);
  else
    hipLaunchKernelGGL(sp_split3<false>, dim3(grid_for(R * C, 256)), dim3(256), 0, s, X, R, C, ld, axis, mx, h0, h1,
                       h2, l, ldo, ex);
  return ha_launch_status();
}

// Fused absmax + split for per-row scales (16-byte aligned rows; returns HA_UNSUPPORTED otherwise,
// the caller then uses ha_split_absmax + ha_split3). *flag |= 1 on inf/nan.
HA_EXPORT int ha_split3_rows(const float* X, int64_t R, int64_t C, int64_t ld, void* hi0, void* hi1, void* lo,
                             int64_t ldo, int* ex, int* flag, void* stream) {
  if (R < 0 || C < 0 || ld < C || ldo < C || !hi0 || !lo) return HA_BAD_ARG;
  if (R == 0 || C == 0) return HA_OK;
  _Float16 *h0 = (_Float16*)hi0, *h1 = (_Float16*)hi1, *l = (_Float16*)lo;
  if (!(C % 4 == 0 && ld % 4 == 0 && ldo % 4 == 0 && aligned16(X) && aligned8(h0) && aligned8(l) &&
        (!h1 || aligned8(h1))))
    return HA_UNSUPPORTED;
  hipLaunchKernelGGL(sp_split3_rows, dim3(grid_for(R, 4)), dim3(256), 0, (hipStream_t)stream, X, R, C, ld, h0, h1, l,
                     ldo, ex, flag);
  return ha_launch_status();
}

// C [M, N] (row-major, leading dimension ldc) *= 2^-(ea[i] + eb[j])
HA_EXPORT int ha_split_unscale(float* Cm, int64_t M, int64_t N, int64_t ldc, const int* ea, const int* eb,
                               void* stream) {
  if (M < 0 || N < 0 || ldc < N) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  if (N % 4 == 0 && ldc % 4 == 0 && aligned16(Cm))
    hipLaunchKernelGGL(sp_unscale<true>, dim3(grid_for(M * (N / 4), 256)), dim3(256), 0, s, Cm, M, N, ldc, ea, eb);
  else
    hipLaunchKernelGGL(sp_unscale<false>, dim3(grid_for(M * N, 256)), dim3(256), 0, s, Cm, M, N, ldc, ea, eb);
  return ha_launch_status();
}
