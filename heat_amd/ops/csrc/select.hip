// Selection kernels: packed (value, index) arg-reductions and per-row top-k
// (K13) for ht.argmax / ht.argmin / ht.topk.
//
// Both order elements by ONE signed 64-bit key:
//     key = (okey(v) << 32) | tie,   tie = 0xFFFFFFFF - idx  (larger key wins: the first index)
// okey maps the value to a signed 32-bit integer with the value's order (floats: sign-magnitude ->
// two's-complement order). The smallest-first variants use ~okey (order reversed). NaN: the best
// key for argmax AND argmin (NumPy returns the first NaN for both) and for top-k largest; the
// worst for top-k smallest (torch.topk treats NaN as the largest value). A whole (value, first index) arg-reduction is then a plain integer MAX - locally in the kernels and
// across ranks as ONE int64 MAX all-reduce over RCCL, replacing the reference's pickled custom
// MPI op (statistics.py:1139-1207) and our round-1 all-gather + fold. Indices must be < 2^32.
//
// Inputs are contiguous [O, L, I] views reduced along L (O = outer, I = inner extent).
#include "common.h"

#include <limits.h>

namespace {

template <typename T> __device__ __forceinline__ float ar_tof(T v) { return (float)v; }
template <> __device__ __forceinline__ float ar_tof<uint16_t>(uint16_t v) {  // bf16 bits
  return __uint_as_float(((unsigned)v) << 16);
}

// signed 32-bit order key of a value; SMALL: reversed order (argmin / smallest top-k). NaN_WINS:
// NaN is the best key in either order (NumPy argmax AND argmin return the first NaN); otherwise
// (top-k smallest) NaN counts as the largest value like torch.topk and so comes last.
template <typename T, bool SMALL, bool NAN_WINS = true>
__device__ __forceinline__ int32_t ar_hi(T v) {
  if constexpr (sizeof(T) <= 4 && !(__is_same(T, float) || __is_same(T, _Float16) || __is_same(T, uint16_t))) {
    const int32_t k = (int32_t)v;  // int8/uint8/int16/int32/bool: already ordered
    return SMALL ? ~k : k;
  } else {
    const float f = ar_tof<T>(v);
    if (f != f) return (NAN_WINS || !SMALL) ? INT32_MAX : INT32_MIN;
    unsigned b = __float_as_uint(f);
    if ((b << 1) == 0u) b = 0u;  // -0.0 == +0.0 (a tie, resolved by the index like NumPy)
    const unsigned o = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    const int32_t k = (int32_t)(o ^ 0x80000000u);
    // ~k of a non-NaN never equals INT32_MAX (that would need k = INT32_MIN = -NaN pattern)
    return SMALL ? ~k : k;
  }
}

__device__ __forceinline__ int64_t ar_key(int32_t hi, uint64_t idx) {
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)idx));
}

__device__ __forceinline__ int64_t ar_wave_max(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// ---------------------------------------------------------------------------------- arg-reduce
// Everything -> one key (axis=None): the global flat index of local element (o, l, i) is
// (o * gL + l + displ) * I + i. Grid-stride, wave + block max, one 64-bit atomicMax per block.
template <typename T, bool SMALL>
__global__ __launch_bounds__(256) void ar_all(const T* __restrict__ x, int64_t O, int64_t L, int64_t I, int64_t gL,
                                              int64_t displ, int64_t* __restrict__ out) {
  __shared__ int64_t red[4];
  int64_t best = INT64_MIN;
  const int64_t total = O * L * I;
  if (O == 1) {
    // the common case (split 0, or no dimension before the split axis): the global flat index is
    // e + displ I - no 64-bit divisions per element (they held the pass at ~1.6 TB/s)
    // (4 independent loads per thread in flight; the grid is capped so the per-block 64-bit
    // atomicMax on the one output word stays at ~2K)
    const int64_t base = displ * I;
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; e + 3 * stride < total; e += 4 * stride) {
      const T v0 = x[e], v1 = x[e + stride], v2 = x[e + 2 * stride], v3 = x[e + 3 * stride];
      const int64_t k0 = ar_key(ar_hi<T, SMALL>(v0), (uint64_t)(e + base));
      const int64_t k1 = ar_key(ar_hi<T, SMALL>(v1), (uint64_t)(e + stride + base));
      const int64_t k2 = ar_key(ar_hi<T, SMALL>(v2), (uint64_t)(e + 2 * stride + base));
      const int64_t k3 = ar_key(ar_hi<T, SMALL>(v3), (uint64_t)(e + 3 * stride + base));
      const int64_t a = k0 > k1 ? k0 : k1, b = k2 > k3 ? k2 : k3;
      const int64_t c = a > b ? a : b;
      best = c > best ? c : best;
    }
    for (; e < total; e += stride) {
      const int64_t k = ar_key(ar_hi<T, SMALL>(x[e]), (uint64_t)(e + base));
      best = k > best ? k : best;
    }
  } else {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
      const int64_t in = e % I, t = e / I;
      const int64_t l = t % L, o = t / L;
      const int64_t k = ar_key(ar_hi<T, SMALL>(x[e]), (uint64_t)((o * gL + l + displ) * I + in));
      best = k > best ? k : best;
    }
  }
  best = ar_wave_max(best);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t b = red[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) b = red[w] > b ? red[w] : b;
    if (b != INT64_MIN) atomicMax(reinterpret_cast<long long*>(out), (long long)b);
  }
}

// I == 1: rows of length L are contiguous. One wave per (row, L-slice); 4 rows per block.
template <typename T, bool SMALL>
__global__ __launch_bounds__(256) void ar_rows(const T* __restrict__ x, int64_t O, int64_t L, int64_t displ,
                                               int64_t chunk, int64_t* __restrict__ out) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= O) return;
  const int lane = threadIdx.x & 63;
  const int64_t l0 = (int64_t)blockIdx.y * chunk;
  const int64_t l1 = l0 + chunk < L ? l0 + chunk : L;
  const T* row = x + o * L;
  int64_t best = INT64_MIN;
  for (int64_t l = l0 + lane; l < l1; l += 64) {
    const int64_t k = ar_key(ar_hi<T, SMALL>(row[l]), (uint64_t)(l + displ));
    best = k > best ? k : best;
  }
  best = ar_wave_max(best);
  if (lane == 0 && best != INT64_MIN) {
    if (gridDim.y == 1) out[o] = best;
    else atomicMax(reinterpret_cast<long long*>(out + o), (long long)best);
  }
}

// I > 1: thread per (o, i) column walking L with stride I (coalesced across threads); the L range
// is split over gridDim.z slices (atomicMax merge) when O * I alone cannot fill the GPU.
template <typename T, bool SMALL>
__global__ __launch_bounds__(256) void ar_cols(const T* __restrict__ x, int64_t O, int64_t L, int64_t I,
                                               int64_t displ, int64_t chunk, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t o = blockIdx.y;
  if (i >= I) return;
  const int64_t l0 = (int64_t)blockIdx.z * chunk;
  const int64_t l1 = l0 + chunk < L ? l0 + chunk : L;
  const T* col = x + o * L * I + i;
  int64_t best = INT64_MIN;
  for (int64_t l = l0; l < l1; ++l) {
    const int64_t k = ar_key(ar_hi<T, SMALL>(col[l * I]), (uint64_t)(l + displ));
    best = k > best ? k : best;
  }
  if (best == INT64_MIN) return;
  if (gridDim.z == 1) out[o * I + i] = best;
  else atomicMax(reinterpret_cast<long long*>(out + o * I + i), (long long)best);
}

int num_cus_cached() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

template <typename T, bool SMALL>
int ar_launch(const void* xv, int64_t O, int64_t L, int64_t I, int64_t gL, int64_t displ, int mode, int64_t* out,
              hipStream_t s) {
  const T* x = (const T*)xv;
  const int64_t target = 8LL * num_cus_cached();  // workgroups wanted in flight
  if (mode == 0) {
    const int64_t total = O * L * I;
    int64_t blocks = (total + 255) / 256;
    const int64_t cap = O == 1 ? target : 4 * target;
    blocks = blocks < cap ? blocks : cap;
    hipLaunchKernelGGL((ar_all<T, SMALL>), dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(256), 0, s, x, O, L, I,
                       gL, displ, out);
  } else if (I == 1) {
    const int64_t bx = (O + 3) / 4;
    int64_t sy = bx >= target ? 1 : (target + bx - 1) / bx;
    const int64_t maxs = (L + 1023) / 1024;  // >= 1024 elements (16 per lane) per slice
    sy = sy < maxs ? sy : maxs;
    sy = sy < 1 ? 1 : sy > 65535 ? 65535 : sy;
    const int64_t chunk = (L + sy - 1) / sy;
    hipLaunchKernelGGL((ar_rows<T, SMALL>), dim3((unsigned)bx, (unsigned)sy), dim3(256), 0, s, x, O, L, displ, chunk,
                       out);
  } else {
    const int64_t bx = (I + 255) / 256;
    if (O > 65535) return HA_UNSUPPORTED;
    int64_t sz = bx * O >= target ? 1 : (target + bx * O - 1) / (bx * O);
    const int64_t maxs = (L + 63) / 64;
    sz = sz < maxs ? sz : maxs;
    sz = sz < 1 ? 1 : sz > 65535 ? 65535 : sz;
    const int64_t chunk = (L + sz - 1) / sz;
    hipLaunchKernelGGL((ar_cols<T, SMALL>), dim3((unsigned)bx, (unsigned)O, (unsigned)sz), dim3(256), 0, s, x, O, L,
                       I, displ, chunk, out);
  }
  return ha_launch_status();
}

// ---------------------------------------------------------------------------------- top-k
// One wave per row of length L (contiguous): every lane keeps its KN best keys sorted in
// registers (insertion only where a key beats the lane's KN-th best: after the first few
// elements that is rare), then 6 butterfly rounds merge the 64 lists: list ^ partner's reversed
// list elementwise max = the top KN of their union as a bitonic sequence, re-sorted by a
// KN-element bitonic merge (all compile-time indexed, registers only).
template <int KN>
__device__ __forceinline__ void tk_insert(int64_t (&t)[KN], int64_t v) {
#pragma unroll
  for (int s = KN - 1; s >= 1; --s) {
    const bool ap = v > t[s - 1];
    const bool ac = v > t[s];
    t[s] = ap ? t[s - 1] : (ac ? v : t[s]);
  }
  t[0] = v > t[0] ? v : t[0];
}

template <int KN>
__device__ __forceinline__ void tk_bitonic_sort_desc(int64_t (&t)[KN]) {
#pragma unroll
  for (int j = KN / 2; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < KN; ++i) {
      const int p = i ^ j;
      if (p > i) {
        const int64_t a = t[i], b = t[p];
        t[i] = a > b ? a : b;
        t[p] = a > b ? b : a;
      }
    }
  }
}

template <typename T, bool SMALL, int KN>
__global__ __launch_bounds__(256) void tk_rows(const T* __restrict__ x, int64_t O, int64_t L, int64_t displ, int k,
                                               T* __restrict__ vals, int64_t* __restrict__ idx) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= O) return;
  const int lane = threadIdx.x & 63;
  const T* row = x + o * L;
  int64_t t[KN];
#pragma unroll
  for (int s = 0; s < KN; ++s) t[s] = INT64_MIN;
  for (int64_t l = lane; l < L; l += 64) {
    const int64_t key = ar_key(ar_hi<T, SMALL, false>(row[l]), (uint64_t)l);
    if (key > t[KN - 1]) tk_insert<KN>(t, key);
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    int64_t u[KN];
#pragma unroll
    for (int s = 0; s < KN; ++s) u[s] = __shfl_xor(t[KN - 1 - s], m, 64);  // partner's list, reversed
#pragma unroll
    for (int s = 0; s < KN; ++s) t[s] = t[s] > u[s] ? t[s] : u[s];
    tk_bitonic_sort_desc<KN>(t);
  }
  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < KN; ++s) {
      if (s < k) {
        const bool ok = t[s] != INT64_MIN;
        const int64_t li = ok ? (int64_t)(0xFFFFFFFFu - (uint32_t)(t[s] & 0xFFFFFFFF)) : 0;
        vals[o * k + s] = ok ? row[li] : row[0];
        idx[o * k + s] = ok ? li + displ : -1;
      }
    }
  }
}

template <typename T, bool SMALL>
int tk_launch(const void* xv, int64_t O, int64_t L, int64_t displ, int k, void* vals, int64_t* idx, hipStream_t s) {
  const T* x = (const T*)xv;
  const dim3 grid((unsigned)((O + 3) / 4));
#define HA_TK_ROWS(KN) \
  hipLaunchKernelGGL((tk_rows<T, SMALL, KN>), grid, dim3(256), 0, s, x, O, L, displ, k, (T*)vals, idx)
  if (k <= 1) HA_TK_ROWS(1);
  else if (k <= 2) HA_TK_ROWS(2);
  else if (k <= 4) HA_TK_ROWS(4);
  else if (k <= 8) HA_TK_ROWS(8);
  else if (k <= 16) HA_TK_ROWS(16);
  else if (k <= 32) HA_TK_ROWS(32);
  else return HA_UNSUPPORTED;
#undef HA_TK_ROWS
  return ha_launch_status();
}

// dtype codes shared with ops/kernels.py
enum { D_F32 = 0, D_F16 = 1, D_BF16 = 2, D_I32 = 3, D_I16 = 4, D_I8 = 5, D_U8 = 6 };

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
// Packed arg-reduction keys. mode 0: everything -> out[0] (must hold INT64_MIN on entry); mode 1:
// along L -> out[O * I] (must hold INT64_MIN on entry). smallest: argmin order.
HA_EXPORT int ha_argreduce(const void* x, int dtype, int64_t O, int64_t L, int64_t I, int64_t gL, int64_t displ,
                           int mode, int smallest, int64_t* out, void* stream) {
  if (O < 0 || L < 0 || I < 0 || !out) return HA_BAD_ARG;
  if (O * L * I == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
#define HA_AR(T)                                                                                   \
  return smallest ? ar_launch<T, true>(x, O, L, I, gL, displ, mode, out, s)                         \
                  : ar_launch<T, false>(x, O, L, I, gL, displ, mode, out, s)
  switch (dtype) {
    case D_F32: HA_AR(float);
    case D_F16: HA_AR(_Float16);
    case D_BF16: HA_AR(uint16_t);
    case D_I32: HA_AR(int32_t);
    case D_I16: HA_AR(int16_t);
    case D_I8: HA_AR(int8_t);
    case D_U8: HA_AR(uint8_t);
    default: return HA_UNSUPPORTED;
  }
#undef HA_AR
}

// Top-k (k <= 32) of each contiguous row of length L: vals [O, k] (input dtype), idx [O, k] int64
// (+ displ; -1 past L), sorted best first.
HA_EXPORT int ha_topk_rows(const void* x, int dtype, int64_t O, int64_t L, int64_t displ, int k, int smallest,
                           void* vals, int64_t* idx, void* stream) {
  if (O < 0 || L <= 0 || k <= 0 || L >= 0xFFFFFFFFLL) return HA_BAD_ARG;
  if (O == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
#define HA_TKL(T)                                                                   \
  return smallest ? tk_launch<T, true>(x, O, L, displ, k, vals, idx, s)              \
                  : tk_launch<T, false>(x, O, L, displ, k, vals, idx, s)
  switch (dtype) {
    case D_F32: HA_TKL(float);
    case D_F16: HA_TKL(_Float16);
    case D_BF16: HA_TKL(uint16_t);
    case D_I32: HA_TKL(int32_t);
    case D_I16: HA_TKL(int16_t);
    case D_I8: HA_TKL(int8_t);
    case D_U8: HA_TKL(uint8_t);
    default: return HA_UNSUPPORTED;
  }
#undef HA_TKL
}
