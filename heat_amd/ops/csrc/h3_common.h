// Shared device code of the fp16x3 ("h3") kernels: operand packing, centroid scaling and the
// per-pair score, included by kmeans_f16x3.hip (assignment) and knn_f16x3.hip (top-k) - split so
// the two large template sets compile in parallel and the top-k kernels rebuild on their own.
#pragma once
#include "common.h"

#include <stdlib.h>

namespace {

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

// fp32 -> bf16 bits, round to nearest even (finite input)
__device__ __forceinline__ unsigned h3_bf16_rn(float x) {
  const unsigned b = __float_as_uint(x);
  return (b + 0x7FFFu + ((b >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float h3_bf16_f(unsigned b) { return __uint_as_float(b << 16); }

constexpr int H3_AMB_SHARDS = 16;  // lists of the certified filter's uncertain points

template <int FPAD, int NPB_ = 2>
struct H3Cfg {
  static constexpr int F2 = FPAD / 2;                  // features per lane half
  static constexpr int KS = F2 / 8;                    // k-steps (16 features each)
  static constexpr int CB = FPAD >= 128 ? 64 : 128;    // centroids per LDS chunk
  static constexpr int NPB = NPB_;                     // 32-point blocks per wave
  static constexpr int WAVES = 4;
  static constexpr int PTS_PER_WG = WAVES * NPB * 32;
  static constexpr int CHUNK_H = CB * FPAD * 2;        // halfs of packed (hi, lo) per chunk
};

// planes[row][0:FPAD] = hi, planes[row][FPAD:2 FPAD] = lo; sx[row] = s_x.
template <int FPAD>
__global__ __launch_bounds__(256) void h3_pack_points(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                      _Float16* __restrict__ planes, float* __restrict__ sx) {
  constexpr int LPR = FPAD / 8;  // lanes per row (divides 64)
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = t / LPR;
  const int grp = (int)(t % LPR);
  const bool live = row < n;
  float v[8];
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int col = grp * 8 + i;
    v[i] = (live && col < f) ? X[row * ldx + col] : 0.f;
    mx = fmaxf(mx, fabsf(v[i]));
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  int e = 0;
  if (mx > 0.f && mx < __builtin_huge_valf()) frexpf(mx, &e);
  const float s = ldexpf(1.f, -e);
  if (!live) return;
  halfx8 hi, lo;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float xs = v[i] * s;
    const _Float16 h = (_Float16)xs;
    hi[i] = h;
    lo[i] = (_Float16)(xs - (float)h);
  }
  *reinterpret_cast<halfx8*>(planes + row * (2 * FPAD) + grp * 8) = hi;
  *reinterpret_cast<halfx8*>(planes + row * (2 * FPAD) + FPAD + grp * 8) = lo;
  if (grp == 0) sx[row] = s;
}

// Centroid packing in two short launches. h3_cscale: per centroid (FPAD/8 lanes, 8 features each)
// max |c_i| and |c|^2 -> ur[chunk][0:CB) = u_c = |c|^2 / 2 (+inf for padding rows) and
// ur[chunk][CB:2CB) = r_c = 2^e (max |c_i| 2^-e in [0.5, 1); 1 for zero / padding rows), plus
// meta[1] = max_c max_i |c_i| and meta[2] = max_c u_c (float bits, atomicMax on zeroed words: valid
// for non-negative floats; used by the certified filter's error bound). u and r of one chunk are
// adjacent so ONE LDS-DMA instruction stages both. h3_pack_centroids: the packed image
//   image[chunk][cb][ks][hl][lane][8] (lane = h*32 + j, centroid chunk*CB + cb*32 + j,
//   features h*F2 + 8 ks .. +8) of c * s_c split into fp16 hi / lo.
template <int FPAD>
__global__ __launch_bounds__(256) void h3_cscale(const float* __restrict__ C, int k, int f, int64_t ldc, int kpad,
                                                 float* __restrict__ ur, float* __restrict__ meta,
                                                 unsigned* __restrict__ vimg) {
  constexpr int G8 = FPAD / 8;  // lanes per centroid (divides 64)
  constexpr int CB = H3Cfg<FPAD>::CB;
  // grid-stride over the kpad * G8 lanes (the loop bound is block-uniform, so every lane of a
  // wave takes part in each step's shuffles); the two maxima are reduced per block and posted
  // with ONE atomicMax pair per block - a pair per centroid serialised on two addresses (5.7 ms
  // for 1e6 rows, the KNN training set, 90 GB/s)
  const int64_t total = (int64_t)kpad * G8;
  float bmx = 0.f, bu = 0.f;
  for (int64_t t0 = (int64_t)blockIdx.x * 256; t0 < total; t0 += (int64_t)gridDim.x * 256) {
    const int64_t t = t0 + threadIdx.x;
    const int c = (int)(t / G8), g8 = (int)(t % G8);
    const bool live = c < k;
    float mx = 0.f, sq = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int fe = g8 * 8 + i;
      const float x = (live && fe < f) ? C[(int64_t)c * ldc + fe] : 0.f;
      mx = fmaxf(mx, fabsf(x));
      sq = fmaf(x, x, sq);
    }
#pragma unroll
    for (int o = 1; o < G8; o <<= 1) {
      mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      sq += __shfl_xor(sq, o, 64);
    }
    if (g8 != 0 || c >= kpad) continue;
    float* urc = ur + (int64_t)(c / CB) * 2 * CB + c % CB;
    // rank-1 A fragment of the -s_c u_c term (see h3_assign_p): lane j of tile c/32 holds its three
    // bf16 pieces in k-slots 0..2, lane j + 32 (k-slots 8..15) zeros
    unsigned* vc = vimg + ((int64_t)(c / 32) * 64 + c % 32) * 2;
    vc[64] = 0u;
    vc[65] = 0u;
    if (!live) {
      urc[0] = __builtin_huge_valf();
      urc[CB] = 1.f;
      vc[0] = 0xFF80u;  // -inf, 0
      vc[1] = 0u;
      continue;
    }
    int e = 0;
    if (mx > 0.f && mx < __builtin_huge_valf()) frexpf(mx, &e);
    urc[0] = 0.5f * sq;
    urc[CB] = ldexpf(1.f, e);
    {
      const float y = -ldexpf(0.5f * sq, -e);  // -s_c u_c, split into hi + mid + lo (24 bits)
      const unsigned hi = h3_bf16_rn(y);
      const float r1 = y - h3_bf16_f(hi);
      const unsigned mid = h3_bf16_rn(r1);
      const unsigned lo = h3_bf16_rn(r1 - h3_bf16_f(mid));
      vc[0] = hi | (mid << 16);
      vc[1] = lo;
    }
    if (mx > 0.f && mx < __builtin_huge_valf()) bmx = fmaxf(bmx, mx);
    if (sq > 0.f && sq < __builtin_huge_valf()) bu = fmaxf(bu, 0.5f * sq);
  }
  // block maxima (non-negative, so 0 is the identity) -> one atomicMax per word per block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    bmx = fmaxf(bmx, __shfl_xor(bmx, o, 64));
    bu = fmaxf(bu, __shfl_xor(bu, o, 64));
  }
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = bmx;
    red[1][wv] = bu;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bmx = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    bu = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
    if (bmx > 0.f) atomicMax(reinterpret_cast<unsigned int*>(meta + 1), __float_as_uint(bmx));
    if (bu > 0.f) atomicMax(reinterpret_cast<unsigned int*>(meta + 2), __float_as_uint(bu));
  }
}

// Grid of h3_cscale: one lane per 8 features of each padded centroid, at most 1024 blocks (a
// grid-stride loop covers the rest), so large point sets post few same-address atomics.
static inline unsigned h3_cscale_grid(int64_t kpad, int g8) {
  const int64_t b = (kpad * g8 + 255) / 256;
  return (unsigned)(b < 1024 ? (b > 0 ? b : 1) : 1024);
}

template <int FPAD>
__global__ __launch_bounds__(256) void h3_pack_centroids(const float* __restrict__ C, int k, int f, int64_t ldc,
                                                         int kpad, _Float16* __restrict__ image,
                                                         const float* __restrict__ ur) {
  using K = H3Cfg<FPAD>;
  constexpr int G8 = FPAD / 8;
  const int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (it >= (int64_t)kpad * G8) return;
  const int c = (int)(it / G8), g8 = (int)(it % G8);
  const int fe = g8 * 8;
  const float s = 1.f / ur[(int64_t)(c / K::CB) * 2 * K::CB + K::CB + c % K::CB];  // exact: a power of two
  halfx8 hi, lo;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = (c < k && fe + i < f) ? C[(int64_t)c * ldc + fe + i] * s : 0.f;
    const _Float16 h = (_Float16)x;
    hi[i] = h;
    lo[i] = (_Float16)(x - (float)h);
  }
  const int h = fe / K::F2, ks = (fe % K::F2) / 8;
  const int chunk = c / K::CB, cb = (c % K::CB) / 32, j = c % 32;
  const int lane = h * 32 + j;
  const int64_t base = ((((int64_t)chunk * (K::CB / 32) + cb) * K::KS + ks) * 2) * 64 * 8;
  *reinterpret_cast<halfx8*>(image + base + (int64_t)lane * 8) = hi;
  *reinterpret_cast<halfx8*>(image + base + 64 * 8 + (int64_t)lane * 8) = lo;
}

// the per-pair score of 2 adjacent accumulator values: s_x (x.c - |c|^2/2) = D r_c - s_x u_c.
// Scalar f32 ops on purpose (the file is built with -fno-slp-vectorize): a v_pk_fma_f32 /
// v_pk_mul_f32 issued beside MFMAs costs ~5x the issue slot of a scalar v_fma_f32 on gfx950, and
// this epilogue runs in the MFMA gaps.
__device__ __forceinline__ floatx2 h3_score2(floatx2 acc, floatx2 r, floatx2 u, floatx2 nsx) {
  floatx2 o;
  o[0] = fmaf(acc[0], r[0], nsx[0] * u[0]);
  o[1] = fmaf(acc[1], r[1], nsx[1] * u[1]);
  return o;
}

int h3_fpad(int f) { return f <= 16 ? 16 : f <= 32 ? 32 : f <= 64 ? 64 : f <= 128 ? 128 : -1; }

// sorted insertion into a lane's descending top-KN list (the kNN kernels)
template <int KN>
__device__ __forceinline__ void topk_insert(float (&tv)[KN], int (&ti)[KN], float v, int id) {
#pragma unroll
  for (int s = KN - 1; s >= 1; --s) {
    const bool ap = v > tv[s - 1];
    const bool ac = v > tv[s];
    tv[s] = ap ? tv[s - 1] : (ac ? v : tv[s]);
    ti[s] = ap ? ti[s - 1] : (ac ? id : ti[s]);
  }
  const bool a0 = v > tv[0];
  tv[0] = a0 ? v : tv[0];
  ti[0] = a0 ? id : ti[0];
}

}  // namespace

