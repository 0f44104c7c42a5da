// hipcc-flags: -fno-slp-vectorize
// K-means assignment on the FP16 matrix cores with a 3-term split ("f16x3"): ~fp32-GEMM accuracy
// at 16x the per-instruction MFMA rate of the f32-input MFMA (v_mfma_f32_32x32x16_f16: 16K MACs
// in 32 cycles/SIMD vs v_mfma_f32_32x32x2_f32: 2K MACs in 64).
//
// Points are scaled per row by a power of two s_x (max |x_i| in [0.5, 1)) and split once per fit
// into fp16 hi = fp16(x s_x), lo = fp16(x s_x - hi) ("planes", cached across Lloyd iterations by
// the caller).  Centroids get their OWN power-of-two scale s_c (max |c_i| s_c in [0.5, 1)) and are
// packed per iteration into the MFMA A-fragment image. Per (point, centroid):
//     D = hi_c.hi_x + hi_c.lo_x + lo_c.hi_x           (three MFMAs, fp32 accumulation)
//       = s_x s_c x.c  up to ~3 * 2^-22 relative per product term
//   argmin_c |c|^2 - 2 x.c  =  argmax_c  D r_c - s_x u_c,   r_c = 1 / s_c,  u_c = |c|^2 / 2
// (r_c is a power of two, so D r_c is exact). The per-centroid scale keeps every centroid's hi/lo
// split at full fp16 precision however different the centroid norms are: with one shared scale a
// centroid 2^-e smaller than the largest one had its lo term pushed into (or below) fp16's
// subnormal range, losing up to e bits of its own products. The epilogue is one packed multiply
// + one packed FMA per pair, a 16-way max per 32-centroid tile and a select that keeps the best
// tile's 16 values; the index is searched once per point at the end.
//
// Layout and orientation follow km_assign (kmeans.hip): centroids = A (rows), points = B
// (columns), the K dimension is permuted so lane half h owns features [h*F2, h*F2 + F2) of its
// point and reads them as 16-byte loads; the packed centroid image in LDS is read with
// conflict-free lane-linear ds_read_b128.
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

// Assignment kernel. A wave keeps NPB 32-point blocks (hi/lo fragments) in registers; the packed
// centroid image is staged chunk by chunk into LDS by LDS-DMA (global_load_lds_dwordx4: the image is
// stored in fragment order, so the copy is lane-linear). Software-pipelined: the argmax epilogue
// of tile t-1 (VALU) is issued in the same basic block as the MFMAs of tile t (ping-pong
// accumulators), and sched_group_barrier pins an MFMA / VALU interleave, so the epilogue fills
// the MFMA issue gaps instead of stalling the matrix pipe once per tile.
// Measured alternatives (tools/microbench/h3_bench.hip, n=12.5M, k=1024, f=64): register-staged
// double buffer 4.39 ms, unpipelined LDS-DMA 4.03 ms, this kernel 4.10 ms with 1 LDS buffer and
// 4.10 ms with 2 (DMA of chunk c+1 under chunk c: no gain, the loop is not load-latency bound).
//
// IND (the re-check pass of the certified filter below): the points are rows[0 .. *rcount) of the
// planes, and a grid of a few workgroups per CU strides over them (the count is only known on the
// device).
template <int FPAD, int NPB_ = 2, bool EPI = true, int MINB = 3, bool IND = false>
__global__ __launch_bounds__(256, MINB) void h3_assign_p(const _Float16* __restrict__ planes, const float* __restrict__ sxv,
                                                   int64_t n, const _Float16* __restrict__ image,
                                                   const float* __restrict__ u, const float* __restrict__ meta,
                                                   int nchunks, int* __restrict__ labels, float* __restrict__ mind,
                                                   const int* __restrict__ rows = nullptr,
                                                   const int* __restrict__ rcount = nullptr, int64_t rcap = 0) {
  using K = H3Cfg<FPAD, NPB_>;
  constexpr int F2 = K::F2, KS = K::KS, CB = K::CB, NPB = K::NPB, CHUNK_H = K::CHUNK_H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  // IND: rows in H3_AMB_SHARDS lists (h1_filter), list s = rows[s rcap ..), rcount[s] entries
  int spre[IND ? H3_AMB_SHARDS + 1 : 1];
  spre[0] = 0;
  if constexpr (IND) {
#pragma unroll
    for (int q = 0; q < H3_AMB_SHARDS; ++q) spre[q + 1] = spre[q] + rcount[q];
  }
  const int64_t cnt = IND ? (int64_t)spre[IND ? H3_AMB_SHARDS : 0] : n;
  for (int64_t blk = blockIdx.x; blk * K::PTS_PER_WG < cnt; blk += IND ? gridDim.x : cnt) {
  const int64_t pbase = blk * K::PTS_PER_WG + (int64_t)wave * (NPB * 32);

  halfx8 bhi[NPB][KS], blo[NPB][KS];
  bf16x8 bsx[NPB];
  float sx[NPB], nsx[NPB], xsq[NPB];
  int64_t prow[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int64_t idx = pbase + pb * 32 + j;
    const int64_t ci = idx < cnt ? idx : cnt - 1;
    int64_t row = ci;
    if constexpr (IND) {
      int q = 0;
#pragma unroll
      for (int t = 1; t < H3_AMB_SHARDS; ++t) q = ci >= spre[t] ? t : q;
      row = rows[q * rcap + (ci - spre[q])];
    }
    prow[pb] = idx < cnt ? row : -1;
    const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bhi[pb][ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
      blo[pb][ks] = *reinterpret_cast<const halfx8*>(pr + FPAD + 8 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xv = (float)bhi[pb][ks][i] + (float)blo[pb][ks][i];
        q = fmaf(xv, xv, q);
      }
    }
    sx[pb] = sxv[row];
    nsx[pb] = -sx[pb];
    xsq[pb] = q;
    // B fragment of the rank-1 term: s_x (a power of two: exact in bf16) in k-slots 0..2
    const unsigned sb = __float_as_uint(sx[pb]) >> 16;
    const u32x4 bw = {h ? 0u : (sb | (sb << 16)), h ? 0u : sb, 0u, 0u};
    bsx[pb] = __builtin_bit_cast(bf16x8, bw);
  }
  float best[NPB];
  int btile[NPB];
  float sv[NPB][16];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    best[pb] = -__builtin_huge_valf();
    btile[pb] = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[pb][r] = -__builtin_huge_valf();
  }

  constexpr int PIECES = CHUNK_H * 2 / 1024;  // 1 KB (64 lanes x 16 B) per DMA instruction
  // two chunk buffers: the epilogue of a chunk's last tile runs during the next chunk's first
  // tile and still reads its u/r from the previous buffer
  constexpr int VPIECES = CB * 16 / 1024;  // rank-1 fragments: 512 B per 32-centroid tile
  constexpr int BUF = CHUNK_H * 2 + CB * 8 + CB * 16;
  const unsigned* vimg = reinterpret_cast<const unsigned*>(meta + 4);
  floatx16 acc[2][NPB];
  const float* pu = nullptr;  // LDS u/r of the tile whose epilogue is pending
  int ptile = -1;
  auto epilogue = [&](const floatx16 (&ac)[NPB], const float* pu_, int tile) {
    // r of the tile straight from LDS (the chunk buffer is still live: see the loop); the
    // accumulator already holds s_c s_x (x.c - u_c) (rank-1 MFMA), so the score is ONE multiply
    floatx4 cr[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) cr[g] = *reinterpret_cast<const floatx4*>(pu_ + CB + 8 * g + 4 * h);
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      float w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = ac[pb][q] * cr[q >> 2][q & 3];
      float m = w[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) m = fmaxf(m, w[r]);
      const bool imp = m > best[pb];
      best[pb] = imp ? m : best[pb];
      btile[pb] = imp ? tile : btile[pb];
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[pb][r] = imp ? w[r] : sv[pb][r];
    }
  };
  for (int ch = 0; ch < nchunks; ++ch) {
    {
      const char* src = reinterpret_cast<const char*>(image + (int64_t)ch * CHUNK_H) + lane * 16;
      unsigned char* dst = smem + (ch & 1) * BUF;
#pragma unroll
      for (int pc = wave; pc < PIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(src + pc * 1024,
                                         (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, 0, 0);
      if (wave == 0 && lane < CB / 2)  // u and r of the chunk (adjacent)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(u + ch * 2 * CB) + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H * 2), 16, 0, 0);
#pragma unroll
      for (int pc = wave; pc < VPIECES; pc += 4)  // rank-1 fragments of the chunk's tiles
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(vimg) + (int64_t)ch * CB * 16 + pc * 1024 + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H * 2 + CB * 8 + pc * 1024),
                                         16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    const unsigned char* buf = smem + (ch & 1) * BUF;
    const _Float16* img = reinterpret_cast<const _Float16*>(buf);
    const float* ub = reinterpret_cast<const float*>(buf + CHUNK_H * 2);
    const unsigned* vb = reinterpret_cast<const unsigned*>(buf + CHUNK_H * 2 + CB * 8);
#pragma unroll
    for (int cb = 0; cb < CB / 32; ++cb) {
      const int cur = cb & 1;  // CB/32 is even: ping-pong slot is compile-time
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const _Float16* a = img + (((cb * KS + ks) * 2) * 64 + lane) * 8;
        const halfx8 ahi = *reinterpret_cast<const halfx8*>(a);
        const halfx8 alo = *reinterpret_cast<const halfx8*>(a + 64 * 8);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) {
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, blo[pb][ks], acc[cur][pb], 0, 0, 0);
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
        }
      }
      {
        // + s_x (-s_c u_c) as one bf16 MFMA (3 pieces x s_x, exact products, fp32 accumulation)
        const uint2 vv = *reinterpret_cast<const uint2*>(vb + (cb * 64 + lane) * 2);
        const u32x4 aw = {vv.x, vv.y, 0u, 0u};
        const bf16x8 av = __builtin_bit_cast(bf16x8, aw);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bsx[pb], acc[cur][pb], 0, 0, 0);
      }
      // epilogue of the previous tile (independent of the MFMAs above)
      if (ptile >= 0) epilogue(acc[cur ^ 1], pu, ptile);
      ptile = ch * (CB / 32) + cb;
      pu = ub + cb * 32;
#pragma unroll
      for (int i = 0; i < (3 * KS + 1) * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then up to 4 VALU
      }
    }
    __syncthreads();  // every wave is done with the buffer before the next chunk's DMA
  }
  if (ptile >= 0) epilogue(acc[((CB / 32) - 1) & 1], pu, ptile);

  int bidx[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    int bi = 15;
#pragma unroll
    for (int r = 14; r >= 0; --r) bi = sv[pb][r] == best[pb] ? r : bi;
    bidx[pb] = btile[pb] * 32 + (bi & 3) + 8 * (bi >> 2) + 4 * h;
  }
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const float ob = __shfl_xor(best[pb], 32, 64);
    const int oi = __shfl_xor(bidx[pb], 32, 64);
    const float xs = xsq[pb] + __shfl_xor(xsq[pb], 32, 64);
    if (ob > best[pb] || (ob == best[pb] && oi < bidx[pb])) {
      best[pb] = ob;
      bidx[pb] = oi;
    }
    const int64_t row = prow[pb];
    if (h == 0 && row >= 0) {
      labels[row] = bidx[pb];
      if (mind) {
        // |x|^2 + |c|^2 - 2 x.c = (xs_scaled / s_x^2) - 2 best / s_x
        const float isx = 1.f / sx[pb];
        mind[row] = fmaxf(xs * isx * isx - 2.f * best[pb] * isx, 0.f);
      }
    }
  }
  }  // point blocks
}

// Certified one-term filter ("h1"). Scores use hi_c . hi_x only (ONE MFMA per k-step instead of
// three), the kernel tracks each point's best AND runner-up score, and a point is assigned here
// only if its best score beats the runner-up by more than twice a rigorous bound E on the
// hi-only error; every other point is appended to `amb_rows` and re-run through the 3-term kernel
// (IND mode of h3_assign_p). In the scaled space (|x_s|_inf, |c_s|_inf < 1), with a, b the fp16
// rounding errors of x_s, c_s (|a_i| <= 2^-11 |x_s,i| or 2^-25 in fp16's subnormal range):
//   |x_s.c_s - hi_x.hi_c| <= sum |x_i b_i| + |a_i c_i| + |a_i b_i| <= 2^-10 (1 + 2^-11) |x_s| |c_s| + f 2^-24
// fp16 x fp16 products are exact in fp32; the fp32 accumulation, the fp32 |c|^2 and the epilogue
// FMA add <= (f + 2) 2^-24 (|x_s||c_s| + s_x u_max); f <= 128 gives
//   E = 1.01 * 2^-10 |x_s| c_max + 2^-16 (|x_s| c_max + s_x u_max) + 2^-16,
// with |x_s| bounded from the hi plane (|x_s| <= |hi_x| (1 + 2^-10)) and c_max = max_c |c_s|.
// The runner-up is exact without a per-value second-best update: per lane it is the larger of the
// second-largest TILE maximum (one med3 per tile) and the second-largest value of the best tile
// (whose 16 values are kept anyway to recover the index).
template <int FPAD, int NPB_ = 2, int MINB = 2>
__global__ __launch_bounds__(256, MINB) void h1_filter(const _Float16* __restrict__ planes, const float* __restrict__ sxv,
                                                 int64_t n, const _Float16* __restrict__ image,
                                                 const float* __restrict__ u, const float* __restrict__ meta,
                                                 int nchunks, int* __restrict__ labels, int* __restrict__ amb_rows,
                                                 int* __restrict__ amb_count, int64_t amb_cap) {
  using K = H3Cfg<FPAD, NPB_>;
  constexpr int F2 = K::F2, KS = K::KS, CB = K::CB, NPB = K::NPB, CHUNK_H = K::CHUNK_H;
  constexpr float NINF = -__builtin_huge_valf();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * K::PTS_PER_WG + (int64_t)wave * (NPB * 32);

  halfx8 bhi[NPB][KS];
  float nsx[NPB], hsq[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    int64_t row = pbase + pb * 32 + j;
    row = row < n ? row : n - 1;
    const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bhi[pb][ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) q = fmaf((float)bhi[pb][ks][i], (float)bhi[pb][ks][i], q);
    }
    nsx[pb] = -sxv[row];
    hsq[pb] = q;
  }
  float best[NPB], sec[NPB];
  int btile[NPB];
  float sv[NPB][16];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    best[pb] = NINF;
    sec[pb] = NINF;
    btile[pb] = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[pb][r] = NINF;
  }

  // only the hi half of every (cb, ks) fragment pair is staged: piece 2q of the chunk -> LDS q
  constexpr int PIECES = CHUNK_H * 2 / 1024 / 2;
  constexpr int BUF = CHUNK_H + CB * 8;  // two buffers, as in h3_assign_p
  floatx16 acc[2][NPB];
  const float* pu = nullptr;  // LDS u/r of the tile whose epilogue is pending
  int ptile = -1;
  auto epilogue = [&](const floatx16 (&ac)[NPB], const float* pu_, int tile) {
    // u and r of the tile straight from LDS (the chunk buffer is still live: see the loop)
    floatx4 cn[4], cr[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      cn[g] = *reinterpret_cast<const floatx4*>(pu_ + 8 * g + 4 * h);
      cr[g] = *reinterpret_cast<const floatx4*>(pu_ + CB + 8 * g + 4 * h);
    }
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      const floatx2 sx2 = {nsx[pb], nsx[pb]};
      float w[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const floatx2 c2 = {cn[q >> 1][(2 * q) & 3], cn[q >> 1][(2 * q + 1) & 3]};
        const floatx2 rc2 = {cr[q >> 1][(2 * q) & 3], cr[q >> 1][(2 * q + 1) & 3]};
        const floatx2 a2 = {ac[pb][2 * q], ac[pb][2 * q + 1]};
        const floatx2 r2 = h3_score2(a2, rc2, c2, sx2);
        w[2 * q] = r2[0];
        w[2 * q + 1] = r2[1];
      }
      float m = w[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) m = fmaxf(m, w[r]);
      sec[pb] = __builtin_amdgcn_fmed3f(best[pb], sec[pb], m);
      const bool imp = m > best[pb];
      best[pb] = imp ? m : best[pb];
      btile[pb] = imp ? tile : btile[pb];
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[pb][r] = imp ? w[r] : sv[pb][r];
    }
  };
  for (int ch = 0; ch < nchunks; ++ch) {
    {
      const char* src = reinterpret_cast<const char*>(image + (int64_t)ch * CHUNK_H) + lane * 16;
      unsigned char* dst = smem + (ch & 1) * BUF;
#pragma unroll
      for (int pc = wave; pc < PIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(src + 2 * pc * 1024,
                                         (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, 0, 0);
      if (wave == 0 && lane < CB / 2)  // u and r of the chunk (adjacent)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(u + ch * 2 * CB) + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    const _Float16* img = reinterpret_cast<const _Float16*>(smem + (ch & 1) * BUF);
    const float* ub = reinterpret_cast<const float*>(smem + (ch & 1) * BUF + CHUNK_H);
#pragma unroll
    for (int cb = 0; cb < CB / 32; ++cb) {
      const int cur = cb & 1;
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const halfx8 ahi = *reinterpret_cast<const halfx8*>(img + ((cb * KS + ks) * 64 + lane) * 8);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
      }
      if (ptile >= 0) epilogue(acc[cur ^ 1], pu, ptile);
      ptile = ch * (CB / 32) + cb;
      pu = ub + cb * 32;
#pragma unroll
      for (int i = 0; i < KS * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);  // then up to 12 VALU
      }
    }
    __syncthreads();
  }
  if (ptile >= 0) epilogue(acc[((CB / 32) - 1) & 1], pu, ptile);

  const float umax = meta[2];
  const float cmax = sqrtf(2.f * umax);  // max_c |c|_2 (unscaled: scores are s_x (x.c - |c|^2/2))
  // uncertain points are appended to one of H3_AMB_SHARDS lists (shard = blockIdx % shards, rows
  // of shard s at amb_rows[s * cap ..), count amb_count[s]) with ONE atomic per workgroup: a
  // wave-level atomic on a single counter serialised ~350K same-address adds on diffuse data
  // (the filter took 4.1 ms there vs 2.3 ms on clustered data with nothing to append)
  __shared__ int wcnt[4 * NPB + 1];
  unsigned long long am[NPB];
  int64_t arow[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    float t1 = NINF, t2 = NINF;
    int bi = 15;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      t2 = __builtin_amdgcn_fmed3f(t1, t2, sv[pb][r]);
      t1 = fmaxf(t1, sv[pb][r]);
    }
#pragma unroll
    for (int r = 14; r >= 0; --r) bi = sv[pb][r] == best[pb] ? r : bi;
    int bidx = btile[pb] * 32 + (bi & 3) + 8 * (bi >> 2) + 4 * h;
    float s2 = fmaxf(sec[pb], t2);
    const float ob = __shfl_xor(best[pb], 32, 64);
    const float os = __shfl_xor(s2, 32, 64);
    const int oi = __shfl_xor(bidx, 32, 64);
    const float xn = sqrtf(hsq[pb] + __shfl_xor(hsq[pb], 32, 64)) * (1.f + 0x1p-10f);
    s2 = fmaxf(fminf(best[pb], ob), fmaxf(s2, os));
    float b = best[pb];
    if (ob > b || (ob == b && oi < bidx)) {
      b = ob;
      bidx = oi;
    }
    const float xc = xn * cmax;
    const float E = 1.01f * 0x1p-10f * xc + 0x1p-16f * (xc - nsx[pb] * umax) + 0x1p-15f * cmax;
    const int64_t row = pbase + pb * 32 + j;
    const bool live = h == 0 && row < n;
    const bool amb = live && !(b - s2 > 2.f * E);
    if (live) labels[row] = bidx;
    am[pb] = __ballot(amb);
    arow[pb] = row;
    if (lane == 0) wcnt[wave * NPB + pb] = (int)__popcll(am[pb]);
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int q = 0; q < 4 * NPB; ++q) {
      const int c = wcnt[q];
      wcnt[q] = run;
      run += c;
    }
    wcnt[4 * NPB] = run ? atomicAdd(amb_count + blockIdx.x % H3_AMB_SHARDS, run) : 0;
  }
  __syncthreads();
  int* const rows_s = amb_rows + (int64_t)(blockIdx.x % H3_AMB_SHARDS) * amb_cap;
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb)
    if ((am[pb] >> lane) & 1ull)
      rows_s[wcnt[4 * NPB] + wcnt[wave * NPB + pb] + (int)__popcll(am[pb] & below)] = (int)arow[pb];
}


// k nearest "centroids" (KNN: the training points) of every point, the same fp16x3 scores as the
// assignment (score = x.c - |c|^2/2 in the scaled space, larger = nearer) with a running top-KN
// list per lane instead of a running max: no n x m distance matrix. A lane keeps its KN best
// (score, index) sorted in registers; a tile's 16 candidates are only inserted where they beat
// the lane's current KN-th best (after the first tiles nearly never: ~KN ln(m) insertions per
// point), so the epilogue is a max + compare per tile in the common case. The two lane halves
// (disjoint centroid halves of the same point) merge their lists at the end. Output: KN squared
// distances (ascending) and int32 indices per point; -1 / +inf where fewer than KN exist.
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

template <int FPAD, int KN>
__global__ __launch_bounds__(256, 2) void h3_topk(const _Float16* __restrict__ planes, const float* __restrict__ sxv,
                                                  int64_t n, const _Float16* __restrict__ image,
                                                  const float* __restrict__ u, const float* __restrict__ meta,
                                                  int nchunks, int cps, int kout, float* __restrict__ dist,
                                                  int* __restrict__ idx) {
  using K = H3Cfg<FPAD, 1>;
  constexpr int F2 = K::F2, KS = K::KS, CB = K::CB, CHUNK_H = K::CHUNK_H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t p = (int64_t)blockIdx.x * K::PTS_PER_WG + wave * 32 + j;
  const int64_t row = p < n ? p : n - 1;

  halfx8 bhi[KS], blo[KS];
  const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
  float q = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bhi[ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
    blo[ks] = *reinterpret_cast<const halfx8*>(pr + FPAD + 8 * ks);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xv = (float)bhi[ks][i] + (float)blo[ks][i];
      q = fmaf(xv, xv, q);
    }
  }
  const float sx = sxv[row];
  const float nsx = -sx;
  float tv[KN];
  int ti[KN];
#pragma unroll
  for (int s = 0; s < KN; ++s) {
    tv[s] = -__builtin_huge_valf();
    ti[s] = -1;
  }
  constexpr int PIECES = CHUNK_H * 2 / 1024;
  // blockIdx.y: a range of centroid chunks (split over the centroids when the points alone cannot
  // fill the GPU); partial lists go to slice blockIdx.y of the outputs
  const int ch0 = blockIdx.y * cps;
  const int ch1 = ch0 + cps < nchunks ? ch0 + cps : nchunks;
  dist += (int64_t)blockIdx.y * n * kout;
  idx += (int64_t)blockIdx.y * n * kout;
  for (int ch = ch0; ch < ch1; ++ch) {
    {
      const char* src = reinterpret_cast<const char*>(image + (int64_t)ch * CHUNK_H) + lane * 16;
#pragma unroll
      for (int pc = wave; pc < PIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(src + pc * 1024,
                                         (__attribute__((address_space(3))) void*)(smem + pc * 1024), 16, 0, 0);
      if (wave == 0 && lane < CB / 2)  // u and r of the chunk (adjacent)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(u + ch * 2 * CB) + lane * 16,
                                         (__attribute__((address_space(3))) void*)(smem + CHUNK_H * 2), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    const _Float16* img = reinterpret_cast<const _Float16*>(smem);
    const float* ub = reinterpret_cast<const float*>(smem + CHUNK_H * 2);
#pragma unroll 2
    for (int cb = 0; cb < CB / 32; ++cb) {
      floatx16 acc = (floatx16)(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const _Float16* a = img + (((cb * KS + ks) * 2) * 64 + lane) * 8;
        const halfx8 ahi = *reinterpret_cast<const halfx8*>(a);
        const halfx8 alo = *reinterpret_cast<const halfx8*>(a + 64 * 8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bhi[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, blo[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bhi[ks], acc, 0, 0, 0);
      }
      float w[16];
      float m = -__builtin_huge_valf();
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const floatx4 cn = *reinterpret_cast<const floatx4*>(ub + cb * 32 + 8 * g + 4 * h);
        const floatx4 cr = *reinterpret_cast<const floatx4*>(ub + CB + cb * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          w[4 * g + i] = fmaf(acc[4 * g + i], cr[i], nsx * cn[i]);
          m = fmaxf(m, w[4 * g + i]);
        }
      }
      if (m > tv[KN - 1]) {
        const int tbase = (ch * (CB / 32) + cb) * 32 + 4 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (w[r] > tv[KN - 1]) topk_insert<KN>(tv, ti, w[r], tbase + (r & 3) + 8 * (r >> 2));
      }
    }
    __syncthreads();
  }
  // merge the partner half's list (disjoint candidates) into lane half 0
#pragma unroll
  for (int s = 0; s < KN; ++s) {
    const float ov = __shfl_xor(tv[s], 32, 64);
    const int oi = __shfl_xor(ti[s], 32, 64);
    if (h == 0 && ov > tv[KN - 1]) topk_insert<KN>(tv, ti, ov, oi);
  }
  const float xs = q + __shfl_xor(q, 32, 64);  // all lanes: a shuffle from an inactive lane is undefined
  if (h == 0 && p < n) {
    const float isx = 1.f / sx;
#pragma unroll
    for (int s = 0; s < KN; ++s)
      if (s < kout) {
        const bool ok = ti[s] >= 0;
        dist[p * kout + s] = ok ? fmaxf(xs * isx * isx - 2.f * tv[s] * isx, 0.f) : __builtin_huge_valf();
        idx[p * kout + s] = ti[s];
      }
  }
}

// Pipelined top-k ("p"): the assignment kernel's structure (h3_assign_p) with a top-k epilogue.
//  * the -s_x s_c u_c term rides in the accumulator as one rank-1 bf16 MFMA per tile, so a score
//    is ONE multiply (acc * r_c) instead of an FMA + a multiply with two LDS vectors per tile;
//  * ping-pong accumulators: the scores / tile maximum / threshold test of tile t-1 are VALU issued
//    in the MFMA gaps of tile t (sched_group_barrier interleave);
//  * the rare insertion (a tile value beating a lane's KN-th best) runs after the tile's MFMAs,
//    only when some lane of the wave needs it (__any), from the 16 stashed scores;
//  * two LDS chunk buffers (the last tile's epilogue reads the previous buffer's r values).
// Round 3's h3_topk ran at 50 % MFMA-busy with 4.7 VALU per MFMA (profiles/pmc_r03.md).
template <int FPAD, int KN, int NPB_>
__global__ __launch_bounds__(256, 2) void h3_topk_p(const _Float16* __restrict__ planes, const float* __restrict__ sxv,
                                                    int64_t n, const _Float16* __restrict__ image,
                                                    const float* __restrict__ u, const float* __restrict__ meta,
                                                    int nchunks, int cps, int kout, float* __restrict__ dist,
                                                    int* __restrict__ idx) {
  using K = H3Cfg<FPAD, NPB_>;
  constexpr int F2 = K::F2, KS = K::KS, CB = K::CB, NPB = K::NPB, CHUNK_H = K::CHUNK_H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * K::PTS_PER_WG + (int64_t)wave * (NPB * 32);

  halfx8 bhi[NPB][KS], blo[NPB][KS];
  bf16x8 bsx[NPB];
  float sx[NPB], xsq[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int64_t pi = pbase + pb * 32 + j;
    const int64_t row = pi < n ? pi : n - 1;
    const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bhi[pb][ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
      blo[pb][ks] = *reinterpret_cast<const halfx8*>(pr + FPAD + 8 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xv = (float)bhi[pb][ks][i] + (float)blo[pb][ks][i];
        q = fmaf(xv, xv, q);
      }
    }
    sx[pb] = sxv[row];
    xsq[pb] = q;
    const unsigned sb = __float_as_uint(sx[pb]) >> 16;  // s_x: a power of two, exact in bf16
    const u32x4 bw = {h ? 0u : (sb | (sb << 16)), h ? 0u : sb, 0u, 0u};
    bsx[pb] = __builtin_bit_cast(bf16x8, bw);
  }
  float tv[NPB][KN];
  int ti[NPB][KN];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
    for (int s = 0; s < KN; ++s) {
      tv[pb][s] = -__builtin_huge_valf();
      ti[pb][s] = -1;
    }
  const int ch0 = blockIdx.y * cps;
  const int ch1 = ch0 + cps < nchunks ? ch0 + cps : nchunks;
  dist += (int64_t)blockIdx.y * n * kout;
  idx += (int64_t)blockIdx.y * n * kout;

  constexpr int PIECES = CHUNK_H * 2 / 1024;
  constexpr int VPIECES = CB * 16 / 1024;
  constexpr int BUF = CHUNK_H * 2 + CB * 8 + CB * 16;
  const unsigned* vimg = reinterpret_cast<const unsigned*>(meta + 4);
  floatx16 acc[2][NPB];
  float w[NPB][16];
  bool need = false;
  const float* pu = nullptr;
  int ptile = -1;
  // scores of the pending tile, its maximum against each lane's current KN-th best (no branch)
  auto epilogue = [&](const floatx16 (&ac)[NPB], const float* pu_) {
    floatx4 cr[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) cr[g] = *reinterpret_cast<const floatx4*>(pu_ + CB + 8 * g + 4 * h);
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
#pragma unroll
      for (int q = 0; q < 16; ++q) w[pb][q] = ac[pb][q] * cr[q >> 2][q & 3];
      float m = w[pb][0];
#pragma unroll
      for (int r = 1; r < 16; ++r) m = fmaxf(m, w[pb][r]);
      need |= m > tv[pb][KN - 1];
    }
  };
  auto insert = [&](int tile) {
    if (__builtin_amdgcn_ballot_w64(need) == 0ull) return;  // wave-uniform: usually nobody
    const int tbase = tile * 32 + 4 * h;
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (w[pb][r] > tv[pb][KN - 1]) topk_insert<KN>(tv[pb], ti[pb], w[pb][r], tbase + (r & 3) + 8 * (r >> 2));
    need = false;
  };
  for (int ch = ch0; ch < ch1; ++ch) {
    {
      const char* src = reinterpret_cast<const char*>(image + (int64_t)ch * CHUNK_H) + lane * 16;
      unsigned char* dst = smem + (ch & 1) * BUF;
#pragma unroll
      for (int pc = wave; pc < PIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(src + pc * 1024,
                                         (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, 0, 0);
      if (wave == 0 && lane < CB / 2)  // u and r of the chunk (adjacent)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(u + ch * 2 * CB) + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H * 2), 16, 0, 0);
#pragma unroll
      for (int pc = wave; pc < VPIECES; pc += 4)  // rank-1 fragments of the chunk's tiles
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(vimg) + (int64_t)ch * CB * 16 + pc * 1024 + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H * 2 + CB * 8 + pc * 1024),
                                         16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    const unsigned char* buf = smem + (ch & 1) * BUF;
    const _Float16* img = reinterpret_cast<const _Float16*>(buf);
    const float* ub = reinterpret_cast<const float*>(buf + CHUNK_H * 2);
    const unsigned* vb = reinterpret_cast<const unsigned*>(buf + CHUNK_H * 2 + CB * 8);
#pragma unroll
    for (int cb = 0; cb < CB / 32; ++cb) {
      const int cur = cb & 1;  // CB/32 is even: ping-pong slot is compile-time
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const _Float16* a = img + (((cb * KS + ks) * 2) * 64 + lane) * 8;
        const halfx8 ahi = *reinterpret_cast<const halfx8*>(a);
        const halfx8 alo = *reinterpret_cast<const halfx8*>(a + 64 * 8);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) {
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, blo[pb][ks], acc[cur][pb], 0, 0, 0);
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
        }
      }
      {
        const uint2 vv = *reinterpret_cast<const uint2*>(vb + (cb * 64 + lane) * 2);
        const u32x4 aw = {vv.x, vv.y, 0u, 0u};
        const bf16x8 av = __builtin_bit_cast(bf16x8, aw);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bsx[pb], acc[cur][pb], 0, 0, 0);
      }
      if (ptile >= 0) epilogue(acc[cur ^ 1], pu);
#pragma unroll
      for (int i = 0; i < (3 * KS + 1) * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then up to 4 VALU
      }
      if (ptile >= 0) insert(ptile);
      ptile = ch * (CB / 32) + cb;
      pu = ub + cb * 32;
    }
    __syncthreads();  // every wave is done with the buffer before the chunk after next is staged
  }
  if (ptile >= 0) {
    epilogue(acc[((CB / 32) - 1) & 1], pu);
    insert(ptile);
  }
  // merge the partner half's list (disjoint candidates) into lane half 0
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
#pragma unroll
    for (int s = 0; s < KN; ++s) {
      const float ov = __shfl_xor(tv[pb][s], 32, 64);
      const int oi = __shfl_xor(ti[pb][s], 32, 64);
      if (h == 0 && ov > tv[pb][KN - 1]) topk_insert<KN>(tv[pb], ti[pb], ov, oi);
    }
    const float xs = xsq[pb] + __shfl_xor(xsq[pb], 32, 64);
    const int64_t pi = pbase + pb * 32 + j;
    if (h == 0 && pi < n) {
      const float isx = 1.f / sx[pb];
#pragma unroll
      for (int s = 0; s < KN; ++s)
        if (s < kout) {
          const bool ok = ti[pb][s] >= 0;
          dist[pi * kout + s] = ok ? fmaxf(xs * isx * isx - 2.f * tv[pb][s] * isx, 0.f) : __builtin_huge_valf();
          idx[pi * kout + s] = ti[pb][s];
        }
    }
  }
}

// Certified one-term top-k ("h1"), the kNN form of h1_filter: scores from hi_c . hi_x only (ONE
// MFMA per k-step instead of three) plus the exact rank-1 u term, each within E of the fp32 score
// (E: h1_filter's bound). A lane keeps its KP best approximate scores and `rej`, the largest score
// it let go (rejected or evicted). After the halves merge, a point is CERTIFIED when
//     rej < a_KN - 2 E          (a_KN = the KN-th best approximate score in the list):
// then every candidate outside the list is, exactly, below KN candidates inside it, so the true
// top-KN is a subset of the KP-list, which the caller rescores exactly. Uncertain points are
// flagged (cert = 0) and re-run through the 3-term kernel by the caller.
// Output per point: KP approximate squared distances (ascending) and int32 indices, cert flag.
template <int KP>
__device__ __forceinline__ void topk_insert_ev(float (&tv)[KP], int (&ti)[KP], float v, int id, float& rej) {
  rej = fmaxf(rej, tv[KP - 1]);  // the evicted last entry (-inf while the list is not full)
  topk_insert<KP>(tv, ti, v, id);
}

// KH: list length per lane half (each half sees half of the rows of C); the two half lists are
// merged into the output list of 16. Measured (bench knn, 1e6 x 1e6 x 128): KH = 16 -> 373 ms +
// 10.8 % of the queries re-checked (81 ms); KH = 8 -> 350 ms but 32.7 % re-checked (222 ms).
// The insertions, not the MFMAs, bound this kernel (7-9 VALU per MFMA): a lane whose tile beats
// its threshold makes the whole wave run the insertion. Parking such tiles in LDS and draining
// them for all lanes together (2 parked tiles per lane) was 5x SLOWER: a drain runs the union of
// the lanes' insertion positions, so batching sparse, uncorrelated insertions does not pay.
// KO: output candidates per point (16: the two half lists merged into 16, what the merge lets go
// raises rej; 32: both half lists kept whole, rej = the halves' own - a wider certification margin,
// so fewer queries fall back to the 3-term kernel, for twice the rescoring input).
template <int FPAD, int KH, int KN, int NPB_, int KO_ = 16>
__global__ __launch_bounds__(256, 2) void h1_topk(const _Float16* __restrict__ planes, const float* __restrict__ sxv,
                                                  int64_t n, const _Float16* __restrict__ image,
                                                  const float* __restrict__ u, const float* __restrict__ meta,
                                                  int nchunks, float* __restrict__ dist, int* __restrict__ idx,
                                                  unsigned char* __restrict__ cert) {
  using K = H3Cfg<FPAD, NPB_>;
  constexpr int F2 = K::F2, KS = K::KS, CB = K::CB, NPB = K::NPB, CHUNK_H = K::CHUNK_H;
  constexpr float NINF = -__builtin_huge_valf();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * K::PTS_PER_WG + (int64_t)wave * (NPB * 32);

  halfx8 bhi[NPB][KS];
  bf16x8 bsx[NPB];
  float sx[NPB], hsq[NPB], xsq[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int64_t pi = pbase + pb * 32 + j;
    const int64_t row = pi < n ? pi : n - 1;
    const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
    float q = 0.f, q3 = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bhi[pb][ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
      const halfx8 lo = *reinterpret_cast<const halfx8*>(pr + FPAD + 8 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float hv = (float)bhi[pb][ks][i];
        q = fmaf(hv, hv, q);
        const float xv = hv + (float)lo[i];
        q3 = fmaf(xv, xv, q3);
      }
    }
    sx[pb] = sxv[row];
    hsq[pb] = q;
    xsq[pb] = q3;
    const unsigned sb = __float_as_uint(sx[pb]) >> 16;
    const u32x4 bw = {h ? 0u : (sb | (sb << 16)), h ? 0u : sb, 0u, 0u};
    bsx[pb] = __builtin_bit_cast(bf16x8, bw);
  }
  constexpr int KO = KO_;  // output candidates per point
  float tv[NPB][KH], rej[NPB];
  int ti[NPB][KH];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    rej[pb] = NINF;
#pragma unroll
    for (int s2 = 0; s2 < KH; ++s2) {
      tv[pb][s2] = NINF;
      ti[pb][s2] = -1;
    }
  }
  // only the hi half of every (cb, ks) fragment pair is staged (piece 2q of the chunk -> LDS q)
  constexpr int PIECES = CHUNK_H * 2 / 1024 / 2;
  constexpr int VPIECES = CB * 16 / 1024;
  constexpr int BUF = CHUNK_H + CB * 8 + CB * 16;
  const unsigned* vimg = reinterpret_cast<const unsigned*>(meta + 4);
  floatx16 acc[2][NPB];
  float w[NPB][16];
  bool need = false;
  const float* pu = nullptr;
  int ptile = -1;
  auto epilogue = [&](const floatx16 (&ac)[NPB], const float* pu_) {
    floatx4 cr[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) cr[g] = *reinterpret_cast<const floatx4*>(pu_ + CB + 8 * g + 4 * h);
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
#pragma unroll
      for (int q = 0; q < 16; ++q) w[pb][q] = ac[pb][q] * cr[q >> 2][q & 3];
      float m = w[pb][0];
#pragma unroll
      for (int r = 1; r < 16; ++r) m = fmaxf(m, w[pb][r]);
      const bool nd = m > tv[pb][KH - 1];
      rej[pb] = nd ? rej[pb] : fmaxf(rej[pb], m);  // the whole tile is let go
      need |= nd;
    }
  };
  auto insert = [&](int tile) {
    if (__builtin_amdgcn_ballot_w64(need) == 0ull) return;
    const int tbase = tile * 32 + 4 * h;
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (w[pb][r] > tv[pb][KH - 1])
          topk_insert_ev<KH>(tv[pb], ti[pb], w[pb][r], tbase + (r & 3) + 8 * (r >> 2), rej[pb]);
        else
          rej[pb] = fmaxf(rej[pb], w[pb][r]);
      }
    need = false;
  };
  for (int ch = 0; ch < nchunks; ++ch) {
    {
      const char* src = reinterpret_cast<const char*>(image + (int64_t)ch * CHUNK_H) + lane * 16;
      unsigned char* dst = smem + (ch & 1) * BUF;
#pragma unroll
      for (int pc = wave; pc < PIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(src + 2 * pc * 1024,
                                         (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, 0, 0);
      if (wave == 0 && lane < CB / 2)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(u + ch * 2 * CB) + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H), 16, 0, 0);
#pragma unroll
      for (int pc = wave; pc < VPIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(vimg) + (int64_t)ch * CB * 16 + pc * 1024 + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK_H + CB * 8 + pc * 1024),
                                         16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    const unsigned char* buf = smem + (ch & 1) * BUF;
    const _Float16* img = reinterpret_cast<const _Float16*>(buf);
    const float* ub = reinterpret_cast<const float*>(buf + CHUNK_H);
    const unsigned* vb = reinterpret_cast<const unsigned*>(buf + CHUNK_H + CB * 8);
#pragma unroll
    for (int cb = 0; cb < CB / 32; ++cb) {
      const int cur = cb & 1;
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const halfx8 ahi = *reinterpret_cast<const halfx8*>(img + ((cb * KS + ks) * 64 + lane) * 8);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
      }
      {
        const uint2 vv = *reinterpret_cast<const uint2*>(vb + (cb * 64 + lane) * 2);
        const u32x4 aw = {vv.x, vv.y, 0u, 0u};
        const bf16x8 av = __builtin_bit_cast(bf16x8, aw);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bsx[pb], acc[cur][pb], 0, 0, 0);
      }
      if (ptile >= 0) epilogue(acc[cur ^ 1], pu);
#pragma unroll
      for (int i = 0; i < (KS + 1) * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);  // then up to 12 VALU
      }
      if (ptile >= 0) insert(ptile);
      ptile = ch * (CB / 32) + cb;
      pu = ub + cb * 32;
    }
    __syncthreads();
  }
  if (ptile >= 0) {
    epilogue(acc[((CB / 32) - 1) & 1], pu);
    insert(ptile);
  }
  const float umax = meta[2];
  const float cmax = sqrtf(2.f * umax);
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    // merge the two half lists (disjoint candidates) into the output list of KO: whatever the
    // merge lets go raises rej
    float mv[KO];
    int mi[KO];
#pragma unroll
    for (int s2 = 0; s2 < KO; ++s2) {
      mv[s2] = s2 < KH ? tv[pb][s2 < KH ? s2 : 0] : NINF;
      mi[s2] = s2 < KH ? ti[pb][s2 < KH ? s2 : 0] : -1;
    }
#pragma unroll
    for (int s2 = KO; s2 < KH; ++s2) rej[pb] = fmaxf(rej[pb], tv[pb][s2]);
    float orj = __shfl_xor(rej[pb], 32, 64);
#pragma unroll
    for (int s2 = 0; s2 < KH; ++s2) {
      const float ov = __shfl_xor(tv[pb][s2], 32, 64);
      const int oi = __shfl_xor(ti[pb][s2], 32, 64);
      if (h == 0) {
        if (ov > mv[KO - 1]) topk_insert_ev<KO>(mv, mi, ov, oi, rej[pb]);
        else orj = fmaxf(orj, ov);
      }
    }
    rej[pb] = fmaxf(rej[pb], orj);
    const float xn = sqrtf(hsq[pb] + __shfl_xor(hsq[pb], 32, 64)) * (1.f + 0x1p-10f);
    const float xs = xsq[pb] + __shfl_xor(xsq[pb], 32, 64);
    const float xc = xn * cmax;
    const float E = 1.01f * 0x1p-10f * xc + 0x1p-16f * (xc + sx[pb] * umax) + 0x1p-15f * cmax;
    const int64_t pi = pbase + pb * 32 + j;
    if (h == 0 && pi < n) {
      const float isx = 1.f / sx[pb];
#pragma unroll
      for (int s2 = 0; s2 < KO; ++s2) {
        const bool ok = mi[s2] >= 0;
        dist[pi * KO + s2] = ok ? fmaxf(xs * isx * isx - 2.f * mv[s2] * isx, 0.f) : __builtin_huge_valf();
        idx[pi * KO + s2] = mi[s2];
      }
      cert[pi] = (mi[KN - 1] >= 0 && rej[pb] < mv[KN - 1] - 2.f * E) ? 1 : 0;
    }
  }
}

// Resident-centroid assignment ("r"): ONE workgroup per CU (NW waves) stages up to RC centroid
// chunks into LDS once (128 KB: 512 centroids at f = 64) and its waves then stream point blocks
// through them with no further barrier or staging; per-wave point blocks are independent. k above
// the resident capacity runs in phases over the centroid chunks, carrying each point's running
// best (value, index) through global memory (the planes are re-read once per phase). Compared with
// h3_assign_p (a workgroup per 256 points re-staging all k centroids chunk by chunk behind a
// barrier), this removes the per-chunk DMA + barrier and the per-workgroup start-up: 2.27 vs
// 2.52 ms at k = 512, 1.24 vs 1.39 ms at k = 200 (n = 12.5M, f = 64,
// tools/microbench/resident_bench.py). In phases (k = 1024) it is no faster (4.32-4.42 vs 4.39 ms
// alone, 5.28 vs 5.07 ms per full Lloyd step), so callers use it where the centroids fit. A
// 16-wave NPB = 1 variant (4 waves/SIMD) was no faster either (4.45 ms): the loop is bound by the
// MFMA + epilogue issue, not by latency.
// first: no carried state; last: write labels (+ mind) instead of the carried state.
// SGV > 0 pins an MFMA / SGV-VALU interleave with sched_group_barrier (measured 4: 4.60 ms, none
// or 8: 4.32 ms at k = 1024; default none).
template <int FPAD, int NPB_, int NW, int SGV = 0>
__global__ __launch_bounds__(NW * 64, 1) void h3_assign_r(const _Float16* __restrict__ planes,
                                                          const float* __restrict__ sxv, int64_t n,
                                                          const _Float16* __restrict__ image,
                                                          const float* __restrict__ u, const float* __restrict__ meta,
                                                          int ch0, int nch, int first, int last,
                                                          float* __restrict__ pbest, int* __restrict__ pidx,
                                                          int* __restrict__ labels, float* __restrict__ mind) {
  using K = H3Cfg<FPAD, NPB_>;
  constexpr int F2 = K::F2, KS = K::KS, CB = K::CB, NPB = K::NPB, CHUNK_H = K::CHUNK_H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  // ---- stage this phase's chunks (image by LDS-DMA, u by plain loads), once
  {
    const char* src = reinterpret_cast<const char*>(image + (int64_t)ch0 * CHUNK_H) + lane * 16;
    const int pieces = nch * (CHUNK_H * 2 / 1024);
    for (int pc = wave; pc < pieces; pc += NW)
      __builtin_amdgcn_global_load_lds(src + (int64_t)pc * 1024,
                                       (__attribute__((address_space(3))) void*)(smem + pc * 1024), 16, 0, 0);
    float* us = reinterpret_cast<float*>(smem + (size_t)nch * CHUNK_H * 2);
    for (int e = tid; e < nch * 2 * CB; e += NW * 64) us[e] = u[(int64_t)ch0 * 2 * CB + e];
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  const float* ubase = reinterpret_cast<const float*>(smem + (size_t)nch * CHUNK_H * 2);

  for (int64_t blk = (int64_t)blockIdx.x * NW + wave; blk * (NPB * 32) < n; blk += (int64_t)gridDim.x * NW) {
    const int64_t pbase = blk * (NPB * 32);
    halfx8 bhi[NPB][KS], blo[NPB][KS];
    float sx[NPB], nsx[NPB], xsq[NPB];
    int64_t prow[NPB];
    float best[NPB];
    int btile[NPB], pin[NPB];
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      const int64_t idx = pbase + pb * 32 + j;
      const int64_t row = idx < n ? idx : n - 1;
      prow[pb] = idx < n ? row : -1;
      const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
      float q = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bhi[pb][ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
        blo[pb][ks] = *reinterpret_cast<const halfx8*>(pr + FPAD + 8 * ks);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xv = (float)bhi[pb][ks][i] + (float)blo[pb][ks][i];
          q = fmaf(xv, xv, q);
        }
      }
      sx[pb] = sxv[row];
      nsx[pb] = -sx[pb];
      xsq[pb] = q;
      // carried best of the earlier phases (lower centroid indices win ties: strict > below)
      best[pb] = first ? -__builtin_huge_valf() : pbest[row];
      pin[pb] = first ? 0 : pidx[row];
      btile[pb] = -1;
    }
    float sv[NPB][16];
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[pb][r] = -__builtin_huge_valf();

    floatx16 acc[2][NPB];
    const float* pu = nullptr;  // LDS u/r of the tile whose epilogue is pending
    int ptile = -1;
    auto epilogue = [&](const floatx16 (&ac)[NPB], const float* pu_, int tile) {
    // u and r of the tile straight from LDS (the chunk buffer is still live: see the loop)
    floatx4 cn[4], cr[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      cn[g] = *reinterpret_cast<const floatx4*>(pu_ + 8 * g + 4 * h);
      cr[g] = *reinterpret_cast<const floatx4*>(pu_ + CB + 8 * g + 4 * h);
    }
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) {
        const floatx2 sx2 = {nsx[pb], nsx[pb]};
        float w[16];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const floatx2 c2 = {cn[q >> 1][(2 * q) & 3], cn[q >> 1][(2 * q + 1) & 3]};
          const floatx2 rc2 = {cr[q >> 1][(2 * q) & 3], cr[q >> 1][(2 * q + 1) & 3]};
          const floatx2 a2 = {ac[pb][2 * q], ac[pb][2 * q + 1]};
          const floatx2 r2 = h3_score2(a2, rc2, c2, sx2);
          w[2 * q] = r2[0];
          w[2 * q + 1] = r2[1];
        }
        float m = w[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, w[r]);
        const bool imp = m > best[pb];
        best[pb] = imp ? m : best[pb];
        btile[pb] = imp ? tile : btile[pb];
#pragma unroll
        for (int r = 0; r < 16; ++r) sv[pb][r] = imp ? w[r] : sv[pb][r];
      }
    };
    for (int ch = 0; ch < nch; ++ch) {
      const _Float16* img = reinterpret_cast<const _Float16*>(smem + (size_t)ch * CHUNK_H * 2);
      const float* ub = ubase + ch * 2 * CB;
#pragma unroll
      for (int cb = 0; cb < CB / 32; ++cb) {
        const int cur = cb & 1;
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const _Float16* a = img + (((cb * KS + ks) * 2) * 64 + lane) * 8;
          const halfx8 ahi = *reinterpret_cast<const halfx8*>(a);
          const halfx8 alo = *reinterpret_cast<const halfx8*>(a + 64 * 8);
#pragma unroll
          for (int pb = 0; pb < NPB; ++pb) {
            acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
            acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, blo[pb][ks], acc[cur][pb], 0, 0, 0);
            acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bhi[pb][ks], acc[cur][pb], 0, 0, 0);
          }
        }
        if (ptile >= 0) epilogue(acc[cur ^ 1], pu, ptile);
        ptile = (ch0 + ch) * (CB / 32) + cb;
        pu = ub + cb * 32;
        if constexpr (SGV > 0) {
#pragma unroll
          for (int i = 0; i < 3 * KS * NPB; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, SGV, 0);  // then up to SGV VALU
          }
        }
      }
    }
    if (ptile >= 0) epilogue(acc[((CB / 32) - 1) & 1], pu, ptile);

    int bidx[NPB];
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      int bi = 15;
#pragma unroll
      for (int r = 14; r >= 0; --r) bi = sv[pb][r] == best[pb] ? r : bi;
      bidx[pb] = btile[pb] >= 0 ? btile[pb] * 32 + (bi & 3) + 8 * (bi >> 2) + 4 * h : pin[pb];
    }
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      const float ob = __shfl_xor(best[pb], 32, 64);
      const int oi = __shfl_xor(bidx[pb], 32, 64);
      const float xs = xsq[pb] + __shfl_xor(xsq[pb], 32, 64);
      if (ob > best[pb] || (ob == best[pb] && oi < bidx[pb])) {
        best[pb] = ob;
        bidx[pb] = oi;
      }
      const int64_t row = prow[pb];
      if (h == 0 && row >= 0) {
        if (last) {
          labels[row] = bidx[pb];
          if (mind) {
            const float isx = 1.f / sx[pb];
            mind[row] = fmaxf(xs * isx * isx - 2.f * best[pb] * isx, 0.f);
          }
        } else {
          pbest[row] = best[pb];
          pidx[row] = bidx[pb];
        }
      }
    }
  }
}

int h3_fpad(int f) { return f <= 16 ? 16 : f <= 32 ? 32 : f <= 64 ? 64 : f <= 128 ? 128 : -1; }

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
// Feature padding used by the planes (row stride = 2 * fpad halfs), -1 if unsupported.
HA_EXPORT int ha_h3_fpad(int f) { return h3_fpad(f); }

HA_EXPORT int ha_h3_pack_points(const float* X, int64_t n, int f, int64_t ldx, void* planes, float* sx,
                                void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t threads = n * (fpad / 8);
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  _Float16* p = (_Float16*)planes;
  switch (fpad) {
    case 16: hipLaunchKernelGGL(h3_pack_points<16>, dim3(blocks), dim3(256), 0, s, X, n, f, ldx, p, sx); break;
    case 32: hipLaunchKernelGGL(h3_pack_points<32>, dim3(blocks), dim3(256), 0, s, X, n, f, ldx, p, sx); break;
    case 64: hipLaunchKernelGGL(h3_pack_points<64>, dim3(blocks), dim3(256), 0, s, X, n, f, ldx, p, sx); break;
    default: hipLaunchKernelGGL(h3_pack_points<128>, dim3(blocks), dim3(256), 0, s, X, n, f, ldx, p, sx); break;
  }
  return ha_launch_status();
}

// Workspace bytes for the centroid image + u + meta.
HA_EXPORT int64_t ha_h3_workspace_bytes(int k, int f) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || k <= 0) return -1;
  const int cb = fpad >= 128 ? 64 : 128;
  const int64_t kpad = (int64_t)(k + cb - 1) / cb * cb;
  // image + (u, r) per chunk + meta {-, max|c|_inf, u_max, -} + rank-1 u-term fragments (64 lanes x
  // 8 B per 32-centroid tile)
  return kpad * fpad * 2 * 2 + kpad * 8 + 16 + kpad * 16;
}

HA_EXPORT int ha_h3_assign(const void* planes, const float* sx, int64_t n, int f, const float* C, int k, int64_t ldc,
                           void* workspace, int* labels, float* mind, void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || k <= 0) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const int cb = fpad >= 128 ? 64 : 128;
  const int kpad = (k + cb - 1) / cb * cb;
  _Float16* image = (_Float16*)workspace;
  float* u = (float*)((char*)workspace + (int64_t)kpad * fpad * 4);
  float* meta = u + 2 * kpad;
  const _Float16* p = (const _Float16*)planes;
  // FPAD 128 keeps one 32-point block per wave (two spill: 4.62 -> 4.20 ms at f=100, k=1024, n=6.25M)
#define HA_H3(FP)                                                                                           \
  case FP: {                                                                                                \
    constexpr int NPB = FP >= 128 ? 1 : 2, MINB = 2;  /* 2 chunk buffers (~66 KB) per WG: 2 WGs/CU */                                        \
    using KC = H3Cfg<FP, NPB>;                                                                              \
    /* no memset of meta[1..2]: only h1_filter reads them (bench A/B: -12 us per step) */                  \
    hipLaunchKernelGGL(h3_cscale<FP>, dim3(h3_cscale_grid(kpad, FP / 8)), dim3(256), 0, s, C, k, f, ldc, kpad, u, meta, (unsigned*)(meta + 4));         \
    hipLaunchKernelGGL(h3_pack_centroids<FP>, dim3((unsigned)(((int64_t)kpad * (FP / 8) + 255) / 256)),  \
                       dim3(256), 0, s, C, k, f, ldc, kpad, image, u);                               \
    const size_t lds = 2 * ((size_t)KC::CHUNK_H * 2 + KC::CB * 8 + KC::CB * 16);                            \
    const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);                         \
    hipFuncSetAttribute(reinterpret_cast<const void*>(h3_assign_p<FP, NPB, true, MINB>),                    \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                              \
    hipLaunchKernelGGL((h3_assign_p<FP, NPB, true, MINB>), dim3(blocks), dim3(256), lds, s, p, sx, n, image, u, \
                       meta, kpad / KC::CB, labels, mind);                                                 \
    break;                                                                                                  \
  }
  switch (fpad) {
    HA_H3(16)
    HA_H3(32)
    HA_H3(64)
    HA_H3(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_H3
  return ha_launch_status();
}

// rows of one uncertain-point list: the points of the filter workgroups b with b % shards == s
static int64_t h3_amb_cap(int64_t n, int64_t pts_per_wg) {
  const int64_t wgs = (n + pts_per_wg - 1) / pts_per_wg;
  return (wgs + H3_AMB_SHARDS - 1) / H3_AMB_SHARDS * pts_per_wg;
}

// int32 words of the certified assignment's scratch: the H3_AMB_SHARDS row lists, then the
// H3_AMB_SHARDS counts (amb_rows = scratch, amb_count = scratch + ha_h3_amb_rows(n)).
HA_EXPORT int64_t ha_h3_amb_rows(int64_t n) { return H3_AMB_SHARDS * h3_amb_cap(n, 256); }
HA_EXPORT int ha_h3_amb_shards() { return H3_AMB_SHARDS; }

// Certified one-term assignment: h1_filter over all points, then the 3-term kernel over the points
// it could not certify. amb_rows: int32[ha_h3_amb_rows(n)] scratch; amb_count: ha_h3_amb_shards()
// int32 list counts, zeroed here; their sum is the
// number of re-checked points afterwards. Labels are identical to ha_h3_assign's up to points
// whose two best centroids are within the 3-term kernel's own rounding of each other.
HA_EXPORT int ha_h3_assign_certified(const void* planes, const float* sx, int64_t n, int f, const float* C, int k,
                                     int64_t ldc, void* workspace, int* labels, int* amb_rows, int* amb_count,
                                     void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || k <= 0) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  if (n > INT32_MAX) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const int cb = fpad >= 128 ? 64 : 128;
  const int kpad = (k + cb - 1) / cb * cb;
  _Float16* image = (_Float16*)workspace;
  float* u = (float*)((char*)workspace + (int64_t)kpad * fpad * 4);
  float* meta = u + 2 * kpad;
  const _Float16* p = (const _Float16*)planes;
  hipMemsetAsync(amb_count, 0, H3_AMB_SHARDS * sizeof(int), s);
#define HA_H1(FP)                                                                                           \
  case FP: {                                                                                                \
    constexpr int NPB = FP >= 128 ? 1 : 2, MINB = 2;  /* 2 chunk buffers (~66 KB) per WG: 2 WGs/CU */                                        \
    constexpr int NPB1 = FP >= 128 ? 1 : 2, MINB1 = 2;                                                      \
    using KC = H3Cfg<FP, NPB>;                                                                              \
    using K1 = H3Cfg<FP, NPB1>;                                                                             \
    hipMemsetAsync(meta, 0, 4 * sizeof(float), s);                                                          \
    hipLaunchKernelGGL(h3_cscale<FP>, dim3(h3_cscale_grid(kpad, FP / 8)), dim3(256), 0, s, C, k, f, ldc, kpad, u, meta, (unsigned*)(meta + 4));         \
    hipLaunchKernelGGL(h3_pack_centroids<FP>, dim3((unsigned)(((int64_t)kpad * (FP / 8) + 255) / 256)),  \
                       dim3(256), 0, s, C, k, f, ldc, kpad, image, u);                               \
    const size_t lds1 = 2 * ((size_t)K1::CHUNK_H + K1::CB * 8);                                                   \
    const unsigned blocks1 = (unsigned)((n + K1::PTS_PER_WG - 1) / K1::PTS_PER_WG);                        \
    hipFuncSetAttribute(reinterpret_cast<const void*>(h1_filter<FP, NPB1, MINB1>),                          \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);                             \
    const int64_t cap = h3_amb_cap(n, K1::PTS_PER_WG);                                                     \
    hipLaunchKernelGGL((h1_filter<FP, NPB1, MINB1>), dim3(blocks1), dim3(256), lds1, s, p, sx, n, image, u, meta, \
                       kpad / K1::CB, labels, amb_rows, amb_count, cap);                                   \
    const size_t lds = 2 * ((size_t)KC::CHUNK_H * 2 + KC::CB * 8 + KC::CB * 16);                            \
    const int64_t maxb = (n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG;                                        \
    const unsigned blocks = (unsigned)(maxb < (int64_t)ncu * MINB ? maxb : (int64_t)ncu * MINB);            \
    hipFuncSetAttribute(reinterpret_cast<const void*>(h3_assign_p<FP, NPB, true, MINB, true>),              \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                              \
    hipLaunchKernelGGL((h3_assign_p<FP, NPB, true, MINB, true>), dim3(blocks), dim3(256), lds, s, p, sx, n, image, u, \
                       meta, kpad / KC::CB, labels, (float*)nullptr, (const int*)amb_rows, (const int*)amb_count, \
                       cap);                                                                               \
    break;                                                                                                  \
  }
  switch (fpad) {
    HA_H1(16)
    HA_H1(32)
    HA_H1(64)
    HA_H1(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_H1
  return ha_launch_status();
}

// Certified one-term k nearest rows of C (see h1_topk): dist / idx [n, kp] approximate squared
// distances ascending + int32 row indices (the caller rescores them exactly), cert [n] uint8 (1 =
// the true kn nearest are among the kp). kn <= 8 with kp = 16 or 32. workspace: ha_h3_workspace_bytes.
HA_EXPORT int ha_h1_topk(const void* planes, const float* sx, int64_t n, int f, const float* C, int m, int64_t ldc,
                         void* workspace, int kn, int kp, float* dist, int* idx, unsigned char* cert, void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || m <= 0 || kn < 1 || kn > 8 || (kp != 16 && kp != 32)) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const int cb = fpad >= 128 ? 64 : 128;
  const int kpad = (m + cb - 1) / cb * cb;
  _Float16* image = (_Float16*)workspace;
  float* u = (float*)((char*)workspace + (int64_t)kpad * fpad * 4);
  float* meta = u + 2 * kpad;
  const _Float16* p = (const _Float16*)planes;
  // the error bound needs max |c| and max u (atomicMax into zeroed words)
  if (hipMemsetAsync(meta, 0, 16, s) != hipSuccess) return HA_LAUNCH;
#define HA_H1TK_KO(FP, KN, KO)                                                                                 \
  hipFuncSetAttribute(reinterpret_cast<const void*>(h1_topk<FP, 16, KN, NPBT, KO>),                             \
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                    \
  hipLaunchKernelGGL((h1_topk<FP, 16, KN, NPBT, KO>), dim3(blocks), dim3(256), lds, s, p, sx, n, image, u, meta,  \
                     kpad / KC::CB, dist, idx, cert)
#define HA_H1TK_KN(FP, KN)                                                                                     \
  if (kp == 32) {                                                                                              \
    HA_H1TK_KO(FP, KN, 32);                                                                                    \
  } else {                                                                                                     \
    HA_H1TK_KO(FP, KN, 16);                                                                                    \
  }
#define HA_H1TK(FP)                                                                                              \
  case FP: {                                                                                                     \
    constexpr int NPBT = FP >= 128 ? 1 : 2;                                                                      \
    using KC = H3Cfg<FP, NPBT>;                                                                                  \
    hipLaunchKernelGGL(h3_cscale<FP>, dim3(h3_cscale_grid(kpad, FP / 8)), dim3(256), 0, s, C, m, f, ldc, kpad, u,  \
                       meta, (unsigned*)(meta + 4));                                                             \
    hipLaunchKernelGGL(h3_pack_centroids<FP>, dim3((unsigned)(((int64_t)kpad * (FP / 8) + 255) / 256)),       \
                       dim3(256), 0, s, C, m, f, ldc, kpad, image, u);                                           \
    const size_t lds = 2 * ((size_t)KC::CHUNK_H + KC::CB * 8 + KC::CB * 16);                                    \
    const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);                              \
    if (kn <= 1) { HA_H1TK_KN(FP, 1); }                                                                          \
    else if (kn <= 4) { HA_H1TK_KN(FP, 4); }                                                                     \
    else { HA_H1TK_KN(FP, 8); }                                                                                  \
    break;                                                                                                       \
  }
  switch (fpad) {
    HA_H1TK(16)
    HA_H1TK(32)
    HA_H1TK(64)
    HA_H1TK(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_H1TK
#undef HA_H1TK_KN
#undef HA_H1TK_KO
  return ha_launch_status();
}

// k nearest rows of C (m rows, e.g. KNN training points) for each of the n packed points:
// dist [n, kout] squared distances ascending, idx [n, kout] int32 (row of C; -1 past m).
// kout <= 16. workspace: ha_h3_workspace_bytes(m, f). splits > 1: the centroid chunks are divided
// over `splits` workgroup columns and dist/idx hold `splits` partial [n, kout] lists (the caller
// merges them); ha_h3_topk_chunks(m, f) gives the number of chunks to divide.
HA_EXPORT int ha_h3_topk_chunks(int m, int f) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || m <= 0) return -1;
  const int cb = fpad >= 128 ? 64 : 128;
  return (m + cb - 1) / cb;
}

HA_EXPORT int ha_h3_topk(const void* planes, const float* sx, int64_t n, int f, const float* C, int m, int64_t ldc,
                         void* workspace, int kout, int splits, float* dist, int* idx, void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || m <= 0 || kout <= 0 || kout > 16) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  if (splits < 1 || splits > ha_h3_topk_chunks(m, f) || splits > 65535) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int cb = fpad >= 128 ? 64 : 128;
  const int kpad = (m + cb - 1) / cb * cb;
  // HEAT_H3_TOPK_V1=1: the round-3 kernel (A/B)
  static const bool v1 = getenv("HEAT_H3_TOPK_V1") && getenv("HEAT_H3_TOPK_V1")[0] == '1';
  _Float16* image = (_Float16*)workspace;
  float* u = (float*)((char*)workspace + (int64_t)kpad * fpad * 4);
  float* meta = u + 2 * kpad;
  const _Float16* p = (const _Float16*)planes;
#define HA_TK_LAUNCH(FP, KN)                                                                                 \
  do {                                                                                                       \
  if (v1) {                                                                                                  \
    hipLaunchKernelGGL((h3_topk<FP, KN>), dim3(blocks, splits), dim3(256), lds, s, p, sx, n, image, u, meta,    \
                       kpad / KC::CB, (kpad / KC::CB + splits - 1) / splits, kout, dist, idx);              \
  } else {                                                                                                   \
    constexpr int NPBT = FP >= 128 ? 1 : 2;                                                                  \
    using KP = H3Cfg<FP, NPBT>;                                                                              \
    const size_t ldsp = 2 * ((size_t)KP::CHUNK_H * 2 + KP::CB * 8 + KP::CB * 16);                           \
    const unsigned bp = (unsigned)((n + KP::PTS_PER_WG - 1) / KP::PTS_PER_WG);                               \
    hipFuncSetAttribute(reinterpret_cast<const void*>(h3_topk_p<FP, KN, NPBT>),                               \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsp);                              \
    hipLaunchKernelGGL((h3_topk_p<FP, KN, NPBT>), dim3(bp, splits), dim3(256), ldsp, s, p, sx, n, image, u,   \
                       meta, kpad / KC::CB, (kpad / KC::CB + splits - 1) / splits, kout, dist, idx);        \
  }                                                                                                          \
  } while (0)
#define HA_TK(FP)                                                                                            \
  case FP: {                                                                                                 \
    using KC = H3Cfg<FP, 1>;                                                                                 \
    /* meta[1..2] (filter bound) unused: no memset */                                                           \
    hipLaunchKernelGGL(h3_cscale<FP>, dim3(h3_cscale_grid(kpad, FP / 8)), dim3(256), 0, s, C, m, f, ldc, kpad, u, meta, (unsigned*)(meta + 4));          \
    hipLaunchKernelGGL(h3_pack_centroids<FP>, dim3((unsigned)(((int64_t)kpad * (FP / 8) + 255) / 256)),   \
                       dim3(256), 0, s, C, m, f, ldc, kpad, image, u);                                \
    const size_t lds = (size_t)KC::CHUNK_H * 2 + KC::CB * 8;                                                 \
    const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);                          \
    if (kout <= 4)                                                                                           \
      HA_TK_LAUNCH(FP, 4);                                                                                   \
    else if (kout <= 8)                                                                                      \
      HA_TK_LAUNCH(FP, 8);                                                                                   \
    else                                                                                                     \
      HA_TK_LAUNCH(FP, 16);                                                                                  \
    break;                                                                                                   \
  }
  switch (fpad) {
    HA_TK(16)
    HA_TK(32)
    HA_TK(64)
    HA_TK(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_TK
#undef HA_TK_LAUNCH
  return ha_launch_status();
}

// Resident-centroid assignment (h3_assign_r): chunks resident per phase and number of phases.
constexpr int H3R_LDS = 128 * 1024;   // image budget per workgroup (+ u)
constexpr int H3R_NW = 8;             // waves per workgroup (one workgroup per CU)

HA_EXPORT int ha_h3r_phases(int k, int f) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || k <= 0) return -1;
  const int cb = fpad >= 128 ? 64 : 128;
  const int nchunks = (k + cb - 1) / cb;
  const int rc = H3R_LDS / (cb * fpad * 4);
  return (nchunks + rc - 1) / rc;
}

// scratch: n floats + n ints (carried best between phases; unused with one phase)
HA_EXPORT int ha_h3_assign_r(const void* planes, const float* sx, int64_t n, int f, const float* C, int k,
                             int64_t ldc, void* workspace, void* scratch, int num_cus, int* labels, float* mind,
                             void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || k <= 0 || num_cus <= 0) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const int cb = fpad >= 128 ? 64 : 128;
  const int kpad = (k + cb - 1) / cb * cb;
  const int nchunks = kpad / cb;
  const int rc = H3R_LDS / (cb * fpad * 4);
  const int phases = (nchunks + rc - 1) / rc;
  if (phases > 1 && !scratch) return HA_BAD_ARG;
  _Float16* image = (_Float16*)workspace;
  float* u = (float*)((char*)workspace + (int64_t)kpad * fpad * 4);
  float* meta = u + 2 * kpad;
  const _Float16* p = (const _Float16*)planes;
  float* pb = (float*)scratch;
  int* pi = scratch ? (int*)((char*)scratch + n * sizeof(float)) : nullptr;
  const int64_t blocks_needed = (n + 64 * H3R_NW - 1) / (64 * H3R_NW);
  const unsigned grid = (unsigned)(blocks_needed < num_cus ? blocks_needed : num_cus);
#define HA_H3R(FP)                                                                                          \
  case FP: {                                                                                                \
    constexpr int NPB = FP >= 128 ? 1 : 2;                                                                  \
    using KC = H3Cfg<FP, NPB>;                                                                              \
    /* meta[1..2] (filter bound) unused: no memset */                                                          \
    hipLaunchKernelGGL(h3_cscale<FP>, dim3(h3_cscale_grid(kpad, FP / 8)), dim3(256), 0, s, C, k, f, ldc, kpad, u, meta, (unsigned*)(meta + 4));         \
    hipLaunchKernelGGL(h3_pack_centroids<FP>, dim3((unsigned)(((int64_t)kpad * (FP / 8) + 255) / 256)),  \
                       dim3(256), 0, s, C, k, f, ldc, kpad, image, u);                               \
    for (int ph = 0; ph < phases; ++ph) {                                                                   \
      const int c0 = ph * rc, nc = nchunks - c0 < rc ? nchunks - c0 : rc;                                   \
      const size_t lds = (size_t)nc * KC::CHUNK_H * 2 + (size_t)nc * KC::CB * 8;                            \
      hipFuncSetAttribute(reinterpret_cast<const void*>(h3_assign_r<FP, NPB, H3R_NW>),                      \
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                            \
      hipLaunchKernelGGL((h3_assign_r<FP, NPB, H3R_NW>), dim3(grid), dim3(H3R_NW * 64), lds, s, p, sx, n, image, \
                         u, meta, c0, nc, ph == 0, ph == phases - 1, pb, pi, labels, mind);                  \
    }                                                                                                       \
    break;                                                                                                  \
  }
  switch (fpad) {
    HA_H3R(16)
    HA_H3R(32)
    HA_H3R(64)
    HA_H3R(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_H3R
  return ha_launch_status();
}
