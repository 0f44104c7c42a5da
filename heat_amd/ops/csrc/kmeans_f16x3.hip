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
#include "h3_common.h"

namespace {

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
