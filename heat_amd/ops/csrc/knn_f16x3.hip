// hipcc-flags: -fno-slp-vectorize
// k nearest rows (kNN, cdist_topk) on the FP16 matrix cores with the fp16x3 split of
// kmeans_f16x3.hip (shared packing / scaling code in h3_common.h): h3_topk / h3_topk_p (3-term
// scores + register top-k). The certified one-term screening kernel h1_topk is in knn_h1.hip.
#include "h3_common.h"

namespace {

// k nearest "centroids" (KNN: the training points) of every point, the same fp16x3 scores as the
// assignment (score = x.c - |c|^2/2 in the scaled space, larger = nearer) with a running top-KN
// list per lane instead of a running max: no n x m distance matrix. A lane keeps its KN best
// (score, index) sorted in registers; a tile's 16 candidates are only inserted where they beat
// the lane's current KN-th best (after the first tiles nearly never: ~KN ln(m) insertions per
// point), so the epilogue is a max + compare per tile in the common case. The two lane halves
// (disjoint centroid halves of the same point) merge their lists at the end. Output: KN squared
// distances (ascending) and int32 indices per point; -1 / +inf where fewer than KN exist.

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

}  // namespace

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

