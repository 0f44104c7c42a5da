// hipcc-flags: -fno-slp-vectorize
// Certified one-term kNN top-k (h1_topk, see its comment) on the FP16 matrix cores: the screening
// pass of ops.knn_topk; uncertain points go back through h3_topk_p (knn_f16x3.hip). Split from
// knn_f16x3.hip so that the two kernel families compile in parallel.
#include "h3_common.h"

namespace {

// s_waitcnt vmcnt(N), expcnt / lgkmcnt left alone (gfx9 encoding: vmcnt bits 3:0 and 15:14,
// expcnt 6:4, lgkmcnt 11:8)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4; LDS address = lds + 16 lane) issued
// through inline asm: for the builtin the compiler's wait-count pass cannot tell which LDS bytes
// the transfer writes and puts s_waitcnt vmcnt(0) before the next LDS read - i.e. it waits for
// the prefetched chunk too. The asm form is invisible to that pass (its own vmcnt waits only
// become more conservative); the kernel waits for its transfers with counted vm_wait<N>().
__device__ __forceinline__ void lds_dma16(const void* g, unsigned lds) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
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
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
  // chunk staging: FOUR LDS buffers, two chunks in flight. Round 4 waited for each chunk's DMA
  // right after issuing it, and the 3-buffer / one-ahead version measured only 2 % faster (368 ms,
  // 31 % MFMA-busy): a workgroup streams the whole training image (the L2 serves ~92 % of it,
  // FETCH_SIZE), so the chunk rate is latency x bytes in flight - 17.5 KB per workgroup was not
  // enough. Now chunk ch + 2 is issued while ch is computed (35 KB per workgroup, 70 KB per CU in
  // flight). One barrier per chunk: at the barrier of chunk ch every wave has finished chunk
  // ch - 1, the last reader of buffer (ch + 2) % 4 (chunk ch - 2's deferred last-tile epilogue).
  // Per wave the u / v pieces are issued before the image pieces (vmcnt retires in order).
  constexpr int IMGW = PIECES / 4;
  static_assert(PIECES % 4 == 0 && IMGW >= 1 && IMGW <= 4, "image pieces per wave");
  static_assert(VPIECES <= 4, "v pieces per chunk");
  // DMA instructions per chunk issued by this wave (u: wave 0; v piece pc: wave pc; image: IMGW)
  const int per_chunk = (wave == 0 ? 1 : 0) + (wave < VPIECES ? 1 : 0) + IMGW;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem);
  auto issue = [&](int ch) {
    const char* src = reinterpret_cast<const char*>(image + (int64_t)ch * CHUNK_H) + lane * 16;
    const unsigned dst = lds0 + (ch & 3) * BUF;
    if (wave == 0 && lane < CB / 2) lds_dma16(reinterpret_cast<const char*>(u + ch * 2 * CB) + lane * 16, dst + CHUNK_H);
#pragma unroll
    for (int pc = wave; pc < VPIECES; pc += 4)
      lds_dma16(reinterpret_cast<const char*>(vimg) + (int64_t)ch * CB * 16 + pc * 1024 + lane * 16,
                dst + CHUNK_H + CB * 8 + pc * 1024);
#pragma unroll
    for (int pc = wave; pc < PIECES; pc += 4) lds_dma16(src + 2 * pc * 1024, dst + pc * 1024);
  };
  if (nchunks > 0) issue(0);
  if (nchunks > 1) issue(1);
  for (int ch = 0; ch < nchunks; ++ch) {
    __builtin_amdgcn_sched_barrier(0);
    // this wave's pieces of chunk ch have landed once at most chunk ch + 1's are outstanding
    if (ch + 1 < nchunks) {
      if (per_chunk == IMGW) vm_wait<IMGW>();
      else if (per_chunk == IMGW + 1) vm_wait<IMGW + 1>();
      else vm_wait<IMGW + 2>();
    } else {
      vm_wait<0>();
    }
    // a raw barrier: __syncthreads() would add s_waitcnt vmcnt(0), i.e. wait for the prefetch too
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (ch + 2 < nchunks) issue(ch + 2);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned char* buf = smem + (ch & 3) * BUF;
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

}  // namespace

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
    const size_t lds = 4 * ((size_t)KC::CHUNK_H + KC::CB * 8 + KC::CB * 16);  /* 4 chunk buffers */            \
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
