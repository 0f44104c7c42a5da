// hipcc-flags: -fno-slp-vectorize
// 128 x 128-tile exact fp32 GEMM, LDS-DMA pipelined: the mid-size products whose
// 256 x 256 tiles cannot fill the 256 CUs (1024^3 .. 6144^3, split-K) and the short-K tall
// trailing update of the Householder QR, C[m, N] -= V[m, 256] X[256, N] (K = 256: 16 k-stages per
// tile, so the tile's prologue and its C traffic must overlap another workgroup's MFMAs - two
// workgroups per CU here, one for the 256-tile kernel).
//
// Round-5 form (gemm_small.hip: gemm_f32s) staged operands through registers: global loads ->
// VGPRs -> ds_write -> barrier -> ds_read, one barrier per 32 k, measured 35 % MFMA-busy with 38 %
// of wave cycles waiting. This kernel moves operands global -> LDS directly:
//   * LDS-DMA (global_load_lds_dwordx4 by inline asm, 1 KB per wave-instruction) into a ring of
//     NBUF stage buffers of 16 k (16 KB per stage: 8 pieces per operand, 2 + 2 per wave), NBUF - 1
//     stages in flight, one raw s_barrier per stage behind a COUNTED vmcnt (never vmcnt(0) in the
//     steady state) - the DMA of stage t + NBUF - 1 spans the barriers of the stages before it;
//   * asm DMA instead of the builtin: the compiler's wait-count pass cannot tell which LDS bytes
//     a builtin DMA writes and would put vmcnt(0) before every LDS read (all prefetches waited);
//   * fragments of stage t + 1 read (ds_read_b128 / ds_read_b64, conflict-free) into the second
//     register set while stage t's MFMAs run;
//   * k-contiguous operands are imaged [k/4][row][4] (a lane reads 16 B of its row per k-chunk),
//     row-contiguous ones [k][row] (one piece = two whole k-rows). For a row-contiguous operand
//     the 32 x 32 block's rows are INTERLEAVED - block b, lane r <-> tile row 2 r + b - so one
//     ds_read_b64 feeds both blocks of a wave (the epilogue maps rows / columns back);
//   * 4 waves of 64 x 64 (2 x 2 v_mfma_f32_32x32x2_f32 accumulators, 64 registers), two
//     workgroups per CU (NBUF = 4: 66 KB of LDS each) so one workgroup's epilogue / prologue
//     overlaps the other's MFMAs;
//   * accumulate: the epilogue loads a whole accumulator row's C values (32 loads in flight)
//     before it stores (C preloaded into the accumulators measured slower on gemm_f32t and rounds
//     every partial sum at the scale of C: 40x the error at K = 256, profiles/update_ab_r06.jsonl);
//   * XCD-aware grouped tile order (each XCD takes a contiguous range of tiles, walked in groups
//     of 8 row panels, so both operand panels are re-read from that XCD's L2).
// Reference hot loops: heat/core/linalg/basics.py:1650-1732 (block GEMMs), heat/core/linalg/qr.py:
// 353, 942 (tile QR updates).
#include "common.h"

#include <stdlib.h>

#include <type_traits>

namespace {

constexpr int MB = 128;       // tile rows / columns
constexpr int MK = 16;        // k per stage
constexpr int MOP = 8192;     // bytes per operand per stage (128 rows x 16 k x 4 B)
constexpr int MSTAGE = 2 * MOP;

// 32-bit: the host caps the grid at 2^31 tiles (64-bit divisions are long SALU sequences)
__device__ __forceinline__ unsigned gm_xcd_remap(unsigned orig, unsigned nwg) {
  const unsigned q = nwg / 8, r = nwg % 8, xcd = orig % 8, loc = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// LDS-DMA of 16 bytes per lane to LDS byte address lds + 16 lane (wave-uniform lds); M0 saved /
// restored around it (the compiler treats M0 as reserved and would not see a clobber)
__device__ __forceinline__ void gm_dma16(const void* g, unsigned lds) {
  unsigned saved;
  const unsigned base = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(base)
               : "memory");
}

// at most N of this wave's vector-memory ops outstanding, LDS ops retired, then the barrier (any
// N < 64: the count is an assembler immediate; an earlier three-case form fell back to vmcnt(0)
// for the counts of the 256 x 128 variant, 12 and 6)
template <int N>
__device__ __forceinline__ void gm_wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void gm_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// One operand's staging for this lane, TR tile rows (128 or 256). KC (k-contiguous, [rows][K]
// with leading dimension ld): G = TR / 64 row groups; piece q = k-chunk q / G (4 k), rows
// 64 (q % G) + lane; image [4 chunks][TR rows][4] - piece q at q KB. Else row-contiguous ([K][rows]):
// RP = TR / 4 lanes per k-row, piece q = k-rows KPP q + lane / RP (KPP = 64 / RP), 4 rows
// 4 (lane % RP) .. + 3; image [16 k][TR rows] at 4 TR bytes per k-row - piece q at q KB too.
// Out-of-range rows are clamped (their results are masked at the store).
template <bool KC, int TR>
struct GmSrc {
  static constexpr int G = TR / 64, RP = TR / 4, KPP = 64 / RP;
  const float* rp[G];  // KC: this lane's row of each 64-row group
  const float* cp;     // row-contiguous: this lane's 4-row group at k = lane / RP
  int64_t ld;
  __device__ __forceinline__ void init(const float* P, int64_t ld_, int64_t rows, int64_t r0, int lane) {
    ld = ld_;
    if (KC) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int64_t row = r0 + 64 * g + lane;
        rp[g] = P + (row < rows ? row : rows - 1) * ld;
      }
    } else {
      int64_t c = r0 + 4 * (lane % RP);
      c = c + 4 <= rows ? c : rows - 4;
      cp = P + (int64_t)(lane / RP) * ld + c;
    }
  }
  // source of piece q of the stage at k0 (whole stage in range)
  __device__ __forceinline__ const float* src(int64_t k0, int q) const {
    return KC ? rp[q % G] + k0 + 4 * (q / G) : cp + (k0 + KPP * q) * ld;
  }
  // the same with the k index clamped into [0, K) (the tail stage; the clamped entries are zeroed
  // after they land). KC requires K % 4 == 0.
  __device__ __forceinline__ const float* src_clamped(int64_t k0, int q, int64_t K, int lane) const {
    if (KC) {
      const int64_t k = k0 + 4 * (q / G) + 4 <= K ? k0 + 4 * (q / G) : K - 4;
      return rp[q % G] + k;
    }
    const int64_t k = k0 + KPP * q + lane / RP;
    return cp + ((k < K ? k : K - 1) - lane / RP) * ld;
  }
  __device__ __forceinline__ bool beyond(int64_t k0, int q, int64_t K, int lane) const {
    return KC ? k0 + 4 * (q / G) >= K : k0 + KPP * q + lane / RP >= K;
  }
};

// Fragments of one stage for a wave: a[b][s], b[b][s] = block b's operand at k = 8 h + s.
template <int WMB, int WNB>
struct GmFrag {
  float a[WMB][8], b[WNB][8];
};

// AK: A k-major ([K][M], m contiguous) - else row-major ([M][K], k contiguous).
// BK_: B k-major ([K][N], n contiguous) - else n-major ([N][K], k contiguous).
// WMB: 32 x 32 blocks per wave along M - 2: 128 x 128 tiles (waves of 64 x 64, 64 KB of LDS for
// NBUF = 4, the default); 4: 256 x 128 tiles (waves of 128 x 64: 0.75 LDS floats per MFMA instead
// of 1, 43 instead of 32 flop per staged byte; NBUF = 3, 72 KB; measured slower - A/B only). Two
// workgroups per CU either way.
// GSZ = 2 (A/B): stages in pairs under ONE barrier (a 32-deep K slice per barrier): the pair's
// DMA lands during the previous pair, whose ring slots it then refills; K a whole number of pairs.
template <bool AK, bool BK_, int WMB, int NBUF, int WNB = 2, int GSZ = 1>
__global__ __launch_bounds__(256, 2) void gemm_f32m(const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C, int64_t M, int64_t N, int64_t K,
                                                    int64_t lda, int64_t ldb, int64_t ldc, float alpha, int beta,
                                                    int64_t kps, int64_t cslice) {
  constexpr int TM = 64 * WMB;          // tile rows
  constexpr int TN = 64 * WNB;          // tile columns
  constexpr int AOP = TM * MK * 4;      // bytes of A per stage
  constexpr int BOP = TN * MK * 4;      // bytes of B per stage
  constexpr int STG = AOP + BOP;        // bytes per stage
  constexpr int PAW = TM / 64;          // A pieces per wave per stage (TM / 16 pieces / 4 waves)
  constexpr int PBW = TN / 64;          // B pieces per wave per stage
  constexpr int AHEAD = NBUF - 1;       // stages in flight
  constexpr int DPS = PAW + PBW;        // DMA instructions per wave per stage
  static_assert(NBUF * STG <= 80 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r = lane & 31;
  const unsigned tn = (unsigned)((N + TN - 1) / TN), tm = (unsigned)((M + TM - 1) / TM);
  const unsigned bid = gm_xcd_remap(blockIdx.x, tm * tn);
  constexpr unsigned GM = 8;
  const unsigned grp = bid / (GM * tn), gfirst = grp * GM;
  const unsigned gsz = tm - gfirst < GM ? tm - gfirst : GM;
  const int64_t m0 = (int64_t)(gfirst + (bid % (GM * tn)) % gsz) * TM, n0 = (int64_t)((bid % (GM * tn)) / gsz) * TN;
  // split-K: slice blockIdx.y = k in [y kps MK, min((y + 1) kps MK, K)) into C + y cslice
  {
    const int64_t k0 = (int64_t)blockIdx.y * kps * MK;
    A += AK ? k0 * lda : k0;
    B += BK_ ? k0 * ldb : k0;
    K = K - k0 < kps * MK ? K - k0 : kps * MK;
    C += (int64_t)blockIdx.y * cslice;
  }
  GmSrc<!AK, TM> sa;
  GmSrc<!BK_, TN> sb;
  sa.init(A, lda, M, m0, lane);
  sb.init(B, ldb, N, n0, lane);
  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;

  auto stage = [&](int64_t t, bool full) {
    const unsigned dst = sbase + (unsigned)((t % NBUF) * STG);
    const int64_t k0 = t * MK;
#pragma unroll
    for (int i = 0; i < PAW; ++i) {
      const int q = PAW * wave + i;
      gm_dma16(full ? sa.src(k0, q) : sa.src_clamped(k0, q, K, lane), dst + q * 1024);
    }
#pragma unroll
    for (int i = 0; i < PBW; ++i) {
      const int q = PBW * wave + i;
      gm_dma16(full ? sb.src(k0, q) : sb.src_clamped(k0, q, K, lane), dst + AOP + q * 1024);
    }
  };
  auto zero_tail = [&](int64_t t) {
    unsigned char* dst = smem + (t % NBUF) * STG;
    const int64_t k0 = t * MK;
#pragma unroll
    for (int i = 0; i < PAW; ++i) {
      const int q = PAW * wave + i;
      if (sa.beyond(k0, q, K, lane)) *reinterpret_cast<floatx4*>(dst + q * 1024 + lane * 16) = (floatx4)(0.f);
    }
#pragma unroll
    for (int i = 0; i < PBW; ++i) {
      const int q = PBW * wave + i;
      if (sb.beyond(k0, q, K, lane)) *reinterpret_cast<floatx4*>(dst + AOP + q * 1024 + lane * 16) = (floatx4)(0.f);
    }
  };

  // fragment reads, NB blocks of an operand per wave over TR tile rows. k-contiguous operand,
  // block b: row 32 b + r of the wave's rows, k-chunks 2 h and 2 h + 1 (two ds_read_b128).
  // Row-contiguous: rows NB r .. NB r + NB - 1 of the wave's rows (blocks 0 .. NB - 1) at k-row
  // 8 h + s (one ds_read_b64 / b128 per s; conflict-free: a lane group spans 64 banks).
  typedef float floatx2 __attribute__((ext_vector_type(2)));
  auto opnd = [&](const unsigned char* b, int w0, auto kc_tag, auto nb_tag, auto tr_tag, float (*o)[8])
      __attribute__((always_inline)) {
    constexpr bool kc = decltype(kc_tag)::value;
    constexpr int NB = decltype(nb_tag)::value, TR = decltype(tr_tag)::value;
    if constexpr (kc) {
#pragma unroll
      for (int bl = 0; bl < NB; ++bl) {
        const int row = w0 + 32 * bl + r;
        const floatx4 x0 = *reinterpret_cast<const floatx4*>(b + (2 * h) * (TR * 16) + row * 16);
        const floatx4 x1 = *reinterpret_cast<const floatx4*>(b + (2 * h + 1) * (TR * 16) + row * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          o[bl][s] = x0[s];
          o[bl][4 + s] = x1[s];
        }
      }
    } else if constexpr (NB == 1) {
#pragma unroll
      for (int s = 0; s < 8; ++s) o[0][s] = *reinterpret_cast<const float*>(b + (8 * h + s) * (TR * 4) + (w0 + r) * 4);
    } else if constexpr (NB == 2) {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const floatx2 v = *reinterpret_cast<const floatx2*>(b + (8 * h + s) * (TR * 4) + (w0 + 2 * r) * 4);
        o[0][s] = v[0];
        o[1][s] = v[1];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(b + (8 * h + s) * (TR * 4) + (w0 + 4 * r) * 4);
#pragma unroll
        for (int bl = 0; bl < 4; ++bl) o[bl][s] = v[bl];
      }
    }
  };
  auto load = [&](GmFrag<WMB, WNB>& F, int64_t t) {
    const unsigned char* base = smem + (t % NBUF) * STG;
    opnd(base, wm * 32 * WMB, std::integral_constant<bool, !AK>(), std::integral_constant<int, WMB>(),
         std::integral_constant<int, TM>(), F.a);
    opnd(base + AOP, wn * 32 * WNB, std::integral_constant<bool, !BK_>(), std::integral_constant<int, WNB>(),
         std::integral_constant<int, TN>(), F.b);
  };

  // accumulator (block bm, bn) element g <-> tile row / column (see the header)
  auto crow = [&](int bm, int g) -> int {
    const int rho = (g & 3) + 8 * (g >> 2) + 4 * h;
    return wm * 32 * WMB + (AK ? WMB * rho + bm : 32 * bm + rho);
  };
  auto ccol = [&](int bn) -> int { return wn * 32 * WNB + (BK_ ? WNB * r + bn : 32 * bn + r); };

  floatx16 acc[WMB][WNB];
  const bool full = m0 + TM <= M && n0 + TN <= N;
#pragma unroll
  for (int bm = 0; bm < WMB; ++bm)
#pragma unroll
    for (int bn = 0; bn < WNB; ++bn) acc[bm][bn] = (floatx16)(0.f);

  auto mma_row = [&](const GmFrag<WMB, WNB>& F, int bm) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int bn = 0; bn < WNB; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(F.a[bm][s], F.b[bn][s], acc[bm][bn], 0, 0, 0);
  };
  // the stage's MFMAs in two halves around the barrier: by block rows, or (one block row) by k-steps
  auto mma_half = [&](const GmFrag<WMB, WNB>& F, int part) {
    if constexpr (WMB >= 2) {
#pragma unroll
      for (int bm = part * WMB / 2; bm < (part + 1) * WMB / 2; ++bm) mma_row(F, bm);
    } else {
#pragma unroll
      for (int s = 4 * part; s < 4 * part + 4; ++s)
#pragma unroll
        for (int bn = 0; bn < WNB; ++bn)
          acc[0][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(F.a[0][s], F.b[bn][s], acc[0][bn], 0, 0, 0);
    }
  };

  const int64_t nk = K > 0 ? (K + MK - 1) / MK : 0;
  const bool tail = (K % MK) != 0;
  // stage t landed (this wave's DMA) and visible to every wave; later stages may be in flight
  auto ready = [&](int64_t t) {
    const int64_t later = nk - 1 - t < AHEAD - 1 ? nk - 1 - t : AHEAD - 1;  // stages issued after t
    if (tail && t == nk - 1) {
      gm_vm_wait<0>();
      zero_tail(t);
    }
    if (later >= 2) gm_wait_barrier<2 * DPS>();
    else if (later == 1) gm_wait_barrier<DPS>();
    else gm_wait_barrier<0>();
  };
  // steady state: stage t + AHEAD issued (whole, in range), MFMAs of the first half of the block
  // rows around it, the counted wait for stage t + 1 + barrier, then stage t + 1's fragment reads
  // between the second half's MFMAs
  auto step_full = [&](int64_t t, const GmFrag<WMB, WNB>& Fc, GmFrag<WMB, WNB>& Fn) {
    stage(t + AHEAD, true);
    mma_half(Fc, 0);
#pragma unroll
    for (int q = 0; q < DPS; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * WMB * WNB / DPS, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);              // VMEM read (the asm DMA)
    }
    __builtin_amdgcn_sched_barrier(0);
    gm_wait_barrier<(AHEAD - 1) * DPS>();
    load(Fn, t + 1);
    mma_half(Fc, 1);
    __builtin_amdgcn_sched_barrier(0);
  };
  // whole tiles with 256 ldc < 2^31: a uniform 64-bit tile base + 32-bit lane offsets in the
  // epilogue (the row terms dr ldc are scalar products), no bounds tests - the 64-bit per-element
  // form was ~1000 VALU per tile-wave against 512 MFMAs on the K = 256 update. (Loading C at the
  // start of the last k-stage instead measured 18 % slower on that update: 214 VGPRs; a persistent
  // grid with cross-tile DMA prefetch measured 5 % slower; profiles/gemm_mid_r06.jsonl.)
  const bool fast = full && ldc < (1 << 23);
  auto step = [&](int64_t t, const GmFrag<WMB, WNB>& Fc, GmFrag<WMB, WNB>& Fn) {
    if (t + AHEAD < nk) stage(t + AHEAD, !(tail && t + AHEAD == nk - 1));
    mma_half(Fc, 0);
    if (t + 1 < nk) {
      ready(t + 1);
      load(Fn, t + 1);
    }
    mma_half(Fc, 1);
  };

  GmFrag<WMB, WNB> F0, F1;
  if (GSZ == 2 && NBUF == 4 && !tail && nk % 2 == 0) {
    stage(0, true);
    stage(1, true);
    for (int64_t t = 0; t < nk; t += 2) {
      // stages t, t + 1 are this wave's only DMAs in flight: landed, and past the barrier every
      // wave has landed its pieces and finished reading stages t - 2, t - 1 (the slots refilled now)
      gm_wait_barrier<0>();
      load(F0, t);
      const bool more = t + 2 < nk;
      if (more) stage(t + 2, true);
      mma_half(F0, 0);
      if (more) stage(t + 3, true);
      load(F1, t + 1);
      mma_half(F0, 1);
      mma_half(F1, 0);
      mma_half(F1, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
  for (int64_t t = 0; t < AHEAD && t < nk; ++t) stage(t, !(tail && t == nk - 1));
  if (nk > 0) {
    ready(0);
    load(F0, 0);
  }
  int64_t t = 0;
  // the unconditional form of steps t and t + 1 needs stage t + 1 + AHEAD whole (not the tail)
  const int64_t nfull = nk - (tail ? 1 : 0);
  for (; t + AHEAD + 1 < nfull; t += 2) {
    step_full(t, F0, F1);
    step_full(t + 1, F1, F0);
  }
  for (; t < nk; t += 2) {
    step(t, F0, F1);
    if (t + 1 < nk) step(t + 1, F1, F0);
  }
  }

  // epilogue: element (bm, bn, g) -> C[m0 + crow(bm, g)][n0 + ccol(bn)]
  if (fast) {
    float* Ct = C + m0 * ldc + n0;
    const int l = (int)ldc;
    // one accumulator row's C values (32 loads in flight) before its stores
#pragma unroll
    for (int bm = 0; bm < WMB; ++bm) {
      float cv[WNB][16];
      if (beta) {
#pragma unroll
        for (int bn = 0; bn < WNB; ++bn)
#pragma unroll
          for (int g = 0; g < 16; ++g) cv[bn][g] = Ct[crow(bm, g) * l + ccol(bn)];
      }
#pragma unroll
      for (int bn = 0; bn < WNB; ++bn)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          float v = alpha * acc[bm][bn][g];
          if (beta) v += cv[bn][g];
          Ct[crow(bm, g) * l + ccol(bn)] = v;
        }
    }
    return;
  }
#pragma unroll
  for (int bm = 0; bm < WMB; ++bm) {
    float cv[WNB][16];
    if (beta) {
#pragma unroll
      for (int bn = 0; bn < WNB; ++bn) {
        const int64_t gc = n0 + ccol(bn);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int64_t gr = m0 + crow(bm, g);
          cv[bn][g] = (gr < M && gc < N) ? C[gr * ldc + gc] : 0.f;
        }
      }
    }
#pragma unroll
    for (int bn = 0; bn < WNB; ++bn) {
      const int64_t gc = n0 + ccol(bn);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int64_t gr = m0 + crow(bm, g);
        float v = alpha * acc[bm][bn][g];
        if (beta) v += cv[bn][g];
        if (gr < M && gc < N) C[gr * ldc + gc] = v;
      }
    }
  }
}

template <bool AK, bool BK_>
int f32m_launch(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, float alpha, int beta, int64_t slices, int64_t cslice, int wide, hipStream_t s) {
  const int64_t tm = wide == 1 ? 256 : wide == 2 ? 64 : MB, tnn = wide == 2 || wide == 3 ? 64 : MB;
  const int64_t tiles = ((M + tm - 1) / tm) * ((N + tnn - 1) / tnn);
  const int64_t nk = (K + MK - 1) / MK, kps = (nk + slices - 1) / slices;
  const int64_t ns = (nk + kps - 1) / kps;
  if (tiles > 0x7fffffffLL || ns > 65535) return HA_UNSUPPORTED;
  const dim3 g((unsigned)tiles, (unsigned)ns), b(256);
  if (wide == 2)
    hipLaunchKernelGGL((gemm_f32m<AK, BK_, 1, 4, 1>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps,
                       cslice);
  else if (wide == 3)
    hipLaunchKernelGGL((gemm_f32m<AK, BK_, 2, 4, 1>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps,
                       cslice);
  else if (wide == 4)
    hipLaunchKernelGGL((gemm_f32m<AK, BK_, 2, 4, 2, 2>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta,
                       kps, cslice);
  else if (wide)
    hipLaunchKernelGGL((gemm_f32m<AK, BK_, 4, 3>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
  else
    hipLaunchKernelGGL((gemm_f32m<AK, BK_, 2, 4>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
  return ha_launch_status();
}

}  // namespace

// The number of K slices ha_gemm_f32m launches for (K, slices): ceil(nk / ceil(nk / slices)),
// nk = ceil(K / 16).
HA_EXPORT int64_t ha_gemm_f32m_slices(int64_t K, int64_t slices) {
  const int64_t nk = (K + MK - 1) / MK;
  if (nk <= 0 || slices < 1) return 1;
  const int64_t kps = (nk + slices - 1) / slices;
  return (nk + kps - 1) / kps;
}

// C[M, N] (row-major, ldc) = alpha A B (+ C if beta), exact fp32 products and accumulation.
// a_kmajor: A element (m, k) at A[k lda + m] (else A[m lda + k]); b_kmajor: B element (k, n) at
// B[k ldb + n] (else B[n ldb + k]). slices > 1: split-K over 16-k stages, slice y -> C + y cslice
// (beta must be 0; the caller sums the partials). tile: 0 auto, 1 128 x 128, 2 256 x 128, 3 64 x 64,
// 5 128 x 128 with a barrier per PAIR of 16-k stages (A/B), 4 128 x 64 (A/B only: slower than the 128 x 128 or 64 x 64 form at every square and update shape,
// profiles/gemm_mid_r06.jsonl r6v rows).
// Requirements (else HA_UNSUPPORTED): 16-byte
// aligned A and B, lda and ldb multiples of 4, the contiguous extent of each operand (K for a
// k-contiguous one, M / N for the other) a multiple of 4, M, N, K >= 4.
HA_EXPORT int ha_gemm_f32m(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, float alpha, int beta, int64_t slices,
                           int64_t cslice, int tile, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C || slices < 1) return HA_BAD_ARG;
  if (slices > 1 && beta) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  if (K < 4 || M < 4 || N < 4 || lda % 4 || ldb % 4 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return HA_UNSUPPORTED;
  if ((a_kmajor ? M : K) % 4 || (b_kmajor ? N : K) % 4) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  // tile 1: 128 x 128, 2: 256 x 128 (wide), 0: 128 x 128 unless HEAT_GM_WIDE=1. The wide tile
  // measured slower on every shape (71 vs 84 % MFMA-busy at 6144^3, update 25.2 vs 23.3 ms;
  // profiles/gemm_mid_r06.jsonl, r6j rows): an A/B form only
  static const int wide_env = getenv("HEAT_GM_WIDE") ? atoi(getenv("HEAT_GM_WIDE")) : 0;
  const int wide = tile == 5 ? 4 : tile == 4 ? 3 : tile == 3 ? 2 : tile == 2 ? 1 : tile == 1 ? 0 : wide_env;
#define HA_F32M(AK, BK) return f32m_launch<AK, BK>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, slices, cslice, wide, s)
  if (a_kmajor) {
    if (b_kmajor) HA_F32M(true, true);
    HA_F32M(true, false);
  }
  if (b_kmajor) HA_F32M(false, true);
  HA_F32M(false, false);
#undef HA_F32M
}
