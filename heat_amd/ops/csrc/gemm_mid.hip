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

// at most N of this wave's vector-memory ops outstanding, LDS ops retired, then the barrier
template <int N>
__device__ __forceinline__ void gm_wait_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void gm_vm_wait() {
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One operand's staging for this lane. KC (k-contiguous, [rows][K] with leading dimension ld):
// piece q = k-chunk q >> 1 (4 k), rows 64 (q & 1) + lane; image [4 chunks][128 rows][4] - piece q
// at q KB. Else row-contiguous ([K][rows]): piece q = k-rows 2 q + (lane >> 5), 4 rows
// 4 (lane & 31) .. + 3; image [16 k][128 rows] at 512 B per k-row - piece q at q KB too.
// Out-of-range rows are clamped (their results are masked at the store).
template <bool KC>
struct GmSrc {
  const float* rp[2];  // KC: this lane's row of each 64-row group
  const float* cp;     // row-contiguous: this lane's 4-row group at k = lane >> 5
  int64_t ld;
  __device__ __forceinline__ void init(const float* P, int64_t ld_, int64_t rows, int64_t r0, int lane) {
    ld = ld_;
    if (KC) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int64_t row = r0 + 64 * g + lane;
        rp[g] = P + (row < rows ? row : rows - 1) * ld;
      }
    } else {
      int64_t c = r0 + 4 * (lane & 31);
      c = c + 4 <= rows ? c : rows - 4;
      cp = P + (int64_t)(lane >> 5) * ld + c;
    }
  }
  // source of piece q of the stage at k0 (whole stage in range)
  __device__ __forceinline__ const float* src(int64_t k0, int q) const {
    return KC ? rp[q & 1] + k0 + 4 * (q >> 1) : cp + (k0 + 2 * q) * ld;
  }
  // the same with the k index clamped into [0, K) (the tail stage; the clamped entries are zeroed
  // after they land). KC requires K % 4 == 0.
  __device__ __forceinline__ const float* src_clamped(int64_t k0, int q, int64_t K, int lane) const {
    if (KC) {
      const int64_t k = k0 + 4 * (q >> 1) + 4 <= K ? k0 + 4 * (q >> 1) : K - 4;
      return rp[q & 1] + k;
    }
    const int64_t k = k0 + 2 * q + (lane >> 5);
    return cp + ((k < K ? k : K - 1) - (lane >> 5)) * ld;
  }
  __device__ __forceinline__ bool beyond(int64_t k0, int q, int64_t K, int lane) const {
    return KC ? k0 + 4 * (q >> 1) >= K : k0 + 2 * q + (lane >> 5) >= K;
  }
};

// Fragments of one stage for a wave: a[b][s], bb[b][s] = block b's operand at k = 8 h + s.
struct GmFrag {
  float a[2][8], b[2][8];
};

// AK: A k-major ([K][M], m contiguous) - else row-major ([M][K], k contiguous).
// BK_: B k-major ([K][N], n contiguous) - else n-major ([N][K], k contiguous).
// NBUF: ring slots (4: 64 KB, two workgroups per CU).
template <bool AK, bool BK_, int NBUF>
__global__ __launch_bounds__(256, 2) void gemm_f32m(const float* __restrict__ A,
                                                                      const float* __restrict__ B,
                                                                      float* __restrict__ C, int64_t M, int64_t N,
                                                                      int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                                                                      float alpha, int beta, int64_t kps,
                                                                      int64_t cslice) {
  constexpr int AHEAD = NBUF - 1;   // stages in flight
  constexpr int DPS = 4;            // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * MSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r = lane & 31;
  const unsigned tn = (unsigned)((N + MB - 1) / MB), tm = (unsigned)((M + MB - 1) / MB);
  const unsigned bid = gm_xcd_remap(blockIdx.x, tm * tn);
  constexpr unsigned GM = 8;
  const unsigned grp = bid / (GM * tn), gfirst = grp * GM;
  const unsigned gsz = tm - gfirst < GM ? tm - gfirst : GM;
  const int64_t m0 = (int64_t)(gfirst + (bid % (GM * tn)) % gsz) * MB, n0 = (int64_t)((bid % (GM * tn)) / gsz) * MB;
  // split-K: slice blockIdx.y = k in [y kps MK, min((y + 1) kps MK, K)) into C + y cslice
  {
    const int64_t k0 = (int64_t)blockIdx.y * kps * MK;
    A += AK ? k0 * lda : k0;
    B += BK_ ? k0 * ldb : k0;
    K = K - k0 < kps * MK ? K - k0 : kps * MK;
    C += (int64_t)blockIdx.y * cslice;
  }
  GmSrc<!AK> sa;
  GmSrc<!BK_> sb;
  sa.init(A, lda, M, m0, lane);
  sb.init(B, ldb, N, n0, lane);
  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;

  auto stage = [&](int64_t t, bool full) {
    const unsigned dst = sbase + (unsigned)((t % NBUF) * MSTAGE);
    const int64_t k0 = t * MK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = 2 * wave + i;
      gm_dma16(full ? sa.src(k0, q) : sa.src_clamped(k0, q, K, lane), dst + q * 1024);
      gm_dma16(full ? sb.src(k0, q) : sb.src_clamped(k0, q, K, lane), dst + MOP + q * 1024);
    }
  };
  auto zero_tail = [&](int64_t t) {
    unsigned char* dst = smem + (t % NBUF) * MSTAGE;
    const int64_t k0 = t * MK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = 2 * wave + i;
      if (sa.beyond(k0, q, K, lane)) *reinterpret_cast<floatx4*>(dst + q * 1024 + lane * 16) = (floatx4)(0.f);
      if (sb.beyond(k0, q, K, lane)) *reinterpret_cast<floatx4*>(dst + MOP + q * 1024 + lane * 16) = (floatx4)(0.f);
    }
  };

  // fragment reads. k-contiguous operand, block b: row 32 b + r of the wave's 64, k-chunks 2 h and
  // 2 h + 1 (two ds_read_b128). Row-contiguous: rows 2 r, 2 r + 1 of the wave's 64 (blocks 0, 1)
  // at k-row 8 h + s (one ds_read_b64 per s).
  auto load = [&](GmFrag& F, int64_t t) {
    const unsigned char* base = smem + (t % NBUF) * MSTAGE;
    auto opnd = [&](const unsigned char* b, int w0, bool kc, float (&o)[2][8]) __attribute__((always_inline)) {
      if (kc) {
#pragma unroll
        for (int bl = 0; bl < 2; ++bl) {
          const int row = w0 + 32 * bl + r;
          const floatx4 x0 = *reinterpret_cast<const floatx4*>(b + (2 * h) * 2048 + row * 16);
          const floatx4 x1 = *reinterpret_cast<const floatx4*>(b + (2 * h + 1) * 2048 + row * 16);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            o[bl][s] = x0[s];
            o[bl][4 + s] = x1[s];
          }
        }
      } else {
        typedef float floatx2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const floatx2 v = *reinterpret_cast<const floatx2*>(b + (8 * h + s) * 512 + (w0 + 2 * r) * 4);
          o[0][s] = v[0];
          o[1][s] = v[1];
        }
      }
    };
    opnd(base, wm * 64, !AK, F.a);
    opnd(base + MOP, wn * 64, !BK_, F.b);
  };

  // accumulator (block bm, bn) element g <-> tile row / column (see the header)
  auto crow = [&](int bm, int g) -> int {
    const int rho = (g & 3) + 8 * (g >> 2) + 4 * h;
    return wm * 64 + (AK ? 2 * rho + bm : 32 * bm + rho);
  };
  auto ccol = [&](int bn) -> int { return wn * 64 + (BK_ ? 2 * r + bn : 32 * bn + r); };

  floatx16 acc[2][2];
  const bool full = m0 + MB <= M && n0 + MB <= N;
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) acc[bm][bn] = (floatx16)(0.f);

  auto mma_row = [&](const GmFrag& F, int bm) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(F.a[bm][s], F.b[bn][s], acc[bm][bn], 0, 0, 0);
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
  // steady state: stage t + AHEAD issued (whole, in range), MFMAs of block row 0 around it, the
  // counted wait for stage t + 1 + barrier, then stage t + 1's fragment reads between block row
  // 1's MFMAs
  auto step_full = [&](int64_t t, const GmFrag& Fc, GmFrag& Fn) {
    stage(t + AHEAD, true);
    mma_row(Fc, 0);
#pragma unroll
    for (int q = 0; q < DPS; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (the asm DMA)
    }
    __builtin_amdgcn_sched_barrier(0);
    gm_wait_barrier<(AHEAD - 1) * DPS>();
    load(Fn, t + 1);
    mma_row(Fc, 1);
    __builtin_amdgcn_sched_barrier(0);
  };
  // whole tiles with 128 ldc < 2^31: a uniform 64-bit tile base + 32-bit lane offsets in the
  // epilogue (the row terms dr ldc are scalar products), no bounds tests - the 64-bit per-element
  // form was ~1000 VALU per tile-wave against 512 MFMAs on the K = 256 update. (Loading C at the
  // start of the last k-stage instead measured 18 % slower on that update: 214 VGPRs;
  // profiles/gemm_mid_r06.jsonl.)
  const bool fast = full && ldc < (1 << 23);
  auto step = [&](int64_t t, const GmFrag& Fc, GmFrag& Fn) {
    if (t + AHEAD < nk) stage(t + AHEAD, !(tail && t + AHEAD == nk - 1));
    mma_row(Fc, 0);
    if (t + 1 < nk) {
      ready(t + 1);
      load(Fn, t + 1);
    }
    mma_row(Fc, 1);
  };

  GmFrag F0, F1;
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

  // epilogue: element (bm, bn, g) -> C[m0 + crow(bm, g)][n0 + ccol(bn)]
  if (fast) {
    float* Ct = C + m0 * ldc + n0;
    const int l = (int)ldc;
    // one accumulator row's C values (32 loads in flight) before its stores
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
      float cv[2][16];
      if (beta) {
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
          for (int g = 0; g < 16; ++g) cv[bn][g] = Ct[crow(bm, g) * l + ccol(bn)];
      }
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
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
  for (int bm = 0; bm < 2; ++bm) {
    float cv[2][16];
    if (beta) {
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) {
        const int64_t gc = n0 + ccol(bn);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int64_t gr = m0 + crow(bm, g);
          cv[bn][g] = (gr < M && gc < N) ? C[gr * ldc + gc] : 0.f;
        }
      }
    }
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
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

// Persistent form (one slice, K % 32 == 0, at least two workgroups' worth of tiles per CU): a
// grid of two workgroups per CU, each walking its tiles as ONE stream of k-stages, so the DMA of
// the next tile's first stages is in flight during the current tile's last MFMAs and its epilogue.
// With one launch-wide grid of equal tiles the two workgroups of a CU start and finish together:
// their prologue (stage-0 latency) and epilogue (C traffic) phases coincide and leave the SIMDs
// idle, which 16-stage tiles (the Householder update, K = 256) cannot amortise.
// Tile order: XCD x = blockIdx % 8 owns the contiguous logical tiles [x Tx, (x + 1) Tx) (grouped
// GM-row-panel order inside), workgroup j of that XCD takes every Gx-th of them.
// Wait counting across the epilogue: the epilogue drains vmcnt (after its first C loads), so every
// stage DMA'd before it has landed - those stages' readies skip the vmcnt and only barrier; the
// stages DMA'd after it are counted as usual (the epilogue's stores are older than them, and two
// stages later they are long acknowledged).
template <bool AK, bool BK_>
__global__ __launch_bounds__(256, 2) void gemm_f32m_p(const float* __restrict__ A, const float* __restrict__ B,
                                                       float* __restrict__ C, int64_t M, int64_t N, int64_t K,
                                                       int64_t lda, int64_t ldb, int64_t ldc, float alpha, int beta) {
  constexpr int NBUF = 4, AHEAD = 3, DPS = 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * MSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r = lane & 31;
  const unsigned tn = (unsigned)((N + MB - 1) / MB), tm = (unsigned)((M + MB - 1) / MB);
  const unsigned tiles = tm * tn;
  const unsigned x = blockIdx.x % 8, j = blockIdx.x / 8, Gx = gridDim.x / 8;
  const unsigned Tx = (tiles + 7) / 8, tbeg = x * Tx;
  const unsigned tend = tbeg + Tx < tiles ? tbeg + Tx : tiles;
  const unsigned ntl = tbeg + j < tend ? (tend - tbeg - j + Gx - 1) / Gx : 0;
  const int64_t nk = K / MK;
  const int64_t TT = (int64_t)ntl * nk;
  if (TT == 0) return;
  constexpr unsigned GM = 8;
  auto tile_of = [&](int64_t i, int64_t& m0, int64_t& n0) {
    const unsigned L = tbeg + j + (unsigned)i * Gx;
    const unsigned grp = L / (GM * tn), gfirst = grp * GM;
    const unsigned gsz = tm - gfirst < GM ? tm - gfirst : GM;
    m0 = (int64_t)(gfirst + (L % (GM * tn)) % gsz) * MB;
    n0 = (int64_t)((L % (GM * tn)) / gsz) * MB;
  };
  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  GmSrc<!AK> sa;
  GmSrc<!BK_> sb;
  int64_t dT = 0;   // next stage to DMA
  auto issue = [&]() {
    if (dT < TT) {
      const int64_t ks = dT % nk;
      if (ks == 0) {
        int64_t dm0, dn0;
        tile_of(dT / nk, dm0, dn0);
        sa.init(A, lda, M, dm0, lane);
        sb.init(B, ldb, N, dn0, lane);
      }
      const unsigned dst = sbase + (unsigned)((dT % NBUF) * MSTAGE);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = 2 * wave + i;
        gm_dma16(sa.src(ks * MK, q), dst + q * 1024);
        gm_dma16(sb.src(ks * MK, q), dst + MOP + q * 1024);
      }
    }
    ++dT;
  };
  auto load = [&](GmFrag& F, int64_t t) {
    const unsigned char* base = smem + (t % NBUF) * MSTAGE;
    auto opnd = [&](const unsigned char* b, int w0, bool kc, float (&o)[2][8]) __attribute__((always_inline)) {
      if (kc) {
#pragma unroll
        for (int bl = 0; bl < 2; ++bl) {
          const int row = w0 + 32 * bl + r;
          const floatx4 x0 = *reinterpret_cast<const floatx4*>(b + (2 * h) * 2048 + row * 16);
          const floatx4 x1 = *reinterpret_cast<const floatx4*>(b + (2 * h + 1) * 2048 + row * 16);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            o[bl][s] = x0[s];
            o[bl][4 + s] = x1[s];
          }
        }
      } else {
        typedef float floatx2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const floatx2 v = *reinterpret_cast<const floatx2*>(b + (8 * h + s) * 512 + (w0 + 2 * r) * 4);
          o[0][s] = v[0];
          o[1][s] = v[1];
        }
      }
    };
    opnd(base, wm * 64, !AK, F.a);
    opnd(base + MOP, wn * 64, !BK_, F.b);
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) acc[bm][bn] = (floatx16)(0.f);
  auto mma_row = [&](const GmFrag& F, int bm) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(F.a[bm][s], F.b[bn][s], acc[bm][bn], 0, 0, 0);
  };

  int64_t landed = -1;   // every stage <= landed is known to be in LDS (an epilogue drained vmcnt)
  auto ready = [&](int64_t t) {
    const int64_t later = dT - 1 - t;   // stages DMA'd after t (dT - 1: the last one issued)
    if (t <= landed) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else if (later >= 2) {
      gm_wait_barrier<2 * DPS>();
    } else if (later == 1) {
      gm_wait_barrier<DPS>();
    } else {
      gm_wait_barrier<0>();
    }
  };
  auto epilogue = [&](int64_t i) {
    int64_t m0, n0;
    tile_of(i, m0, n0);
    // lane coordinates made opaque per tile: otherwise the compiler hoists all 64 element
    // offsets (64-bit) out of the tile loop and spills them
    int he = h, re = r;
    asm volatile("" : "+v"(he), "+v"(re));
    auto crow = [&](int bm, int g) -> int {
      const int rho = (g & 3) + 8 * (g >> 2) + 4 * he;
      return wm * 64 + (AK ? 2 * rho + bm : 32 * bm + rho);
    };
    auto ccol = [&](int bn) -> int { return wn * 64 + (BK_ ? 2 * re + bn : 32 * bn + re); };
    const bool full = m0 + MB <= M && n0 + MB <= N;
    if (full && ldc < (1 << 23)) {
      float* Ct = C + m0 * ldc + n0;
      const unsigned l = (unsigned)ldc;
#pragma unroll
      for (int bm = 0; bm < 2; ++bm) {
        float cv[2][16];
        if (beta) {
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
#pragma unroll
            for (int g = 0; g < 16; ++g) cv[bn][g] = Ct[(unsigned)crow(bm, g) * l + (unsigned)ccol(bn)];
        }
        if (bm == 0) gm_vm_wait<0>();
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            float v = alpha * acc[bm][bn][g];
            if (beta) v += cv[bn][g];
            Ct[(unsigned)crow(bm, g) * l + (unsigned)ccol(bn)] = v;
          }
      }
    } else {
      gm_vm_wait<0>();
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) {
          const int64_t gc = n0 + ccol(bn);
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int64_t gr = m0 + crow(bm, g);
            if (gr < M && gc < N) {
              float v = alpha * acc[bm][bn][g];
              if (beta) v += C[gr * ldc + gc];
              C[gr * ldc + gc] = v;
            }
          }
        }
    }
    landed = dT - 1;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) acc[bm][bn] = (floatx16)(0.f);
  };
  auto body = [&](int64_t t, const GmFrag& Fc, GmFrag& Fn) {
    issue();            // stage t + AHEAD (of this tile or the next)
    mma_row(Fc, 0);
    if (t + 1 < TT) {
      ready(t + 1);
      load(Fn, t + 1);
    }
    mma_row(Fc, 1);
  };

  // nk even (host: K % 32 == 0): every tile starts with its fragments in F0
  GmFrag F0, F1;
  for (int q = 0; q < AHEAD; ++q) issue();
  ready(0);
  load(F0, 0);
  int64_t t = 0;
  for (unsigned i = 0; i < ntl; ++i) {
    for (int64_t ks = 0; ks < nk; ks += 2, t += 2) {
      body(t, F0, F1);
      body(t + 1, F1, F0);
    }
    epilogue(i);
  }
}

template <bool AK, bool BK_>
int f32m_launch(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, float alpha, int beta, int64_t slices, int64_t cslice, hipStream_t s) {
  // (a three-slot ring with three workgroups per CU measured 2-4 % slower with the 32-bit-offset
  // epilogue, profiles/gemm_mid_r06.jsonl, and spills with the early C loads: not instantiated)
  const int64_t tiles = ((M + MB - 1) / MB) * ((N + MB - 1) / MB);
  const int64_t nk = (K + MK - 1) / MK, kps = (nk + slices - 1) / slices;
  const int64_t ns = (nk + kps - 1) / kps;
  if (tiles > 0x7fffffffLL || ns > 65535) return HA_UNSUPPORTED;
  // persistent grid: HEAT_GM_PERSIST=n from n tiles per CU on
  // (A/B: measured 5 % slower than the one-tile-per-workgroup grid on the K = 256 update,
  // profiles/gemm_mid_r06.jsonl - off by default)
  static const int pmin = getenv("HEAT_GM_PERSIST") ? atoi(getenv("HEAT_GM_PERSIST")) : 0;
  static const int ncu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  if (pmin > 0 && ns == 1 && K % (2 * MK) == 0 && tiles >= (int64_t)pmin * ncu) {
    const unsigned G = (unsigned)(2 * ((ncu + 3) / 4) * 4);   // two per CU, a multiple of 8
    hipLaunchKernelGGL((gemm_f32m_p<AK, BK_>), dim3(G), dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta);
    return ha_launch_status();
  }
  const dim3 g((unsigned)tiles, (unsigned)ns), b(256);
  hipLaunchKernelGGL((gemm_f32m<AK, BK_, 4>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
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
// (beta must be 0; the caller sums the partials). Requirements (else HA_UNSUPPORTED): 16-byte
// aligned A and B, lda and ldb multiples of 4, the contiguous extent of each operand (K for a
// k-contiguous one, M / N for the other) a multiple of 4, M, N, K >= 4.
HA_EXPORT int ha_gemm_f32m(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, float alpha, int beta, int64_t slices,
                           int64_t cslice, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C || slices < 1) return HA_BAD_ARG;
  if (slices > 1 && beta) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  if (K < 4 || M < 4 || N < 4 || lda % 4 || ldb % 4 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return HA_UNSUPPORTED;
  if ((a_kmajor ? M : K) % 4 || (b_kmajor ? N : K) % 4) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
#define HA_F32M(AK, BK) return f32m_launch<AK, BK>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, slices, cslice, s)
  if (a_kmajor) {
    if (b_kmajor) HA_F32M(true, true);
    HA_F32M(true, false);
  }
  if (b_kmajor) HA_F32M(false, true);
  HA_F32M(false, false);
#undef HA_F32M
}
