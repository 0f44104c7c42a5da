// 256 x 256-tile GEMMs on the gfx950 matrix cores, the hot path of ht.matmul,
// CholeskyQR2 and the Householder trailing update (reference hot loops: linalg/basics.py:1650-1732
// block GEMMs; linalg/qr.py:96, 353, 887, 942 tile QRs).
//
// Two kernels share one pipeline:
//   gemm_h3t  fp32 GEMM at fp16 matrix-core speed: D = hi_A hi_B + hi_A lo_B + lo_A hi_B over
//             fp16 planes of power-of-two row-scaled operands (3 v_mfma_f32_32x32x16_f16 per
//             fragment pair, fp32 accumulation), exact 2^-(eA_i + eB_j) unscale in the epilogue;
//   gemm_f32t exact fp32 on v_mfma_f32_32x32x2_f32 (a k-ordered fp32 fma chain per product).
//
// Pipeline (one 256-thread workgroup per CU, 4 waves of 128 x 128 = 4 x 4 accumulators of 32 x 32,
// 256 accumulator registers per lane):
//   * one K-stage = 32 KB of operands (h3: 4 fp16 planes x 256 rows x 16 k; f32: 2 fp32 operands
//     x 256 rows x 16 k), staged by LDS-DMA (global_load_lds_dwordx4, 1 KB per wave-instruction,
//     8 per wave per stage) into 4 LDS buffers (128 KB): 3 stages in flight, one raw s_barrier per
//     stage behind a COUNTED vmcnt (never vmcnt(0) in the loop), so the DMA of stage t+3 spans the
//     barriers of stages t+1 and t+2;
//   * fragments of stage t+1 are read (ds_read_b128, conflict-free images) into the second
//     register set while the MFMAs of stage t run;
//   * h3 operands arrive in a K8-panel layout [K/8][rows][8] written by the split kernels below,
//     so every DMA piece is a contiguous 1 KB (64 rows x 16 B) and the LDS image is
//     [plane][k-chunk][row][8 halfs]; rows padded to 256, K to 16 (zeros) - no edge code;
//   * f32 operands are read in place from any of the four layouts (no copy): a row-major
//     (k-contiguous) operand is imaged [k/4][row][4] (lane l of a piece reads 16 B of row l), a
//     k-major one [k][row] (a piece is one contiguous 1 KB k-row); out-of-range rows are clamped
//     (results masked), the K tail is zeroed in LDS after it lands. The k order inside an MFMA is
//     permuted (lane half h, step s <-> k = 8h + s) so a row-major fragment is two 16-B reads;
//   * XCD-aware block order: the blocks of one XCD walk the N tiles of one row panel, which is
//     then re-read from that XCD's L2.
#include "common.h"

#include <stdlib.h>

namespace {

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));

constexpr int TB = 256;        // block tile (rows and columns)
constexpr int TK = 16;         // K per stage
constexpr int TSTAGE = 32768;  // bytes per stage
constexpr int TNBUF = 4;       // LDS stage buffers
// bits of the kernels' ``upper`` argument
constexpr int TG_UPPER_TILES = 1;  // square C: only the 256-tiles on or above the diagonal
constexpr int TG_B_UPPER = 2;      // B upper triangular (B[k][n] = 0 for k > n): K clipped per column tile
constexpr int TG_PAIRED = 4;       // with TG_B_UPPER: one workgroup per column-tile pair (p, nbn - 1 - p)

__device__ __forceinline__ int64_t tg_xcd_remap(int64_t orig, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8, loc = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// (m0, n0) of workgroup blockIdx.x: all nbm x nbn tiles, or (upper, square grids) only the tiles
// with tile column >= tile row, enumerated row by row - then the XCD remap spreads the upper
// triangle's uneven rows evenly over the XCDs.
__device__ __forceinline__ void tg_tile(int64_t nbm, int64_t nbn, int upper, int64_t& m0, int64_t& n0) {
  if (!upper) {
    const int64_t bid = tg_xcd_remap(blockIdx.x, nbm * nbn);
    m0 = (bid / nbn) * 256;
    n0 = (bid % nbn) * 256;
    return;
  }
  int64_t bid = tg_xcd_remap(blockIdx.x, nbn * (nbn + 1) / 2), i = 0;
  while (bid >= nbn - i) { bid -= nbn - i; ++i; }
  m0 = i * 256;
  n0 = (i + bid) * 256;
}

__device__ __forceinline__ void tg_dma16(const void* src, unsigned char* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// wait until at most N of this wave's vector-memory ops are outstanding (its DMA of the stage
// about to be read has landed), retire LDS ops, then the workgroup barrier
// (sched_barrier(0) on both sides: register-only MFMAs would otherwise migrate across the
// asm statement, which only orders memory operations)
template <int N>
__device__ __forceinline__ void tg_wait_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void tg_wait_stage(int64_t t, int64_t nk) {
  // stage t has landed; stages t+1, t+2 (when they exist) may still be in flight (8 DMA per stage)
  if (t + 2 < nk) tg_wait_barrier<16>();
  else if (t + 1 < nk) tg_wait_barrier<8>();
  else tg_wait_barrier<0>();
}


// C tile store of a wave's 4 x 4 accumulators of 32 x 32 (row = (g & 3) + 8 (g >> 2) + 4 h,
// column = lane & 31 of each): C = alpha 2^-(eA + eB) acc (+ C if beta); es: the tile's row
// exponents [0, 256) and column exponents [256, 512) in LDS, or null (no scaling).
__device__ __forceinline__ void tg_store_tile(floatx16 (&acc)[4][4], float* __restrict__ C, int64_t M, int64_t N,
                                              int64_t ldc, int64_t m0, int64_t n0, int wm, int wn, int h, int r,
                                              float alpha, int beta, const int* es) {
  const bool full = m0 + TB <= M && n0 + TB <= N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = wm * 128 + i * 32 + 4 * h;
    int er[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) er[g] = es ? es[rl + (g & 3) + 8 * (g >> 2)] : 0;
    // beta: the C values of all four 32 x 32 blocks of this accumulator row are loaded before any
    // is used (64 loads in flight; the fragment registers are dead here), one memory round trip
    // per row instead of one per block
    float cv[4][16];
    if (beta) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t gn = n0 + wn * 128 + j * 32 + r;
        const bool colok = full || gn < N;
        const float* cb = C + (m0 + rl) * ldc + gn;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int dr = (g & 3) + 8 * (g >> 2);
          cv[j][g] = (colok && (full || m0 + rl + dr < M)) ? cb[dr * ldc] : 0.f;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = wn * 128 + j * 32 + r;
      const int64_t gn = n0 + cl;
      const bool colok = full || gn < N;
      const int ec = es ? es[256 + cl] : 0;
      float* cb = C + (m0 + rl) * ldc + gn;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int dr = (g & 3) + 8 * (g >> 2);
        float v = es ? ldexpf(acc[i][j][g], -(er[g] + ec)) : acc[i][j][g];
        v *= alpha;
        if (beta) v += cv[j][g];
        if (colok && (full || m0 + rl + dr < M)) cb[dr * ldc] = v;
      }
    }
    asm volatile("" ::: "memory");
  }
}

// ------------------------------------------------------------------------------------------ h3
struct H3Frag {
  halfx8 ah[4], al[4], bh[4], bl[4];
};

__global__ __launch_bounds__(256, 1) void gemm_h3t(const _Float16* __restrict__ Ahi, const _Float16* __restrict__ Alo,
                                                   const _Float16* __restrict__ Bhi, const _Float16* __restrict__ Blo,
                                                   const int* __restrict__ eA, const int* __restrict__ eB,
                                                   float* __restrict__ C, int64_t M, int64_t N, int64_t Kp,
                                                   int64_t Mp, int64_t Np, int64_t ldc, float alpha, int beta,
                                                   int upper, int64_t kps, int64_t cslice) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[TNBUF * TSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int64_t m0, n0;
  tg_tile(Mp / TB, Np / TB, upper & TG_UPPER_TILES, m0, n0);
  // split-K: slice blockIdx.y covers stages [y kps, min((y + 1) kps, Kp / TK)) into C + y cslice
  const int64_t t0 = (int64_t)blockIdx.y * kps;
  // B upper triangular: column tile n0 only needs k < n0 + 256 (the rest of K multiplies zeros)
  if (upper & TG_B_UPPER) Kp = Kp < n0 + TB ? Kp : n0 + TB;
  C += (int64_t)blockIdx.y * cslice;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r = lane & 31;

  // staging: wave w moves plane w (0 A hi, 1 A lo, 2 B hi, 3 B lo): 2 k-chunks x 4 pieces of 64 rows
  const _Float16* plane = wave == 0 ? Ahi : wave == 1 ? Alo : wave == 2 ? Bhi : Blo;
  const int64_t prow = wave < 2 ? Mp : Np;
  const _Float16* src0 = plane + ((wave < 2 ? m0 : n0) + lane) * 8 + 2 * t0 * prow * 8;
  auto stage = [&](int64_t t) {
    unsigned char* dst = smem + (t & (TNBUF - 1)) * TSTAGE + wave * 8192;
    const _Float16* s = src0 + (2 * t) * prow * 8;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
#pragma unroll
      for (int g = 0; g < 4; ++g) tg_dma16(s + (kc * prow + 64 * g) * 8, dst + kc * 4096 + g * 1024);
  };

  // fragment byte offsets in a stage buffer: plane p, k-chunk h, row
  const int offA = h * 4096 + (wm * 128 + r) * 16;
  const int offB = 2 * 8192 + h * 4096 + (wn * 128 + r) * 16;
  auto load = [&](H3Frag& F, int64_t t) {
    const unsigned char* b = smem + (t & (TNBUF - 1)) * TSTAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      F.bh[i] = *reinterpret_cast<const halfx8*>(b + offB + i * 512);
      F.bl[i] = *reinterpret_cast<const halfx8*>(b + offB + 8192 + i * 512);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      F.ah[i] = *reinterpret_cast<const halfx8*>(b + offA + i * 512);
      F.al[i] = *reinterpret_cast<const halfx8*>(b + offA + 8192 + i * 512);
    }
  };

  floatx16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (floatx16)(0.f);

  auto mma_row = [&](const H3Frag& F, int i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[i], F.bh[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bl[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bh[j], acc[i][j], 0, 0, 0);
    }
  };

  int64_t nk = Kp / TK - t0 < kps ? Kp / TK - t0 : kps;
  nk = nk > 0 ? nk : 0;   // a split-K slice wholly beyond a triangular B's clipped K stores zeros
  // Steady-state stage (t + 3 < nk, no branches, so the scheduler sees one region per half): the
  // DMA of stage t+3 issued between the first accumulator row's MFMAs, the counted wait for stage
  // t+1 + barrier, then stage t+1's 16 fragment reads spread between the other 36 MFMAs. Every
  // DMA / ds_read issues in the shadow of a 32-cycle MFMA instead of in front of the first one.
  auto step_full = [&](int64_t t, const H3Frag& Fc, H3Frag& Fn) {
    stage(t + 3);
    mma_row(Fc, 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (LDS-DMA)
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    tg_wait_barrier<16>();
    load(Fn, t + 1);
    mma_row(Fc, 1);
    mma_row(Fc, 2);
    mma_row(Fc, 3);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
    __builtin_amdgcn_sched_barrier(0);
  };
  // general stage (the last three): DMA / wait only for stages that exist
  auto step = [&](int64_t t, const H3Frag& Fc, H3Frag& Fn) {
    if (t + 3 < nk) stage(t + 3);
    mma_row(Fc, 0);
    if (t + 1 < nk) {
      tg_wait_stage(t + 1, nk);
      load(Fn, t + 1);
    }
    mma_row(Fc, 1);
    mma_row(Fc, 2);
    mma_row(Fc, 3);
  };

  H3Frag F0, F1;
  for (int64_t t = 0; t < 3 && t < nk; ++t) stage(t);
  if (nk > 0) {
    tg_wait_stage(0, nk);
    load(F0, 0);
  }
  int64_t t = 0;
  for (; t + 4 < nk; t += 2) {
    step_full(t, F0, F1);
    step_full(t + 1, F1, F0);
  }
  if (t < nk) {
    step(t, F0, F1);
    if (t + 1 < nk) {
      step(t + 1, F1, F0);
      if (t + 2 < nk) {
        step(t + 2, F0, F1);
        if (t + 3 < nk) step(t + 3, F1, F0);
      }
    }
  }

  // epilogue: the tile's 2 x 256 exponents through LDS (the stage buffers are free once every
  // wave passed this barrier), then C row = m0 + wm 128 + 32 i + (g & 3) + 8 (g >> 2) + 4 h,
  // column = n0 + wn 128 + 32 j + r
  __syncthreads();
  int* es = reinterpret_cast<int*>(smem);
  es[tid] = eA[m0 + tid];
  es[256 + tid] = eB[n0 + tid];
  __syncthreads();
  tg_store_tile(acc, C, M, N, ldc, m0, n0, wm, wn, h, r, alpha, beta, es);
}

// ------------------------------------------------------------------------------------------ f32
// AK: A k-major ([K][M], m contiguous) - else row-major ([M][K], k contiguous).
// BK_: B k-major ([K][N], n contiguous) - else n-major ([N][K], k contiguous).
// MI16: v_mfma_f32_16x16x4_f32 (8 x 8 accumulators of 16 x 16 per wave; lane group g = lane >> 4
// holds k = 4 g + s at step s) - else v_mfma_f32_32x32x2_f32 (4 x 4 of 32 x 32; lane half h holds
// k = 8 h + s). Same FLOP per clock; the chip holds a different clock on each shape.
constexpr int F32_KP = 1040;                 // k-row pitch of a k-major image (16 B pad: no 2-way conflict)
constexpr int F32_OP = 16 * F32_KP;          // bytes per operand per stage
constexpr int F32_STAGE = 2 * F32_OP;        // 33280
static_assert(TNBUF * F32_STAGE <= 160 * 1024, "LDS");

template <bool MI16>
struct F32Frag;
template <>
struct F32Frag<false> {
  float a[4][8], b[4][8];
};
template <>
struct F32Frag<true> {
  floatx4 a[8], b[8];
};

// One f32 operand's DMA sources for this lane: piece q (0..15) of a stage is k-row q of a k-major
// operand (4 consecutive rows per lane, 1 KB contiguous per piece) or k-chunk q >> 2 of row group
// q & 3 of a row-major one (16 B of row 64 (q & 3) + lane); rows clamped into range.
template <bool KM>
struct F32Src {
  const float* base;
  const float* rb[4];
  int64_t ld;
  static constexpr int stride = KM ? F32_KP : 1024;
  __device__ __forceinline__ void init(const float* P, int64_t ld_, int64_t rows, int64_t rbase, int lane) {
    ld = ld_;
    if (KM) {
      int64_t c = rbase + 4 * lane;
      base = P + (c + 4 <= rows ? c : rows - 4);
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t row = rbase + 64 * g + lane;
        rb[g] = P + (row < rows ? row : rows - 1) * ld;
      }
    }
  }
  __device__ __forceinline__ const float* src(int64_t k0, int q) const {
    return KM ? base + (k0 + q) * ld : rb[q & 3] + k0 + 4 * (q >> 2);
  }
  __device__ __forceinline__ const float* src_clamped(int64_t k0, int q, int64_t K) const {
    if (KM) {
      const int64_t k = k0 + q < K ? k0 + q : K - 1;
      return base + k * ld;
    }
    const int64_t k = k0 + 4 * (q >> 2) + 4 <= K ? k0 + 4 * (q >> 2) : K - 4;
    return rb[q & 3] + k;
  }
  __device__ __forceinline__ bool beyond(int64_t k0, int q, int64_t K) const {
    return KM ? k0 + q >= K : k0 + 4 * (q >> 2) >= K;
  }
};

// SP: every wave moves 4 pieces of A and 4 of B (pieces 4 wave .. 4 wave + 3 of each, interleaved)
// - else waves 0, 1 move A and waves 2, 3 move B.
// PRE: accumulate with alpha = +-1, C preloaded into the accumulators (beta == 2). PAIR: triangular
// B, one workgroup per column-tile pair (TG_PAIRED). Separate instantiations: the default kernels
// keep their register allocation.
template <bool AK, bool BK_, bool MI16, bool SP, bool PRE = false, bool PAIR = false>
__global__ __launch_bounds__(256, 1) void gemm_f32t(const float* __restrict__ A_, const float* __restrict__ B_,
                                                    float* __restrict__ C_, int64_t M, int64_t N, int64_t K_,
                                                    int64_t lda, int64_t ldb, int64_t ldc, float alpha, int beta,
                                                    int upper, int64_t kps, int64_t cslice) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[TNBUF * F32_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // B upper triangular + TG_PAIRED: the workgroup computes column tiles p and nbn - 1 - p of one
  // row panel one after the other - (p + 1) + (nbn - p) k-blocks, the same for every workgroup,
  // so the tiles an XCD runs at once stay in step over the shared A panel (with one tile per
  // workgroup the short tiles finish early and their successors re-stream A panels out of step)
  const int64_t nbm = (M + TB - 1) / TB, nbn = (N + TB - 1) / TB;
  constexpr bool paired = PAIR;
#pragma nounroll
  for (int pass = 0; pass < (paired ? 2 : 1); ++pass) {
  const float* A = A_;
  const float* B = B_;
  float* C = C_;
  int64_t K = K_;
  int64_t m0, n0;
  if constexpr (paired) {
    const int64_t np = (nbn + 1) / 2;
    const int64_t bid = tg_xcd_remap(blockIdx.x, nbm * np), pp = bid % np;
    const int64_t j = pass == 0 ? pp : nbn - 1 - pp;
    if (pass == 1) {
      if (j == pp) break;   // odd nbn: the middle tile has no partner
      __syncthreads();      // every wave is done with the first tile's stage buffers
    }
    m0 = (bid / np) * TB;
    n0 = j * TB;
  } else {
    tg_tile(nbm, nbn, upper & TG_UPPER_TILES, m0, n0);
  }
  // B upper triangular: column tile n0 only needs k < n0 + 256 (the rest of K multiplies zeros;
  // n0 + 256 is a multiple of 16, so no new K tail appears)
  if (upper & TG_B_UPPER) K = K < n0 + TB ? K : n0 + TB;
  // split-K: slice blockIdx.y = k in [y kps TK, min((y + 1) kps TK, K)) into C + y cslice
  {
    const int64_t k0 = (int64_t)blockIdx.y * kps * TK;
    A += AK ? k0 * lda : k0;
    B += BK_ ? k0 * ldb : k0;
    K = K - k0 < kps * TK ? K - k0 : kps * TK;
    K = K > 0 ? K : 0;   // a slice wholly beyond the clipped K: zero partial
    C += (int64_t)blockIdx.y * cslice;
  }
  const int wm = wave >> 1, wn = wave & 1;

  // staging: waves 0, 1 move A (16 pieces of 1 KB), waves 2, 3 move B. Piece q (0..15) of an
  // operand: row-major image -> k-chunk q >> 2, rows 64 (q & 3) + lane (at q KB); k-major -> k-row q
  // (at q F32_KP).
  const bool isA = wave < 2;
  const bool km = isA ? AK : BK_;
  const float* P = isA ? A : B;
  const int64_t ld = isA ? lda : ldb, rows = isA ? M : N, rbase = isA ? m0 : n0;
  const int half = wave & 1;  // pieces 8 half .. 8 half + 7
  int64_t rowoff[4];          // row-major images: this lane's clamped row of each 64-row group
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    int64_t row = rbase + 64 * g + lane;
    rowoff[g] = (row < rows ? row : rows - 1) * ld;
  }
  int64_t coloff = rbase + 4 * lane;  // k-major images: 4 consecutive rows (columns of memory)
  coloff = coloff + 4 <= rows ? coloff : rows - 4;
  auto stage = [&](int64_t t) {
    unsigned char* dst = smem + (t & (TNBUF - 1)) * F32_STAGE + (isA ? 0 : F32_OP);
    const int64_t k0 = t * TK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = 8 * half + i;
      if (km) {
        int64_t k = k0 + q;
        k = k < K ? k : K - 1;
        tg_dma16(P + k * ld + coloff, dst + q * F32_KP);
      } else {
        int64_t k = k0 + 4 * (q >> 2);
        k = k + 4 <= K ? k : K - 4;
        tg_dma16(P + rowoff[q & 3] + k, dst + q * 1024);
      }
    }
  };
  // steady-state staging (a whole in-range stage: no clamping, no branches) - the pointer of piece q
  // is lb[q & 3] + a uniform offset (q & 3 == i & 3 since 8 half has no low bits)
  const float* lb[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) lb[g] = P + (km ? coloff : rowoff[g]);
  // koff(q) = (k0 + q qa) lmul + (q >> 2) qb: k-major (1, ld, 0), row-major (0, 1, 4) - arithmetic on
  // wave-uniform integers, so A and B waves run the same branch-free code
  const int dstride = km ? F32_KP : 1024, qa = km ? 1 : 0, qb = km ? 0 : 4;
  const int64_t lmul = km ? ld : 1;
  const int opoff = isA ? 0 : F32_OP;
  auto stage_full = [&](int64_t t) {
    unsigned char* dst = smem + (t & (TNBUF - 1)) * F32_STAGE + opoff;
    const int64_t k0 = t * TK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = 8 * half + i;
      tg_dma16(lb[i & 3] + ((k0 + q * qa) * lmul + (q >> 2) * qb), dst + q * dstride);
    }
  };
  // zero the k >= K entries of this wave's pieces of the last stage (after its own DMA landed)
  auto zero_tail = [&](int64_t t) {
    unsigned char* dst = smem + (t & (TNBUF - 1)) * F32_STAGE + (isA ? 0 : F32_OP);
    const int64_t k0 = t * TK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = 8 * half + i;
      if (km) {
        if (k0 + q >= K) *reinterpret_cast<floatx4*>(dst + q * F32_KP + lane * 16) = (floatx4)(0.f);
      } else {
        if (k0 + 4 * (q >> 2) >= K) *reinterpret_cast<floatx4*>(dst + q * 1024 + lane * 16) = (floatx4)(0.f);
      }
    }
  };
  F32Src<AK> sa;
  F32Src<BK_> sb;
  if constexpr (SP) {
    sa.init(A, lda, M, m0, lane);
    sb.init(B, ldb, N, n0, lane);
  }
  auto stage_sp = [&](int64_t t, bool full) {
    unsigned char* dst = smem + (t & (TNBUF - 1)) * F32_STAGE;
    const int64_t k0 = t * TK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = 4 * wave + i;
      tg_dma16(full ? sa.src(k0, q) : sa.src_clamped(k0, q, K), dst + q * sa.stride);
      tg_dma16(full ? sb.src(k0, q) : sb.src_clamped(k0, q, K), dst + F32_OP + q * sb.stride);
    }
  };
  auto zero_tail_sp = [&](int64_t t) {
    unsigned char* dst = smem + (t & (TNBUF - 1)) * F32_STAGE;
    const int64_t k0 = t * TK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = 4 * wave + i;
      if (sa.beyond(k0, q, K)) *reinterpret_cast<floatx4*>(dst + q * sa.stride + lane * 16) = (floatx4)(0.f);
      if (sb.beyond(k0, q, K))
        *reinterpret_cast<floatx4*>(dst + F32_OP + q * sb.stride + lane * 16) = (floatx4)(0.f);
    }
  };

  auto load = [&](F32Frag<MI16>& F, int64_t t) {
    const unsigned char* b = smem + (t & (TNBUF - 1)) * F32_STAGE;
    if constexpr (MI16) {
      // lane (r16 = lane & 15, g = lane >> 4): rows of block i, k = 4 g + s
      const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ra = wm * 128 + i * 16 + r16, cb = wn * 128 + i * 16 + r16;
        if (AK) {
#pragma unroll
          for (int s = 0; s < 4; ++s) F.a[i][s] = *reinterpret_cast<const float*>(b + (4 * g + s) * F32_KP + ra * 4);
        } else {
          F.a[i] = *reinterpret_cast<const floatx4*>(b + (g * 256 + ra) * 16);
        }
        if (BK_) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            F.b[i][s] = *reinterpret_cast<const float*>(b + F32_OP + (4 * g + s) * F32_KP + cb * 4);
        } else {
          F.b[i] = *reinterpret_cast<const floatx4*>(b + F32_OP + (g * 256 + cb) * 16);
        }
      }
    } else {
      // lane (r, h): rows of block i, k = 8 h + s
      const int h = lane >> 5, r = lane & 31;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra = wm * 128 + i * 32 + r, cb = wn * 128 + i * 32 + r;
        if (AK) {
#pragma unroll
          for (int s = 0; s < 8; ++s) F.a[i][s] = *reinterpret_cast<const float*>(b + (8 * h + s) * F32_KP + ra * 4);
        } else {
          const floatx4 x0 = *reinterpret_cast<const floatx4*>(b + ((2 * h) * 256 + ra) * 16);
          const floatx4 x1 = *reinterpret_cast<const floatx4*>(b + ((2 * h + 1) * 256 + ra) * 16);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            F.a[i][s] = x0[s];
            F.a[i][4 + s] = x1[s];
          }
        }
        if (BK_) {
#pragma unroll
          for (int s = 0; s < 8; ++s)
            F.b[i][s] = *reinterpret_cast<const float*>(b + F32_OP + (8 * h + s) * F32_KP + cb * 4);
        } else {
          const floatx4 y0 = *reinterpret_cast<const floatx4*>(b + F32_OP + ((2 * h) * 256 + cb) * 16);
          const floatx4 y1 = *reinterpret_cast<const floatx4*>(b + F32_OP + ((2 * h + 1) * 256 + cb) * 16);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            F.b[i][s] = y0[s];
            F.b[i][4 + s] = y1[s];
          }
        }
      }
    }
  };

  // accumulators: MI16 8 x 8 of floatx4, else 4 x 4 of floatx16 (256 registers either way)
  floatx16 acc[4][4];
  floatx4 acc16[8][8];
  if constexpr (MI16) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc16[i][j] = (floatx4)(0.f);
  } else if (PRE) {
    // C enters the accumulators (acc = alpha C: exact for the host-checked alpha = +-1), loaded
    // before the first stage's DMA is issued, so the loads' latency hides under the prologue's
    // and the counted wait for stage 0 covers them; the epilogue then only STORES alpha acc =
    // C + alpha A B (a beta epilogue exposed one C load round trip per 32 x 32 block: 16 per tile,
    // which the short-K updates of the Householder QR - 16 k-stages per tile - could not hide)
    const int h = lane >> 5, r = lane & 31;
    const bool full = m0 + TB <= M && n0 + TB <= N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t rg = m0 + wm * 128 + i * 32 + 4 * h;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t gn = n0 + wn * 128 + j * 32 + r;
        const bool colok = full || gn < N;
        const float* cb = C + rg * ldc + gn;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int dr = (g & 3) + 8 * (g >> 2);
          acc[i][j][g] = (colok && (full || rg + dr < M)) ? alpha * cb[dr * ldc] : 0.f;
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (floatx16)(0.f);
  }

  // part p of a stage's MFMAs (p = 0: before the barrier, 1..3 after)
  auto mma_part = [&](const F32Frag<MI16>& F, int p) {
    if constexpr (MI16) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.a[i][p], F.b[j][p], acc16[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(F.a[p][s], F.b[j][s], acc[p][j], 0, 0, 0);
    }
  };

  const int64_t nk = (K + TK - 1) / TK;
  const bool tail = (K % TK) != 0;
  auto ready = [&](int64_t t) {  // stage t landed and visible to every wave
    if (tail && t == nk - 1) {
      if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (SP) zero_tail_sp(t);
      else zero_tail(t);
    }
    tg_wait_stage(t, nk);
  };
  // steady state (t + 3 < nk and stage t + 1 is not the zero-padded tail): branch-free, DMA and
  // fragment reads interleaved with the MFMAs (see gemm_h3t)
  auto step_full = [&](int64_t t, const F32Frag<MI16>& Fc, F32Frag<MI16>& Fn) {
    if constexpr (SP) stage_sp(t + 3, true);
    else stage_full(t + 3);
    mma_part(Fc, 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, MI16 ? 8 : 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
    }
    tg_wait_barrier<16>();
    load(Fn, t + 1);
    mma_part(Fc, 1);
    mma_part(Fc, 2);
    mma_part(Fc, 3);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, MI16 ? 6 : 3, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto step = [&](int64_t t, const F32Frag<MI16>& Fc, F32Frag<MI16>& Fn) {
    if (t + 3 < nk) {
      if constexpr (SP) stage_sp(t + 3, false);
      else stage(t + 3);
    }
    mma_part(Fc, 0);
    if (t + 1 < nk) {
      ready(t + 1);
      load(Fn, t + 1);
    }
    mma_part(Fc, 1);
    mma_part(Fc, 2);
    mma_part(Fc, 3);
  };

  F32Frag<MI16> F0, F1;
  for (int64_t t = 0; t < 3 && t < nk; ++t) {
    if constexpr (SP) stage_sp(t, false);
    else stage(t);
  }
  if (nk > 0) {
    ready(0);
    load(F0, 0);
  }
  int64_t t = 0;
  for (; t + 4 < nk; t += 2) {
    step_full(t, F0, F1);
    step_full(t + 1, F1, F0);
  }
  if (t < nk) {
    step(t, F0, F1);
    if (t + 1 < nk) {
      step(t + 1, F1, F0);
      if (t + 2 < nk) {
        step(t + 2, F0, F1);
        if (t + 3 < nk) step(t + 3, F1, F0);
      }
    }
  }

  if constexpr (MI16) {
    // 16 x 16 C/D map: column = lane & 15, row = 4 (lane >> 4) + reg
    const bool full = m0 + TB <= M && n0 + TB <= N;
    const int r16 = lane & 15, g4 = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t rb = m0 + wm * 128 + i * 16 + g4;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t gn = n0 + wn * 128 + j * 16 + r16;
        const bool colok = full || gn < N;
        float* cb = C + rb * ldc + gn;
        float cv[4];
        if (beta) {
#pragma unroll
          for (int g = 0; g < 4; ++g) cv[g] = (colok && (full || rb + g < M)) ? cb[g * ldc] : 0.f;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float v = alpha * acc16[i][j][g];
          if (beta) v += cv[g];
          if (colok && (full || rb + g < M)) cb[g * ldc] = v;
        }
      }
      asm volatile("" ::: "memory");
    }
  } else {
    tg_store_tile(acc, C, M, N, ldc, m0, n0, wm, wn, lane >> 5, lane & 31, alpha, PRE ? 0 : beta, nullptr);
  }
  }  // pass
}

// ------------------------------------------------------------------------ h3 operand splitting
// Exponent e such that max |row| * 2^e lies in [2^14, 2^15); 0 for zero / non-finite maxima.
__device__ __forceinline__ int tg_exp(float m) { return (m > 0.f && m <= 3.402823466e38f) ? 14 - ilogbf(m) : 0; }
__device__ __forceinline__ bool tg_bad(float v) { return !(fabsf(v) <= 3.402823466e38f); }

__device__ __forceinline__ void tg_split(float v, int e, _Float16& hi, _Float16& lo) {
  const float s = ldexpf(v, e);
  hi = (_Float16)s;
  lo = (_Float16)(s - (float)hi);
}

// Rows of X [R][C] (unit stride along C, leading dimension ld) -> planes [Kp/8][Rp][8] fp16 with a
// power-of-two scale per row; one workgroup per band of 64 rows: the band's row maxima first
// (the band, 64 x C floats, stays in L2 for the second pass), then 64 x 64 tiles transposed
// through LDS so every plane write is a contiguous 1 KB per wave. Rows >= R and k >= C are zero.
template <bool VEC>
__global__ __launch_bounds__(256) void tg_split_rows(const float* __restrict__ X, int64_t R, int64_t C, int64_t ld,
                                                     int64_t Rp, int64_t Kp, _Float16* __restrict__ hi,
                                                     _Float16* __restrict__ lo, int* __restrict__ ex,
                                                     int* __restrict__ flag) {
  __shared__ __attribute__((aligned(16))) _Float16 img[2][8][64][8];
  __shared__ int es[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  bool bad = false;
  for (int q = 0; q < 16; ++q) {
    const int row = wave * 16 + q;
    const int64_t gr = r0 + row;
    float m = 0.f;
    if (gr < R) {
      const float* p = X + gr * ld;
      if (VEC) {
        for (int64_t c = 4 * lane; c < C; c += 256) {
          const floatx4 v = *reinterpret_cast<const floatx4*>(p + c);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            bad |= tg_bad(v[u]);
            m = fmaxf(m, fabsf(v[u]));
          }
        }
      } else {
        for (int64_t c = lane; c < C; c += 64) {
          const float v = p[c];
          bad |= tg_bad(v);
          m = fmaxf(m, fabsf(v));
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) {
      const int e = tg_exp(m);
      es[row] = e;
      if (gr < Rp) ex[gr] = e;
    }
  }
  if (__ballot(bad) != 0ull && lane == 0) atomicOr(flag, 1);
  __syncthreads();
  for (int64_t k0 = 0; k0 < Kp; k0 += 64) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = tid + 256 * q, row = f >> 4, c4 = (f & 15) * 4;
      const int64_t gr = r0 + row, k = k0 + c4;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (gr < R) {
        const float* p = X + gr * ld + k;
        if (VEC) {
          if (k < C) {
            const floatx4 w = *reinterpret_cast<const floatx4*>(p);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = w[u];
          }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (k + u < C) v[u] = p[u];
        }
      }
      const int e = es[row];
      halfx4 hv, lv;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        _Float16 a, b;
        tg_split(v[u], e, a, b);
        hv[u] = a;
        lv[u] = b;
      }
      *reinterpret_cast<halfx4*>(&img[0][c4 >> 3][row][c4 & 7]) = hv;
      *reinterpret_cast<halfx4*>(&img[1][c4 >> 3][row][c4 & 7]) = lv;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = tid + 256 * q, pl = f >> 9, kc = (f >> 6) & 7, row = f & 63;
      const int64_t gk = k0 / 8 + kc;
      if (gk < Kp / 8) {
        _Float16* dst = (pl ? lo : hi) + (gk * Rp + r0 + row) * 8;
        *reinterpret_cast<halfx8*>(dst) = *reinterpret_cast<const halfx8*>(&img[pl][kc][row][0]);
      }
    }
    __syncthreads();
  }
}

// Columns of X [R][C] (contraction along the rows of X): planes [Kp/8][Cp][8], k = row of X,
// scale per column from the maxima mx (ha_split_absmax axis 1). Workgroup = 64 k x 64 columns.
__global__ __launch_bounds__(256) void tg_split_cols(const float* __restrict__ X, int64_t R, int64_t C, int64_t ld,
                                                     int64_t Cp, int64_t Kp, const float* __restrict__ mx,
                                                     _Float16* __restrict__ hi, _Float16* __restrict__ lo,
                                                     int* __restrict__ ex) {
  __shared__ __attribute__((aligned(16))) _Float16 img[2][8][64][8];
  const int tid = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * 64, k0 = (int64_t)blockIdx.y * 64;
  if (blockIdx.y == 0 && tid < 64 && c0 + tid < Cp) ex[c0 + tid] = c0 + tid < C ? tg_exp(mx[c0 + tid]) : 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int f = tid + 256 * q, kr = f >> 6, col = f & 63;
    const int64_t gk = k0 + kr, gc = c0 + col;
    float v = 0.f;
    int e = 0;
    if (gk < R && gc < C) {
      v = X[gk * ld + gc];
      e = tg_exp(mx[gc]);
    }
    _Float16 a, b;
    tg_split(v, e, a, b);
    img[0][kr >> 3][col][kr & 7] = a;
    img[1][kr >> 3][col][kr & 7] = b;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = tid + 256 * q, pl = f >> 9, kc = (f >> 6) & 7, col = f & 63;
    const int64_t gk = k0 / 8 + kc;
    if (gk < Kp / 8) {
      _Float16* dst = (pl ? lo : hi) + (gk * Cp + c0 + col) * 8;
      *reinterpret_cast<halfx8*>(dst) = *reinterpret_cast<const halfx8*>(&img[pl][kc][col][0]);
    }
  }
}

template <bool AK, bool BK_>
int f32t_launch(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, float alpha, int beta, int upper, int64_t slices, int64_t cslice, hipStream_t s) {
  // HEAT_GEMM_F32_SHAPE=16 selects the 16x16x4 MFMA shape, HEAT_GEMM_F32_SPREAD=0 the A-waves /
  // B-waves DMA split (A/B benchmarking)
  static const int shape = getenv("HEAT_GEMM_F32_SHAPE") ? atoi(getenv("HEAT_GEMM_F32_SHAPE")) : 32;
  static const int spread = getenv("HEAT_GEMM_F32_SPREAD") ? atoi(getenv("HEAT_GEMM_F32_SPREAD")) : 1;
  // beta with alpha = +-1 and one slice: C preloaded into the accumulators (beta = 2, 32 x 32
  // shape only) only with HEAT_GEMM_F32_PRELOAD=1 (A/B: 2x slower at K = 256 and 40x the error -
  // every partial sum rounds at the scale of C; profiles/update_ab_r06.jsonl)
  static const int preload = getenv("HEAT_GEMM_F32_PRELOAD") ? atoi(getenv("HEAT_GEMM_F32_PRELOAD")) : 0;
  // triangular B: one workgroup per column-tile pair; HEAT_GEMM_TRI_PAIRED=0 one tile each (A/B)
  static const int pair_env = getenv("HEAT_GEMM_TRI_PAIRED") ? atoi(getenv("HEAT_GEMM_TRI_PAIRED")) : 1;
  if (beta) beta = (preload && shape != 16 && slices == 1 && (alpha == 1.f || alpha == -1.f)) ? 2 : 1;
  const bool pair = (upper & TG_B_UPPER) && !(upper & TG_UPPER_TILES) && pair_env && shape != 16 && beta != 2;
  upper = pair ? (upper | TG_PAIRED) : (upper & ~TG_PAIRED);
  const int64_t nbm = (M + TB - 1) / TB, nbn = (N + TB - 1) / TB;
  const int64_t nwg = (upper & TG_UPPER_TILES) ? nbn * (nbn + 1) / 2 : pair ? nbm * ((nbn + 1) / 2) : nbm * nbn;
  if (nwg > 0x7FFFFFFF || slices > 65535) return HA_UNSUPPORTED;
  const int64_t nk = (K + TK - 1) / TK, kps = (nk + slices - 1) / slices;
  const dim3 grid((unsigned)nwg, (unsigned)((nk + kps - 1) / kps));
  if (shape == 16)
    hipLaunchKernelGGL((gemm_f32t<AK, BK_, true, false>), grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc,
                       alpha, beta, upper, kps, cslice);
  else if (beta == 2)
    hipLaunchKernelGGL((gemm_f32t<AK, BK_, false, true, true>), grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb,
                       ldc, alpha, beta, upper, kps, cslice);
  else if (pair)
    hipLaunchKernelGGL((gemm_f32t<AK, BK_, false, true, false, true>), grid, dim3(256), 0, s, A, B, C, M, N, K, lda,
                       ldb, ldc, alpha, beta, upper, kps, cslice);
  else if (spread)
    hipLaunchKernelGGL((gemm_f32t<AK, BK_, false, true>), grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc,
                       alpha, beta, upper, kps, cslice);
  else
    hipLaunchKernelGGL((gemm_f32t<AK, BK_, false, false>), grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc,
                       alpha, beta, upper, kps, cslice);
  return ha_launch_status();
}

__global__ __launch_bounds__(256) void tg_sum_slices(const float* __restrict__ P, int64_t S, int64_t M, int64_t N,
                                                     int64_t cslice, double* __restrict__ out, int64_t ldo, int upper,
                                                     int accumulate) {
  const int64_t total = M * N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / N, j = e - i * N;
    if (upper && j < i) continue;
    double acc = accumulate ? out[i * ldo + j] : 0.0;
    for (int64_t z = 0; z < S; ++z) acc += (double)P[z * cslice + e];
    out[i * ldo + j] = acc;
  }
}

// tg_sum_slices over groups of 4 consecutive columns (N, cslice multiples of 4, 16-byte aligned P):
// one 16-byte load per slice and 4 slices' loads in flight per thread, and with `upper` the
// groups wholly below the diagonal are never read (the scalar form read one float per thread per
// slice with one load in flight: ~0.5 TB/s on the Gram's slice sums)
__global__ __launch_bounds__(256) void tg_sum_slices4(const float* __restrict__ P, int64_t S, int64_t M, int64_t N,
                                                      int64_t cslice, double* __restrict__ out, int64_t ldo, int upper,
                                                      int accumulate) {
  const int64_t ng = N / 4, total = M * ng;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / ng, j0 = (e - i * ng) * 4;
    if (upper && j0 + 3 < i) continue;
    const floatx4* src = reinterpret_cast<const floatx4*>(P + i * N + j0);
    const int64_t cs4 = cslice / 4;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int64_t z = 0;
    for (; z + 4 <= S; z += 4) {
      floatx4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[(z + u) * cs4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a0 += (double)v[u][0];
        a1 += (double)v[u][1];
        a2 += (double)v[u][2];
        a3 += (double)v[u][3];
      }
    }
    for (; z < S; ++z) {
      const floatx4 v = src[z * cs4];
      a0 += (double)v[0];
      a1 += (double)v[1];
      a2 += (double)v[2];
      a3 += (double)v[3];
    }
    double* o = out + i * ldo + j0;
    const double acc[4] = {a0, a1, a2, a3};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (upper && j0 + u < i) continue;
      o[u] = accumulate ? o[u] + acc[u] : acc[u];
    }
  }
}

// fp32 out[i, j] = alpha * (sum over s of P[s cslice + i N + j], in slice order, fp64) (+ out): the
// split-K epilogue of a GEMM whose few output tiles cannot fill the GPU
__global__ __launch_bounds__(256) void tg_sum_slices32(const float* __restrict__ P, int64_t S, int64_t M, int64_t N,
                                                       int64_t cslice, float* __restrict__ out, int64_t ldo,
                                                       float alpha, int accumulate) {
  const int64_t total = M * N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / N, j = e - i * N;
    double acc = 0.0;
    for (int64_t z = 0; z < S; ++z) acc += (double)P[z * cslice + e];
    const float r = (float)(alpha * acc);
    out[i * ldo + j] = accumulate ? out[i * ldo + j] + r : r;
  }
}

}  // namespace

HA_EXPORT int ha_sum_slices32(const float* P, int64_t S, int64_t M, int64_t N, int64_t cslice, float* out, int64_t ldo,
                              float alpha, int accumulate, void* stream) {
  if (S < 1 || M < 0 || N < 0 || ldo < N) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  const int64_t g = (M * N + 255) / 256;
  hipLaunchKernelGGL(tg_sum_slices32, dim3((unsigned)(g < 16384 ? g : 16384)), dim3(256), 0, (hipStream_t)stream, P,
                     S, M, N, cslice, out, ldo, alpha, accumulate);
  return ha_launch_status();
}

// C[M, N] (row-major, ldc) = alpha A B (+ C if beta), exact fp32. a_kmajor: A element (m, k) at
// A[k lda + m] (else A[m lda + k]); b_kmajor: B element (k, n) at B[k ldb + n] (else B[n ldb + k]).
// Requirements (else HA_UNSUPPORTED, the caller uses ha_gemm_f32): 16-byte aligned bases, leading
// dimensions multiples of 4, the contiguous extent of each operand a multiple of 4, M, N >= 4.
// slices > 1: split-K - slice s of the K range (multiples of 16) goes to C + s cslice (partials
// for ha_sum_slices64). upper bit 1 (M == N): only the 256-tiles on or above the diagonal are
// computed; bit 2: B is upper triangular (B(k, n) = 0 for k > n, e.g. an R^-1 factor): column tile
// n0 runs its K loop only to min(K, n0 + 256) - the zero half of K is never loaded or multiplied.
HA_EXPORT int ha_gemm_f32t(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, float alpha, int beta, int upper,
                           int64_t slices, int64_t cslice, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C || slices < 1 || ((upper & TG_UPPER_TILES) && M != N)) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  if (K < 4 || M < 4 || N < 4 || lda % 4 || ldb % 4 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return HA_UNSUPPORTED;
  if ((a_kmajor ? M : K) % 4 || (b_kmajor ? N : K) % 4) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
#define HA_F32T(AK, BK) return f32t_launch<AK, BK>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, upper, slices, cslice, s)
  if (a_kmajor) {
    if (b_kmajor) HA_F32T(true, true);
    HA_F32T(true, false);
  }
  if (b_kmajor) HA_F32T(false, true);
  HA_F32T(false, false);
#undef HA_F32T
}

// C[M, N] = alpha 2^-(eA_i + eB_j) (Ahi Bhi + Ahi Blo + Alo Bhi) (+ C if beta). Planes in the
// K8-panel layout [Kp/8][Mp][8] / [Kp/8][Np][8] (Mp, Np multiples of 256, Kp of 16, 16-byte
// aligned), exponents int32[Mp] / int32[Np]. slices / upper / cslice: as ha_gemm_f32t.
HA_EXPORT int ha_gemm_h3t(const void* Ahi, const void* Alo, const void* Bhi, const void* Blo, const int* eA,
                          const int* eB, float* C, int64_t M, int64_t N, int64_t Kp, int64_t Mp, int64_t Np,
                          int64_t ldc, float alpha, int beta, int upper, int64_t slices, int64_t cslice,
                          void* stream) {
  if (M < 0 || N < 0 || Kp < 0 || Kp % TK || Mp % TB || Np % TB || Mp < M || Np < N) return HA_BAD_ARG;
  if (slices < 1 || ((upper & TG_UPPER_TILES) && (M != N || Mp != Np))) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  if ((((uintptr_t)Ahi | (uintptr_t)Alo | (uintptr_t)Bhi | (uintptr_t)Blo) & 15) != 0) return HA_BAD_ARG;
  const int64_t nbn = Np / TB;
  const int64_t nwg = (upper & TG_UPPER_TILES) ? nbn * (nbn + 1) / 2 : (Mp / TB) * nbn;
  if (nwg > 0x7FFFFFFF || slices > 65535) return HA_UNSUPPORTED;
  const int64_t nk = Kp / TK, kps = nk > 0 ? (nk + slices - 1) / slices : 1;
  const dim3 grid((unsigned)nwg, (unsigned)(nk > 0 ? (nk + kps - 1) / kps : 1));
  hipLaunchKernelGGL(gemm_h3t, grid, dim3(256), 0, (hipStream_t)stream, (const _Float16*)Ahi, (const _Float16*)Alo,
                     (const _Float16*)Bhi, (const _Float16*)Blo, eA, eB, C, M, N, Kp, Mp, Np, ldc, alpha, beta, upper,
                     kps, cslice);
  return ha_launch_status();
}

// The number of K slices ha_gemm_{f32t,h3t} launch for (K, slices): ceil(nk / ceil(nk / slices)).
HA_EXPORT int64_t ha_gemm_tiled_slices(int64_t K, int64_t slices) {
  const int64_t nk = (K + TK - 1) / TK;
  if (nk <= 0 || slices < 1) return 1;
  const int64_t kps = (nk + slices - 1) / slices;
  return (nk + kps - 1) / kps;
}

// out[i, j] (fp64, ldo) (+)= sum over s = 0 .. S-1 of P[s cslice + i N + j] (fp32), in slice order;
// upper: only j >= i (the rest of out untouched).
HA_EXPORT int ha_sum_slices64(const float* P, int64_t S, int64_t M, int64_t N, int64_t cslice, double* out,
                              int64_t ldo, int upper, int accumulate, void* stream) {
  if (S < 1 || M < 0 || N < 0 || ldo < N) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  if (N % 4 == 0 && cslice % 4 == 0 && ((uintptr_t)P & 15) == 0) {
    const int64_t g4 = (M * (N / 4) + 255) / 256;
    hipLaunchKernelGGL(tg_sum_slices4, dim3((unsigned)(g4 < 16384 ? g4 : 16384)), dim3(256), 0, (hipStream_t)stream,
                       P, S, M, N, cslice, out, ldo, upper, accumulate);
    return ha_launch_status();
  }
  const int64_t total = M * N, g = (total + 255) / 256;
  hipLaunchKernelGGL(tg_sum_slices, dim3((unsigned)(g < 16384 ? g : 16384)), dim3(256), 0, (hipStream_t)stream, P,
                     S, M, N, cslice, out, ldo, upper, accumulate);
  return ha_launch_status();
}

// K8-panel planes of X [R][C] (row stride ld, unit column stride), scaled per row: hi/lo
// [Kp/8][Rp][8] fp16 (Rp % 64 == 0, Kp % 8 == 0, Kp >= C), ex int32[Rp]; *flag |= 1 on inf/nan.
HA_EXPORT int ha_h3_split_rows(const float* X, int64_t R, int64_t C, int64_t ld, int64_t Rp, int64_t Kp, void* hi,
                               void* lo, int* ex, int* flag, void* stream) {
  if (R < 0 || C < 0 || ld < C || Rp < R || Rp % 64 || Kp < C || Kp % 8 || !hi || !lo) return HA_BAD_ARG;
  if (Rp == 0 || Kp == 0) return HA_OK;
  if ((((uintptr_t)hi | (uintptr_t)lo) & 15) != 0) return HA_BAD_ARG;
  const bool vec = C % 4 == 0 && ld % 4 == 0 && ((uintptr_t)X & 15) == 0;
  const dim3 grid((unsigned)(Rp / 64));
  if (vec)
    hipLaunchKernelGGL(tg_split_rows<true>, grid, dim3(256), 0, (hipStream_t)stream, X, R, C, ld, Rp, Kp,
                       (_Float16*)hi, (_Float16*)lo, ex, flag);
  else
    hipLaunchKernelGGL(tg_split_rows<false>, grid, dim3(256), 0, (hipStream_t)stream, X, R, C, ld, Rp, Kp,
                       (_Float16*)hi, (_Float16*)lo, ex, flag);
  return ha_launch_status();
}

// K8-panel planes of the columns of X [R][C] (contraction along R): hi/lo [Kp/8][Cp][8]
// (Cp % 64 == 0, Kp % 8 == 0, Kp >= R), per-column scales from mx (ha_split_absmax, axis 1).
HA_EXPORT int ha_h3_split_cols(const float* X, int64_t R, int64_t C, int64_t ld, int64_t Cp, int64_t Kp,
                               const float* mx, void* hi, void* lo, int* ex, void* stream) {
  if (R < 0 || C < 0 || ld < C || Cp < C || Cp % 64 || Kp < R || Kp % 8 || !hi || !lo) return HA_BAD_ARG;
  if (Cp == 0 || Kp == 0) return HA_OK;
  if ((((uintptr_t)hi | (uintptr_t)lo) & 15) != 0) return HA_BAD_ARG;
  const int64_t gy = (Kp + 63) / 64;
  if (gy > 65535) {
    // tall contraction: one launch per band of 65535 k-tiles
    for (int64_t y0 = 0; y0 < gy; y0 += 65535) {
      const int64_t rows = (gy - y0 < 65535 ? gy - y0 : 65535) * 64;
      const int64_t kb = y0 * 64;
      const int64_t Rb = R - kb < rows ? (R - kb > 0 ? R - kb : 0) : rows;
      const int64_t Kb = Kp - kb < rows ? Kp - kb : rows;
      hipLaunchKernelGGL(tg_split_cols, dim3((unsigned)(Cp / 64), (unsigned)((Kb + 63) / 64)), dim3(256), 0,
                         (hipStream_t)stream, X + kb * ld, Rb, C, ld, Cp, Kb, mx, (_Float16*)hi + kb * Cp,
                         (_Float16*)lo + kb * Cp, ex);
    }
    return ha_launch_status();
  }
  hipLaunchKernelGGL(tg_split_cols, dim3((unsigned)(Cp / 64), (unsigned)gy), dim3(256), 0, (hipStream_t)stream, X, R,
                     C, ld, Cp, Kp, mx, (_Float16*)hi, (_Float16*)lo, ex);
  return ha_launch_status();
}
