// Exact fp32 GEMM on the f32-input matrix cores: C = A B (+ C), fp32 in, fp32 out.
//
// v_mfma_f32_32x32x2_f32 computes a 32x32 tile over k = 2 per instruction with one f32 operand
// VGPR per lane (lane l: A[i = l & 31][k = l >> 5], B[k = l >> 5][j = l & 31]) and is bit-for-bit a
// k-ordered fp32 fma chain - the numerics of a plain fp32 GEMM, no reduced-precision path (gfx950
// has no xf32). Its rate (64 FLOP/clk/SIMD, 64-cycle issue) is so low relative to the bytes it
// consumes that the kernel is MFMA-bound by construction; the design only has to keep every
// SIMD's matrix pipe fed:
//   * 128 x 128 block tile, 4 waves of 64 x 64 (2 x 2 accumulators of 32 x 32: 4 independent
//     64-cycle chains per wave) or 128 x 256 (2 x 4, 8 chains), BK = 16, 2 workgroups per CU;
//   * A and B staged through LDS in k-major images ([BK][BM] / [BK][BN], rows padded by 32 floats)
//     so each MFMA operand is one conflict-free ds_read_b32 (32 consecutive floats per lane half,
//     the halves 32 banks apart); the NEXT k-tile is loaded into registers (float4) while the
//     current one is multiplied (register double buffer), written after the MFMAs, one barrier
//     per k-tile;
//   * any operand layout: A row-major [M][K] (transposed into the k-major image on the LDS write)
//     or k-major [K][M]; B k-major [K][N] or transposed [N][K] - template flags, so X^T X, X X^T
//     and all four matmul layouts run without a copy;
//   * XCD-aware block order: consecutive block ids (one XCD each round-robin) are remapped so an
//     XCD walks the column blocks of ONE row panel of A - the panel is re-read from that XCD's L2;
//   * the 4 GB descriptor limit of the vendor BLAS does not apply: all offsets are 64-bit.
// Edges (M, N, K not multiples of the tile) are zero-filled on load and masked on store.
#include "common.h"

namespace {

constexpr int GM_BM = 128, GM_BK = 16, GM_PAD = 32;
constexpr int GM_LDA = GM_BM + GM_PAD;  // k-major A image row length (floats)

// XCD-aware bijective remap of a linear block id (nwg blocks, 8 XCDs dispatched round-robin)
__device__ __forceinline__ int64_t gm_xcd_remap(int64_t orig, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8, loc = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// A_KM: A stored k-major (element (m, k) at A[k * lda + m]); else row-major (A[m * lda + k]).
// B_NM: B stored n-major (element (k, n) at B[n * ldb + k]); else k-major (B[k * ldb + n]).
// VEC: 16-byte global loads (the contiguous dimension's extent, ld and base are multiples of 4).
// NT: 32-column accumulator tiles per wave (2: 128 x 128 block; 4: 128 x 256 block, 8 chains per
// wave and 6 operand reads per 8 MFMAs). ACC: C += A B.
template <bool A_KM, bool B_NM, bool VEC, int NT, bool ACC>
__global__ __launch_bounds__(256, 2) void gemm_f32(const float* __restrict__ A, const float* __restrict__ B,
                                                   float* __restrict__ C, int64_t M, int64_t N, int64_t K,
                                                   int64_t lda, int64_t ldb, int64_t ldc) {
  constexpr int BN = 64 * NT, LDB = BN + GM_PAD;
  __shared__ __attribute__((aligned(16))) float smem[2 * GM_BK * (GM_LDA + LDB)];
  float* As = smem;                       // [2][BK][LDA]
  float* Bs = smem + 2 * GM_BK * GM_LDA;  // [2][BK][LDB]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t nbn = (N + BN - 1) / BN, nbm = (M + GM_BM - 1) / GM_BM;
  const int64_t bid = gm_xcd_remap(blockIdx.x, nbm * nbn);
  const int64_t m0 = (bid / nbn) * GM_BM, n0 = (bid % nbn) * BN;
  const int wm = wave >> 1, wn = wave & 1;  // 2 x 2 waves of 64 x (32 NT)

  // ---- staging maps (float4 per thread and load): row-major A (m, k..k+3): thread ->
  // (m = t / 4 + 64 q, k4 = 4 (t % 4)); k-major A (k, m..m+3): thread -> (k = t / 32 + 8 q,
  // m4 = 4 (t % 32)). B: k-major (k, n..n+3): (k = t / (BN/4) + (1024/BN) q, n4 = 4 (t % (BN/4)));
  // n-major (n, k..k+3): (n = t / 4 + 64 q, k4 = 4 (t % 4)).
  constexpr int QA = GM_BM * GM_BK / 1024, QB = BN * GM_BK / 1024, BQ = BN / 4;
  float4 ra[QA], rb[QB];
  auto load_tiles = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      int64_t gm, gk;
      if (A_KM) { gk = k0 + tid / 32 + 8 * q; gm = m0 + 4 * (tid % 32); }
      else { gm = m0 + tid / 4 + 64 * q; gk = k0 + 4 * (tid % 4); }
      float4 v = {0.f, 0.f, 0.f, 0.f};
      if (VEC) {
        if (gk < K && gm < M) v = *reinterpret_cast<const float4*>(A + (A_KM ? gk * lda + gm : gm * lda + gk));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t mm = A_KM ? gm + j : gm, kk = A_KM ? gk : gk + j;
          if (mm < M && kk < K) v[j] = A[A_KM ? kk * lda + mm : mm * lda + kk];
        }
      }
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      int64_t bn, bk;
      if (B_NM) { bn = n0 + tid / 4 + 64 * q; bk = k0 + 4 * (tid % 4); }
      else { bk = k0 + tid / BQ + (256 / BQ) * q; bn = n0 + 4 * (tid % BQ); }
      float4 w = {0.f, 0.f, 0.f, 0.f};
      if (VEC) {
        if (bn < N && bk < K) w = *reinterpret_cast<const float4*>(B + (B_NM ? bn * ldb + bk : bk * ldb + bn));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t nn = B_NM ? bn : bn + j, kk = B_NM ? bk + j : bk;
          if (nn < N && kk < K) w[j] = B[B_NM ? nn * ldb + kk : kk * ldb + nn];
        }
      }
      rb[q] = w;
    }
  };
  auto store_tiles = [&](int buf) {
    float* as = As + buf * GM_BK * GM_LDA;
    float* bs = Bs + buf * GM_BK * LDB;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      if (A_KM) {
        *reinterpret_cast<float4*>(as + (tid / 32 + 8 * q) * GM_LDA + 4 * (tid % 32)) = ra[q];
      } else {
        const int mm = tid / 4 + 64 * q, k4 = 4 * (tid % 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) as[(k4 + j) * GM_LDA + mm] = ra[q][j];
      }
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      if (B_NM) {
        const int nn = tid / 4 + 64 * q, k4 = 4 * (tid % 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) bs[(k4 + j) * LDB + nn] = rb[q][j];
      } else {
        *reinterpret_cast<float4*>(bs + (tid / BQ + (256 / BQ) * q) * LDB + 4 * (tid % BQ)) = rb[q];
      }
    }
  };

  floatx16 acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (floatx16)(0.f);

  const int64_t nk = (K + GM_BK - 1) / GM_BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int h = lane >> 5, r = lane & 31;
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) load_tiles((kt + 1) * GM_BK);  // in flight during the MFMAs below
    const float* as = As + cur * GM_BK * GM_LDA + wm * 64 + r;
    const float* bs = Bs + cur * GM_BK * LDB + wn * (32 * NT) + r;
#pragma unroll
    for (int kk = 0; kk < GM_BK; kk += 2) {
      const float a0 = as[(kk + h) * GM_LDA], a1 = as[(kk + h) * GM_LDA + 32];
      float b[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = bs[(kk + h) * LDB + 32 * j];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b[j], acc[0][j], 0, 0, 0);
        acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b[j], acc[1][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);  // the other buffer: last read one barrier ago
    __syncthreads();
  }

  // ---- epilogue: D row = (reg & 3) + 8 (reg >> 2) + 4 h, col = lane & 31
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int64_t gn = n0 + wn * (32 * NT) + j * 32 + r;
    if (gn >= N) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int64_t gm = m0 + wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        if (gm < M) {
          float* c = C + gm * ldc + gn;
          if (ACC) *c += acc[i][j][g];
          else *c = acc[i][j][g];
        }
      }
  }
}

// ------------------------------------------------------------------------------------------
// fp32 GEMM at fp16 matrix-core speed ("fp16x3", the same split as csrc/gemm_split.hip): the
// operands arrive as fp16 hi/lo planes of power-of-two-scaled rows (A: [M][Kp] per row of A;
// B^T: [N][Kp] per column of B; Kp a multiple of 32, zero tail) and ONE kernel forms
//     D = hi_A hi_B + hi_A lo_B + lo_A hi_B      (fp32 accumulation, 3 MFMAs per fragment pair)
// then C = 2^-(eA_i + eB_j) D exactly in the epilogue. Fused, the hi_A and hi_B fragments are read
// once for two products, 4 half-tiles are staged per k-step instead of the tripled-K library
// GEMM's 6, and there is no separate unscale pass over C.
//   * 128 x 128 x 32 block tile, 4 waves of 64 x 64 (2 x 2 accumulators of 32x32x16 f16 MFMAs),
//     2 workgroups per CU;
//   * staging by LDS-DMA (global_load_lds_dwordx4): wave w stages half-tile w (A hi, A lo, B hi,
//     B lo) of the NEXT k-step while the current one is multiplied (2 LDS buffers, 64 KB);
//   * LDS rows are 64 B (32 halfs): the 16-byte chunk c of row r is stored at chunk c ^ ((r >> 2) & 3)
//     (the permutation is applied to the DMA's per-lane SOURCE address, the LDS image stays
//     lane-linear), so a fragment read (32 rows, one chunk) is bank-conflict free;
//   * XCD-aware block order as in gemm_f32.
constexpr int H3_BM = 128, H3_BN = 128, H3_BK = 32, H3_TILE = 128 * 64;  // bytes per half-tile

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256, 2) void gemm_h3(const _Float16* __restrict__ Ahi, const _Float16* __restrict__ Alo,
                                                  const _Float16* __restrict__ Bhi, const _Float16* __restrict__ Blo,
                                                  const int* __restrict__ eA, const int* __restrict__ eB,
                                                  float* __restrict__ C, int64_t M, int64_t N, int64_t Kp, int64_t ldc) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 4 * H3_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t nbn = (N + H3_BN - 1) / H3_BN, nbm = (M + H3_BM - 1) / H3_BM;
  const int64_t bid = gm_xcd_remap(blockIdx.x, nbm * nbn);
  const int64_t m0 = (bid / nbn) * H3_BM, n0 = (bid % nbn) * H3_BN;
  const int wm = wave >> 1, wn = wave & 1;

  // this wave's half-tile source: rows of A (waves 0, 1) or of B^T (waves 2, 3)
  const _Float16* plane = wave == 0 ? Ahi : wave == 1 ? Alo : wave == 2 ? Bhi : Blo;
  const int64_t rbase = wave < 2 ? m0 : n0, rmax = (wave < 2 ? M : N) - 1;
  const int srow = lane >> 2;                                   // row within a 16-row piece
  const int schunk = (lane & 3) ^ ((lane >> 4) & 3);            // source chunk of LDS slot `lane`
  auto stage = [&](int buf, int64_t k0) {
    unsigned char* dst = smem + (buf * 4 + wave) * H3_TILE;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t row = rbase + 16 * j + srow;
      row = row < rmax ? row : rmax;  // clamped edge rows: valid addresses, results masked later
      const _Float16* src = plane + row * Kp + k0 + schunk * 8;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16, 0, 0);
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (floatx16)(0.f);

  const int h = lane >> 5, r = lane & 31;
  // fragment byte offsets inside a half-tile: row (tile row + r), chunk (2 s + h) swizzled
  int offA[2][2], offB[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ra = wm * 64 + i * 32 + r, rb = wn * 64 + i * 32 + r;
      offA[s][i] = ra * 64 + (((2 * s + h) ^ ((ra >> 2) & 3)) * 16);
      offB[s][i] = rb * 64 + (((2 * s + h) ^ ((rb >> 2) & 3)) * 16);
    }

  const int64_t nk = Kp / H3_BK;
  stage(0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * H3_BK);  // DMA in flight during the MFMAs below
    const unsigned char* base = smem + cur * 4 * H3_TILE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      halfx8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = *reinterpret_cast<const halfx8*>(base + 0 * H3_TILE + offA[s][i]);
        al[i] = *reinterpret_cast<const halfx8*>(base + 1 * H3_TILE + offA[s][i]);
        bh[i] = *reinterpret_cast<const halfx8*>(base + 2 * H3_TILE + offB[s][i]);
        bl[i] = *reinterpret_cast<const halfx8*>(base + 3 * H3_TILE + offB[s][i]);
      }
      // small terms first, the hi.hi product last (each accumulator is revisited every 4 MFMAs)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of the next k-step has landed ...
    __syncthreads();                // ... and every wave's, before anyone reads that buffer
  }

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t gn = n0 + wn * 64 + j * 32 + r;
    if (gn >= N) continue;
    const int ebn = eB[gn];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int64_t gm = m0 + wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        if (gm < M) C[gm * ldc + gn] = ldexpf(acc[i][j][g], -(eA[gm] + ebn));
      }
  }
}

template <int NT>
int gemm_f32_launch(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                    int64_t ldb, int64_t ldc, int a_kmajor, int b_nmajor, int accumulate, hipStream_t s) {
  const int64_t nwg = ((M + GM_BM - 1) / GM_BM) * ((N + 64 * NT - 1) / (64 * NT));
  if (nwg > 0x7FFFFFFF) return HA_UNSUPPORTED;
  // 16-byte loads need the contiguous extent, the leading dimension and the base 4-float aligned
  const int64_t a_contig = a_kmajor ? M : K, b_contig = b_nmajor ? K : N;
  const bool vec = a_contig % 4 == 0 && b_contig % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 &&
                   ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0;
  const dim3 grid((unsigned)nwg), block(256);
#define HA_GM(AK, BN_, V)                                                                                         \
  do {                                                                                                           \
    if (accumulate) hipLaunchKernelGGL((gemm_f32<AK, BN_, V, NT, true>), grid, block, 0, s, A, B, C, M, N, K, lda, ldb, ldc); \
    else hipLaunchKernelGGL((gemm_f32<AK, BN_, V, NT, false>), grid, block, 0, s, A, B, C, M, N, K, lda, ldb, ldc);  \
  } while (0)
  if (vec) {
    if (a_kmajor) { if (b_nmajor) HA_GM(true, true, true); else HA_GM(true, false, true); }
    else { if (b_nmajor) HA_GM(false, true, true); else HA_GM(false, false, true); }
  } else {
    if (a_kmajor) { if (b_nmajor) HA_GM(true, true, false); else HA_GM(true, false, false); }
    else { if (b_nmajor) HA_GM(false, true, false); else HA_GM(false, false, false); }
  }
#undef HA_GM
  return ha_launch_status();
}

}  // namespace

// C[M, N] (row-major, ldc) = A B (+ C if accumulate). a_kmajor: A element (m, k) at A[k * lda + m]
// (else A[m * lda + k]); b_nmajor: B element (k, n) at B[n * ldb + k] (else B[k * ldb + n]).
// variant: 2 = 128 x 128 block tile, 4 = 128 x 256 (NT accumulator columns per wave).
HA_EXPORT int ha_gemm_f32(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                          int64_t ldb, int64_t ldc, int a_kmajor, int b_nmajor, int accumulate, int variant,
                          void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  if (variant == 4) return gemm_f32_launch<4>(A, B, C, M, N, K, lda, ldb, ldc, a_kmajor, b_nmajor, accumulate, s);
  return gemm_f32_launch<2>(A, B, C, M, N, K, lda, ldb, ldc, a_kmajor, b_nmajor, accumulate, s);
}

// C[M, N] = 2^-(eA_i + eB_j) (Ahi Bhi^T + Ahi Blo^T + Alo Bhi^T): planes [M][Kp] / [N][Kp] fp16
// (Kp % 32 == 0, zero tail, 16-byte aligned bases), exponents int32.
HA_EXPORT int ha_gemm_h3(const void* Ahi, const void* Alo, const void* Bhi, const void* Blo, const int* eA,
                         const int* eB, float* C, int64_t M, int64_t N, int64_t Kp, int64_t ldc, void* stream) {
  if (M < 0 || N < 0 || Kp < 0 || Kp % H3_BK != 0) return HA_BAD_ARG;
  if (M == 0 || N == 0) return HA_OK;
  if ((((uintptr_t)Ahi | (uintptr_t)Alo | (uintptr_t)Bhi | (uintptr_t)Blo) & 15) != 0) return HA_BAD_ARG;
  const int64_t nwg = ((M + H3_BM - 1) / H3_BM) * ((N + H3_BN - 1) / H3_BN);
  if (nwg > 0x7FFFFFFF) return HA_UNSUPPORTED;
  hipLaunchKernelGGL(gemm_h3, dim3((unsigned)nwg), dim3(256), 0, (hipStream_t)stream, (const _Float16*)Ahi,
                     (const _Float16*)Alo, (const _Float16*)Bhi, (const _Float16*)Blo, eA, eB, C, M, N, Kp, ldc);
  return ha_launch_status();
}
