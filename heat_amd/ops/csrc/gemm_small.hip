// 128 x 128-tile exact fp32 GEMM with split-K: the products the 256 x 256 kernel
// of gemm_tiled.hip cannot spread over the 256 CUs - 1024^3 .. 6144^3 (16 .. 576 tiles of 256^2:
// a fraction of a wave, or 2.25 waves), and the short-K tall updates of the Householder QR
// (C[1.25e6, 3840] -= V[1.25e6, 256] X[256, 3840]: K = 256 is 16 k-stages, which the 256-tile
// kernel's 3-stage LDS-DMA prologue and 256 KB C epilogue per tile do not amortise). Before this
// kernel those shapes went to hipBLASLt (profiles/gemm_small_r04.jsonl: 9x at 1024^3).
//
// Design: 4 waves, each a 64 x 64 quadrant (2 x 2 v_mfma_f32_32x32x2_f32 accumulators = 64
// registers), 32-k stages double-buffered in LDS through registers (the next stage's global loads
// are in flight during the current stage's 64 MFMAs per wave), two workgroups per CU (70.6 KB of
// LDS each). The k order inside a stage is permuted - lane half h owns k = 16 h + s at MFMA step
// s - so a row-major A fragment is four ds_read_b128 of its row. A: row-major [M][K] or k-major
// [K][M]; B: k-major [K][N] or n-major [N][K]. split-K: grid.y = slices, slice y writes its
// partial to C + y cslice (summed by ha_sum_slices32/64). XCD-aware tile order (each XCD takes a
// contiguous range of tiles, walked in groups of 8 row panels so A and B panels stay in its L2).
#include "common.h"

namespace {

constexpr int GB = 128, GK = 32;  // GK: the slice granularity (kps is a multiple of it)
constexpr int B_LD = GB + 4;    // Bs[k][n]

__device__ __forceinline__ int64_t gs_xcd_remap(int64_t orig, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8, loc = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// GKT: k per LDS stage - 32 (default: 70.6 KB of LDS, two workgroups per CU) or 16 (A/B,
// HEAT_GS_K16=1: 37.4 KB and fewer registers, three workgroups per CU, twice the barriers)
template <bool AK, bool BN, bool PRIO = false, int GKT = 32>
__global__ __launch_bounds__(256, GKT == 16 ? 3 : 2) void gemm_f32s(const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C, int64_t M, int64_t N, int64_t K,
                                                    int64_t lda, int64_t ldb, int64_t ldc, float alpha, int beta,
                                                    int64_t kps, int64_t cslice) {
  constexpr int A_LD = GKT + 4;  // As[row][k]: 144 / 80-byte rows (conflict-free row-per-lane b128 reads)
  constexpr int A_SZ = GB * A_LD, B_SZ = GKT * B_LD, ST_SZ = A_SZ + B_SZ;  // floats per stage
  constexpr int NP = GKT / 8;     // 16-byte pieces per thread per operand and stage
  constexpr int PR = GKT / 4;     // 16-byte pieces per row of a k-contiguous operand stage
  constexpr int HS = GKT / 2;     // k steps per stage; lane half h owns k = HS h + s at step s
  __shared__ __attribute__((aligned(16))) float sm[2 * ST_SZ];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int64_t tn = (N + GB - 1) / GB, tm = (M + GB - 1) / GB;
  const int64_t bid = gs_xcd_remap(blockIdx.x, tm * tn);
  // grouped order: consecutive tiles (the ones an XCD runs together) cover GM row panels x a run
  // of column panels, so both operand panels are reused from that XCD's L2 (row-major order
  // shared only the A panel: a 128-tile stage needs 32 B/FLOP-ish operand feed, ~4.5 TB/s at 150 TF)
  constexpr int64_t GM = 8;
  const int64_t grp = bid / (GM * tn), gfirst = grp * GM;
  const int64_t gsz = tm - gfirst < GM ? tm - gfirst : GM;
  const int64_t m0 = (gfirst + (bid % (GM * tn)) % gsz) * GB, n0 = ((bid % (GM * tn)) / gsz) * GB;
  const int64_t kb = (int64_t)blockIdx.y * kps;
  const int64_t ke = K - kb < kps ? K : kb + kps;
  C += (int64_t)blockIdx.y * cslice;

  floatx4 ra[NP], rb[NP];
  // piece p = tid + 256 i of a stage (1024 16-byte pieces per operand)
  // interior tiles (every stage of a slice is whole: kps is a multiple of 32) take the unguarded
  // 16-byte loads; only edge tiles and the last partial stage evaluate per-piece bounds
  const bool inner = m0 + GB <= M && n0 + GB <= N;
  auto gload = [&](int64_t k0) {
    if (inner && k0 + GKT <= ke) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int p = tid + 256 * i;
        ra[i] = !AK ? *reinterpret_cast<const floatx4*>(A + (m0 + p / PR) * lda + k0 + 4 * (p % PR))
                    : *reinterpret_cast<const floatx4*>(A + (k0 + (p >> 5)) * lda + m0 + 4 * (p & 31));
        rb[i] = !BN ? *reinterpret_cast<const floatx4*>(B + (k0 + (p >> 5)) * ldb + n0 + 4 * (p & 31))
                    : *reinterpret_cast<const floatx4*>(B + (n0 + p / PR) * ldb + k0 + 4 * (p % PR));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int p = tid + 256 * i;
      if (!AK) {  // row-major: row p / PR, k 4 (p % PR)
        const int64_t gr = m0 + p / PR, gk = k0 + 4 * (p % PR);
        const float* s = A + gr * lda + gk;
        if (gr < M && gk + 4 <= ke) {
          ra[i] = *reinterpret_cast<const floatx4*>(s);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) ra[i][j] = (gr < M && gk + j < ke) ? s[j] : 0.f;
        }
      } else {    // k-major: k p >> 5, rows 4 (p & 31)
        const int64_t gk = k0 + (p >> 5), gr = m0 + 4 * (p & 31);
        const float* s = A + gk * lda + gr;
        if (gk < ke && gr + 4 <= M) {
          ra[i] = *reinterpret_cast<const floatx4*>(s);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) ra[i][j] = (gk < ke && gr + j < M) ? s[j] : 0.f;
        }
      }
      if (!BN) {  // k-major [K][N]: k p >> 5, columns 4 (p & 31)
        const int64_t gk = k0 + (p >> 5), gc = n0 + 4 * (p & 31);
        const float* s = B + gk * ldb + gc;
        if (gk < ke && gc + 4 <= N) {
          rb[i] = *reinterpret_cast<const floatx4*>(s);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) rb[i][j] = (gk < ke && gc + j < N) ? s[j] : 0.f;
        }
      } else {    // n-major [N][K]: column p / PR, k 4 (p % PR)
        const int64_t gc = n0 + p / PR, gk = k0 + 4 * (p % PR);
        const float* s = B + gc * ldb + gk;
        if (gc < N && gk + 4 <= ke) {
          rb[i] = *reinterpret_cast<const floatx4*>(s);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) rb[i][j] = (gc < N && gk + j < ke) ? s[j] : 0.f;
        }
      }
    }
  };
  auto sstore = [&](int buf) {
    float* As = sm + buf * ST_SZ;
    float* Bs = As + A_SZ;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int p = tid + 256 * i;
      if (!AK) {
        *reinterpret_cast<floatx4*>(As + (p / PR) * A_LD + 4 * (p % PR)) = ra[i];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) As[(4 * (p & 31) + j) * A_LD + (p >> 5)] = ra[i][j];
      }
      if (!BN) {
        *reinterpret_cast<floatx4*>(Bs + (p >> 5) * B_LD + 4 * (p & 31)) = rb[i];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) Bs[(4 * (p % PR) + j) * B_LD + p / PR] = rb[i][j];
      }
    }
  };

  floatx16 acc[2][2];
  if (beta == 2) {
    // C preloaded into the accumulators (acc = alpha C, alpha = +-1 checked by the host) before
    // the first stage's loads: the epilogue only stores alpha acc = C + alpha A B (see gemm_f32t)
    const bool fullc = m0 + GB <= M && n0 + GB <= N;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
      const int64_t rb0 = m0 + wm * 64 + bm * 32 + 4 * h;
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) {
        const int64_t gc = n0 + wn * 64 + bn * 32 + r;
        const float* cp = C + rb0 * ldc + gc;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int dr = (g & 3) + 8 * (g >> 2);
          acc[bm][bn][g] = (fullc || (rb0 + dr < M && gc < N)) ? alpha * cp[dr * ldc] : 0.f;
        }
      }
    }
  } else {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = (floatx16)(0.f);
  }
  auto compute = [&](int buf) {
    const float* As = sm + buf * ST_SZ;
    const float* Bs = As + A_SZ;
    floatx4 fa[2][HS / 4];
    float fb[2][HS];
    // fragments in 4 groups of 4 k-steps; group q + 1 is read while group q's 16 MFMAs run
    // (reading all 40 first exposed the LDS latency once per stage, 38 % of wave cycles waiting)
    auto frag = [&](int q) __attribute__((always_inline)) {
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
        fa[bm][q] = *reinterpret_cast<const floatx4*>(As + (wm * 64 + bm * 32 + r) * A_LD + HS * h + 4 * q);
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
#pragma unroll
        for (int s = 4 * q; s < 4 * q + 4; ++s) fb[bn][s] = Bs[(HS * h + s) * B_LD + wn * 64 + bn * 32 + r];
    };
    frag(0);
    // PRIO (A/B, HEAT_GS_PRIO=1): the wave in its MFMA phase wins issue arbitration over the other
    // workgroup's wave on the SIMD, which then runs its loads / barrier meanwhile (the two
    // workgroups drift out of phase instead of reaching their barriers together)
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < HS / 4; ++q) {
      if (q + 1 < HS / 4) frag(q + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 4 * q; s < 4 * q + 4; ++s)
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[bm][q][s & 3], fb[bn][s], acc[bm][bn], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  const int64_t nk = (ke - kb + GKT - 1) / GKT;
  if (nk > 0) {
    gload(kb);
    sstore(0);
    __syncthreads();
  }
  for (int64_t t = 0; t < nk; ++t) {
    if (t + 1 < nk) gload(kb + (t + 1) * GKT);  // in flight during this stage's MFMAs
    compute(t & 1);
    if (t + 1 < nk) sstore((t + 1) & 1);
    __syncthreads();
  }
  // epilogue: 32 x 32 C/D map - column r, rows (g & 3) + 8 (g >> 2) + 4 h
  const bool full = m0 + GB <= M && n0 + GB <= N;
#pragma unroll
  for (int bm = 0; bm < 2; ++bm) {
    const int64_t rb0 = m0 + wm * 64 + bm * 32 + 4 * h;
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
      const int64_t gc = n0 + wn * 64 + bn * 32 + r;
      float* cp = C + rb0 * ldc + gc;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int dr = (g & 3) + 8 * (g >> 2);
        if (full || (rb0 + dr < M && gc < N)) {
          float v = alpha * acc[bm][bn][g];
          if (beta == 1) v += cp[dr * ldc];
          cp[dr * ldc] = v;
        }
      }
    }
  }
}

}  // namespace

// The k-slice length (a multiple of the 32-k stage) and the number of slices actually launched
// for a request of `slices`: ceil(K / kps).
HA_EXPORT int64_t ha_gemm_f32s_kps(int64_t K, int64_t slices) {
  if (slices < 1) slices = 1;
  int64_t kps = (K + slices - 1) / slices;
  kps = (kps + GK - 1) / GK * GK;
  return kps > 0 ? kps : GK;
}
HA_EXPORT int64_t ha_gemm_f32s_slices(int64_t K, int64_t slices) {
  const int64_t kps = ha_gemm_f32s_kps(K, slices);
  return K > 0 ? (K + kps - 1) / kps : 1;
}

// C[M, N] (row-major, ldc) = alpha A B (+ C if beta), exact fp32 products and accumulation.
// a_kmajor: A element (m, k) at A[k lda + m] (else A[m lda + k]); b_nmajor: B element (k, n) at
// B[n ldb + k] (else B[k ldb + n]). slices > 1: split-K, slice y -> C + y cslice (beta must be 0).
// Requirements (else HA_UNSUPPORTED): 16-byte aligned A and B, lda and ldb multiples of 4.
HA_EXPORT int ha_gemm_f32s(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, int64_t ldc, int a_kmajor, int b_nmajor, float alpha, int beta, int64_t slices,
                           int64_t cslice, void* stream) {
  if (M <= 0 || N <= 0) return HA_OK;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15) || (lda & 3) || (ldb & 3)) return HA_UNSUPPORTED;
  if (slices > 1 && beta) return HA_BAD_ARG;
  // accumulate with alpha = +-1: C preloaded into the accumulators only with HEAT_GEMM_F32_PRELOAD=1
  // (A/B: slower, and every partial sum rounds at the scale of C, profiles/update_ab_r06.jsonl)
  static const int preload = getenv("HEAT_GEMM_F32_PRELOAD") ? atoi(getenv("HEAT_GEMM_F32_PRELOAD")) : 0;
  if (beta) beta = (preload && (alpha == 1.f || alpha == -1.f)) ? 2 : 1;
  const int64_t tiles = ((M + GB - 1) / GB) * ((N + GB - 1) / GB);
  const int64_t kps = ha_gemm_f32s_kps(K, slices);
  const int64_t ns = ha_gemm_f32s_slices(K, slices);
  if (tiles > 0x7fffffffLL || ns > 65535) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)tiles, (unsigned)ns), b(256);
  static const bool prio = getenv("HEAT_GS_PRIO") && getenv("HEAT_GS_PRIO")[0] == '1';
  // 16-k stages (three workgroups per CU) or 32-k (two): HEAT_GS_K16 = 1 / 0 forces one; by default
  // the wave quantisation decides - W = workgroups / (CUs x workgroups per CU), e(W) = W / ceil(W),
  // 16-k when 1.04 e16 > e32 (measured, tools/r5/gpu_k16.sh: 16-k is ~3-4 % faster per wave on
  // large grids - 1.25e6 x 3840 x 256 21.8 vs 22.6 ms - and 6144^3 3.90 vs 4.37 ms at 3.0 vs 4.5
  // waves, but slower where it leaves a partial wave: 4096^3 1.19 vs 1.11 ms)
  static const int k16_env = getenv("HEAT_GS_K16") ? (getenv("HEAT_GS_K16")[0] == '1' ? 1 : 0) : -1;
  static const int ncu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  bool k16 = k16_env == 1;
  if (k16_env < 0) {
    const double nwg = (double)tiles * (double)ns;
    auto eff = [](double w) { const double c = w > 1.0 ? (double)(int64_t)(w + 0.999999) : 1.0; return w / c; };
    k16 = 1.04 * eff(nwg / (3.0 * ncu)) > eff(nwg / (2.0 * ncu));
  }
  if (k16) {
    if (!a_kmajor && !b_nmajor)
      hipLaunchKernelGGL((gemm_f32s<false, false, false, 16>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta,
                         kps, cslice);
    else if (!a_kmajor && b_nmajor)
      hipLaunchKernelGGL((gemm_f32s<false, true, false, 16>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta,
                         kps, cslice);
    else if (a_kmajor && !b_nmajor)
      hipLaunchKernelGGL((gemm_f32s<true, false, false, 16>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta,
                         kps, cslice);
    else
      hipLaunchKernelGGL((gemm_f32s<true, true, false, 16>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta,
                         kps, cslice);
    return ha_launch_status();
  }
  if (prio) {
    if (!a_kmajor && !b_nmajor)
      hipLaunchKernelGGL((gemm_f32s<false, false, true>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps,
                         cslice);
    else if (!a_kmajor && b_nmajor)
      hipLaunchKernelGGL((gemm_f32s<false, true, true>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps,
                         cslice);
    else if (a_kmajor && !b_nmajor)
      hipLaunchKernelGGL((gemm_f32s<true, false, true>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps,
                         cslice);
    else
      hipLaunchKernelGGL((gemm_f32s<true, true, true>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps,
                         cslice);
    return ha_launch_status();
  }
  if (!a_kmajor && !b_nmajor)
    hipLaunchKernelGGL((gemm_f32s<false, false>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
  else if (!a_kmajor && b_nmajor)
    hipLaunchKernelGGL((gemm_f32s<false, true>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
  else if (a_kmajor && !b_nmajor)
    hipLaunchKernelGGL((gemm_f32s<true, false>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
  else
    hipLaunchKernelGGL((gemm_f32s<true, true>), g, b, 0, s, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, kps, cslice);
  return ha_launch_status();
}
