// K-means iteration for few clusters (k <= 16, the reference benchmark's k = 8; f <= 64):
// assignment AND centroid sums in one pass over the points.
//
// With k this small the MFMA kernels waste most of a 128-centroid tile on padding and each
// workgroup's short life (stage the centroid image, one tile, store) is latency-bound
// (kmeans_f16x3.hip's filter: 2.3 ms per pass at n = 12.5M, f = 64, k = 8), and the separate
// update re-reads the points (0.8 ms). The arithmetic is 2 n k f flops against n f floats read
// once: the iteration is HBM-bound if the points are read exactly once and the inner loop stays
// off the LDS.
//
// Design (measured steps in profiles/README.md):
//  * row-per-lane loads straight from HBM ran at 1.0 TB/s at f = 64 (64 lanes x 16 B at a 256 B
//    stride per instruction re-request every line and thrash L1/L2), so the points are staged: a
//    persistent workgroup (2 waves, 4 per CU) loops over 128-row tiles; each thread issues all of
//    its 16-byte loads of the NEXT tile right after the current one reached LDS (in flight during
//    the compute), then writes them with one ds_write_b128 per piece;
//  * LDS rows are padded to a stride of 4 ceil(f/4) + 4 words: the row-per-thread ds_read_b128 of
//    the assignment is bank-conflict free (stride 68 words at f = 64: lanes of a 16-lane pass start
//    4 banks apart);
//  * the centroids never touch the LDS: a padded copy (k -> KP rows, the padding rows at +inf so
//    they never win; f -> a multiple of 8 with zeros) is read with scalar loads and used as SGPR
//    operands of packed-fp32 VALU ops (an LDS broadcast per (centroid, 4 features) made the loop
//    LDS-bound);
//  * assign: thread r owns row r, KP difference-form accumulators (sum (x - c)^2, exact fp32, no
//    expansion cancellation), strict-< argmin (lowest index on ties);
//  * update on the matrix cores: the per-cluster sums of a tile are onehot(labels)^T X, 4 rows per
//    v_mfma_f32_16x16x4_f32 (k <= 16 clusters = M; 0/1 weights make every product exact, fp32
//    accumulation). A ballot-and-walk over each cluster's rows (LDS-latency bound, +0.6 ms at
//    f = 64, k = 8) and a scalar-branch select-add (+1.1 ms) were slower. Per-workgroup partial
//    sums/counts stay in registers across tiles, are written once and reduced in fp64.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));

constexpr int KS_ROWS = 128;  // rows per tile = threads per workgroup (2 waves)
constexpr int KS_WAVES = KS_ROWS / 64;
constexpr int KS_FMAX = 64;
constexpr int KS_LDMAX = KS_FMAX + 4;  // padded LDS row stride (words) at f = 64
enum { KS_ROW4 = 0, KS_FLAT = 1, KS_SCALAR = 2 };

// features covered by the assignment: a multiple of 16 (a loop iteration takes 16 / CPI...16
// features, see ks_step); the LDS rows are fp + 4 words: 16-byte aligned, zero beyond f, and the
// row-per-lane ds_read_b128 of a 16-lane pass conflict-free (fp + 4 = 4 mod 16 words: the 16 start
// banks are 4 apart modulo 64)
__host__ __device__ inline int ks_fp(int f) { return ((f + 15) / 16) * 16; }
__host__ __device__ inline int ks_ld(int f) { return ks_fp(f) + 4; }

// chunked centroid copy for the scalar (SGPR-operand) reads of the assignment:
// Cq[q][c][4] = C[c][4q .. 4q+3] for the fp / 4 chunks q (+ one zero chunk past the end);
// rows c >= k at +inf (they never win), features >= f zero
__global__ __launch_bounds__(256) void ks_pad_centroids(const float* __restrict__ C, int k, int f, int64_t ldc,
                                                        int kp, float* __restrict__ Cq) {
  const int fp = ks_fp(f);
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kp * (fp + 4)) return;
  const int q = e / (4 * kp), c = (e / 4) % kp, j = 4 * q + (e & 3);
  Cq[e] = c < k ? (j < f ? C[(int64_t)c * ldc + j] : 0.f) : (j == 0 ? __builtin_huge_valf() : 0.f);
}

// acc[c] += (x - c)^2 over one 4-feature chunk for the KP centroids: the centroid pair is an SGPR
// operand of v_pk_add_f32 (x - c in one packed op; the compiler does not select SGPR pairs for
// packed fp32 by itself and fell back to scalar subtracts plus SGPR spills to VGPR lanes)
template <int KP>
__device__ __forceinline__ void ks_chunk(const floatx4 (&cc)[KP], floatx4 x, floatx2 (&acc)[KP]) {
  const floatx2 x0 = {x[0], x[1]}, x1 = {x[2], x[3]};
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    floatx2 d0, d1;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d0) : "v"(x0), "s"((floatx2){cc[c][0], cc[c][1]}));
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d1) : "v"(x1), "s"((floatx2){cc[c][2], cc[c][3]}));
    acc[c] = __builtin_elementwise_fma(d0, d0, acc[c]);
    acc[c] = __builtin_elementwise_fma(d1, d1, acc[c]);
  }
}

// NFB: 16-feature blocks covered by the update (4 for f <= 64, 2 for f <= 32)
// MODE: KS_ROW4 (f % 4 == 0, 16-byte aligned rows: 16-byte pieces of rows), KS_FLAT (contiguous
// rows, f % 4 != 0: the tile is one span read as 16-byte pieces, scattered to the padded rows
// element by element), KS_SCALAR (anything else: 4-byte pieces).
template <int KP, int MODE, bool UPDATE, int NFB = 4>
__global__ __launch_bounds__(KS_ROWS, 4) void ks_step(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                      const float* __restrict__ Cp, int* __restrict__ labels,
                                                      float* __restrict__ mind, float* __restrict__ sums_part,
                                                      float* __restrict__ counts_part) {
  constexpr bool VEC = MODE != KS_SCALAR;
  typedef typename std::conditional<VEC, floatx4, float>::type piece;
  constexpr int PER = VEC ? KS_FMAX / 4 : KS_FMAX;  // pieces per thread per tile at f = 64
  __shared__ __attribute__((aligned(16))) float tile[KS_ROWS * KS_LDMAX];
  __shared__ __attribute__((aligned(16))) int lab[KS_ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ld = ks_ld(f), fp = ks_fp(f);
  const int64_t ntiles = (n + KS_ROWS - 1) / KS_ROWS;
  // zero the padding columns [f, ld) once: stores only ever write columns < f
  for (int e = tid; e < KS_ROWS * (ld - f); e += KS_ROWS) {
    const int r = e / (ld - f), c = f + e % (ld - f);
    tile[r * ld + c] = 0.f;
  }
  constexpr int UB = (NFB + KS_WAVES - 1) / KS_WAVES;  // 16-feature blocks per wave
  constexpr int UG = 4;
  floatx4 uacc[UB][UG];
#pragma unroll
  for (int b = 0; b < UB; ++b)
#pragma unroll
    for (int g = 0; g < UG; ++g) uacc[b][g] = (floatx4)(0.f);
  float ucnt = 0.f;  // wave 0, lane c: count of cluster c

  // piece p of a thread: p = tid + KS_ROWS * i. ROW4 / SCALAR: over the tile's rows x w pieces
  // per row; FLAT: float offset 4 p of the contiguous tile. (row, column) advance incrementally.
  const int w = MODE == KS_ROW4 ? f >> 2 : f;
  const int step = MODE == KS_FLAT ? 4 * KS_ROWS : KS_ROWS;
  const int qrow = step / w, qrem = step - qrow * w;
  const int start = MODE == KS_FLAT ? 4 * tid : tid;
  const int r_init = start / w, c_init = start - (start / w) * w;
  piece buf[PER];
  auto load = [&](int64_t t) {
    const int64_t row0 = t * KS_ROWS;
    const int rows = (int)(n - row0 < KS_ROWS ? n - row0 : KS_ROWS);
    const float* base = X + row0 * ldx;
    if constexpr (MODE == KS_FLAT) {
      const int tot = rows * f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int u = 4 * (tid + KS_ROWS * i);
        if (u + 3 < tot) {
          buf[i] = *reinterpret_cast<const floatx4*>(base + u);
        } else if (u < tot) {  // tail of the data: element-wise, never past the end
#pragma unroll
          for (int q = 0; q < 4; ++q) buf[i][q] = u + q < tot ? base[u + q] : 0.f;
        }
      }
    } else {
      int r = r_init, c = c_init;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        if (r < rows) buf[i] = *reinterpret_cast<const piece*>(base + (int64_t)r * ldx + (VEC ? 4 * c : c));
        r += qrow;
        c += qrem;
        if (c >= w) {
          c -= w;
          ++r;
        }
      }
    }
  };
  auto store = [&](int rows) {
    int r = r_init, c = c_init;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if constexpr (MODE == KS_FLAT) {
        int rq = r, cq = c;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (rq < rows) tile[rq * ld + cq] = buf[i][q];
          if (++cq == f) {
            cq = 0;
            ++rq;
          }
        }
      } else {
        if (r < rows) *reinterpret_cast<piece*>(tile + r * ld + (VEC ? 4 * c : c)) = buf[i];
      }
      r += qrow;
      c += qrem;
      if (c >= w) {
        c -= w;
        ++r;
      }
    }
  };

  int64_t t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    const int64_t row0 = t * KS_ROWS;
    const int rows = (int)(n - row0 < KS_ROWS ? n - row0 : KS_ROWS);
    if (UPDATE && rows < KS_ROWS)
      for (int e = tid; e < (KS_ROWS - rows) * ld; e += KS_ROWS) tile[rows * ld + e] = 0.f;
    store(rows);
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);  // in flight during this tile's compute
    // ---- assign: thread = row, centroids as SGPR operands (wave-uniform scalar loads of CPI
    // chunks per loop iteration, one lgkm wait per iteration)
    {
      const float* xr = tile + (tid < rows ? tid : 0) * ld;
      const floatx4* Cq = reinterpret_cast<const floatx4*>(Cp);
      constexpr int CPI = KP <= 4 ? 2 : 1;  // 4-feature chunks per iteration
      floatx2 acc[KP];
#pragma unroll
      for (int c = 0; c < KP; ++c) acc[c] = (floatx2)(0.f);
      for (int q = 0; q < (fp >> 2); q += CPI) {
        floatx4 cc[CPI][KP];
#pragma unroll
        for (int u = 0; u < CPI; ++u)
#pragma unroll
          for (int c = 0; c < KP; ++c) cc[u][c] = Cq[(q + u) * KP + c];
#pragma unroll
        for (int u = 0; u < CPI; ++u)
          ks_chunk<KP>(cc[u], *reinterpret_cast<const floatx4*>(xr + 4 * (q + u)), acc);
      }
      float best = acc[0][0] + acc[0][1];
      int bi = 0;
#pragma unroll
      for (int c = 1; c < KP; ++c) {
        const float d = acc[c][0] + acc[c][1];
        const bool better = d < best;
        best = better ? d : best;
        bi = better ? c : bi;
      }
      if (tid < rows) {
        if (labels) labels[row0 + tid] = bi;
        if (mind) mind[row0 + tid] = best;
      }
      lab[tid] = tid < rows ? bi : -1;
    }
    if (UPDATE) {
      __syncthreads();
      // ---- update on the matrix cores: S[c][j] += sum_r onehot[r][c] X[r][j] with
      // v_mfma_f32_16x16x4_f32 (A = onehot^T, 16 clusters x 4 rows; B = 4 rows x 16 features;
      // 0/1 weights: exact fp32 products, fp32 accumulation). Wave w owns feature blocks w, w + 2.
      const int kq = lane >> 4, c16 = lane & 15;
      // UG independent accumulator chains per block (a single chain serialises on the MFMA result)
#pragma unroll 2
      for (int r0 = 0; r0 < KS_ROWS; r0 += 4 * UG) {
#pragma unroll
        for (int g = 0; g < UG; ++g) {
          const int r = r0 + 4 * g + kq;
          const float a = lab[r] == c16 ? 1.f : 0.f;
          const float* xrow = tile + r * ld + c16;
          // no branch around the MFMAs (it kept the LDS reads from being hoisted: +0.5 ms): blocks
          // past f read in-bounds LDS and land in discarded columns
#pragma unroll
          for (int b = 0; b < UB; ++b)
            uacc[b][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, xrow[(wave + KS_WAVES * b) * 16], uacc[b][g], 0, 0,
                                                              0);
        }
      }
      if (wave == 0) {
#pragma unroll
        for (int c = 0; c < KP; ++c) {
          // ballots outside the lane select: a ballot inside it would only see lane c
          const int cnt = __popcll(__ballot(lab[lane] == c)) + __popcll(__ballot(lab[64 + lane] == c));
          ucnt += lane == c ? (float)cnt : 0.f;
        }
      }
    }
    __syncthreads();  // the tile is overwritten next
  }
  if (UPDATE) {
    // partials: sums_part[block][c][64] (D layout: col = lane & 15, row = 4 (lane >> 4) + reg),
    // counts_part[block][c]
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int cb = wave + KS_WAVES * b;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * (lane >> 4) + i;
        if (c < KP && cb < NFB)
          sums_part[((int64_t)blockIdx.x * KP + c) * KS_FMAX + cb * 16 + (lane & 15)] =
              (uacc[b][0][i] + uacc[b][1][i]) + (uacc[b][2][i] + uacc[b][3][i]);
      }
    }
    if (wave == 0 && lane < KP) counts_part[(int64_t)blockIdx.x * KP + lane] = ucnt;
  }
}

// The common case as its own kernel: f = 64, 16-byte aligned rows, whole 128-row tiles (the
// generic kernel above takes the tail). Fixed index math keeps the register file to the prefetch
// buffer, the accumulators and ONE live load address: in the generic kernel the compiler hoists
// the per-piece row/column/LDS offsets of the guarded load/store loops out of the tile loop (~60
// VGPRs + spills to AGPRs at 256 registers), and the SGPR-resident centroids spilled into VGPR
// lanes. Thread t's pieces are rows (t >> 4) + 8 i, features 4 (t & 15) .. +3: each load
// instruction covers 4 whole 256-byte rows, and the LDS stores use immediate offsets.
// AHEAD = 2: two register buffers, the loads of tile t + 2 G in flight while tile t is computed
// (151 -> ~215 VGPRs, still two waves per SIMD); AHEAD = 1: one buffer, tile t + G.
template <int KP, bool UPDATE, int AHEAD>
__global__ __launch_bounds__(KS_ROWS, 2) void ks_step64(const float* __restrict__ X, int64_t ntiles, int64_t ldx,
                                                        const float* __restrict__ Cp, int* __restrict__ labels,
                                                        float* __restrict__ mind, float* __restrict__ sums_part,
                                                        float* __restrict__ counts_part) {
  constexpr int LD = KS_LDMAX;
  __shared__ __attribute__((aligned(16))) float tile[KS_ROWS * LD];
  __shared__ int lab[KS_ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c4 = tid & 15, rb = tid >> 4;
  if (tid < KS_ROWS) *reinterpret_cast<floatx4*>(tile + tid * LD + KS_FMAX) = (floatx4)(0.f);  // row padding
  floatx4 uacc[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int g = 0; g < 4; ++g) uacc[b][g] = (floatx4)(0.f);
  float ucnt = 0.f;
  floatx4 buf0[16], buf1[16];
  const int64_t pstride = 8 * ldx;
  typedef const floatx4 __attribute__((address_space(1)))* gptr;  // global, not flat (flat loads count in lgkmcnt)
  auto load = [&](floatx4(&buf)[16], int64_t t) {
    gptr p = (gptr)(X + (t * KS_ROWS + rb) * ldx + 4 * c4);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      buf[i] = __builtin_nontemporal_load(p);
      p += pstride / 4;
      asm volatile("" : "+v"(p));  // one live address, not 16 hoisted ones
    }
  };
  float* const st = tile + rb * LD + 4 * c4;
  const floatx4* Cq = reinterpret_cast<const floatx4*>(Cp);
  constexpr int CPI = KP <= 8 ? 2 : 1;
  auto process = [&](floatx4(&buf)[16], int64_t t, int64_t tnext) {
#pragma unroll
    for (int i = 0; i < 16; ++i) *reinterpret_cast<floatx4*>(st + i * 8 * LD) = buf[i];
    __syncthreads();
    if (tnext < ntiles) load(buf, tnext);  // in flight during this tile's (and the next one's) compute
    const int64_t row0 = t * KS_ROWS;
    {
      const float* xr = tile + tid * LD;
      floatx2 acc[KP];
#pragma unroll
      for (int c = 0; c < KP; ++c) acc[c] = (floatx2)(0.f);
      for (int q = 0; q < KS_FMAX / 4; q += CPI) {
        floatx4 cc[CPI][KP];
#pragma unroll
        for (int u = 0; u < CPI; ++u)
#pragma unroll
          for (int c = 0; c < KP; ++c) cc[u][c] = Cq[(q + u) * KP + c];
#pragma unroll
        for (int u = 0; u < CPI; ++u)
          ks_chunk<KP>(cc[u], *reinterpret_cast<const floatx4*>(xr + 4 * (q + u)), acc);
      }
      float best = acc[0][0] + acc[0][1];
      int bi = 0;
#pragma unroll
      for (int c = 1; c < KP; ++c) {
        const float d = acc[c][0] + acc[c][1];
        const bool better = d < best;
        best = better ? d : best;
        bi = better ? c : bi;
      }
      if (labels) labels[row0 + tid] = bi;
      if (mind) mind[row0 + tid] = best;
      lab[tid] = bi;
    }
    if (UPDATE) {
      __syncthreads();
      // onehot(labels)^T X on v_mfma_f32_16x16x4_f32, wave w owns feature blocks w and w + 2
      const int kq = lane >> 4, c16 = lane & 15;
#pragma unroll 2
      for (int r0 = 0; r0 < KS_ROWS; r0 += 16) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int r = r0 + 4 * g + kq;
          const float a = lab[r] == c16 ? 1.f : 0.f;
          const float* xrow = tile + r * LD + c16;
#pragma unroll
          for (int b = 0; b < 2; ++b)
            uacc[b][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, xrow[(wave + 2 * b) * 16], uacc[b][g], 0, 0, 0);
        }
      }
      if (wave == 0) {
#pragma unroll
        for (int c = 0; c < KP; ++c) {
          const int cnt = __popcll(__ballot(lab[lane] == c)) + __popcll(__ballot(lab[64 + lane] == c));
          ucnt += lane == c ? (float)cnt : 0.f;
        }
      }
    }
    __syncthreads();  // the tile is overwritten next
  };
  const int64_t G = gridDim.x;
  int64_t t = blockIdx.x;
  if (AHEAD == 2) {
    if (t < ntiles) load(buf0, t);
    if (t + G < ntiles) load(buf1, t + G);
    for (; t < ntiles; t += 2 * G) {
      process(buf0, t, t + 2 * G);
      if (t + G >= ntiles) break;
      process(buf1, t + G, t + 3 * G);
    }
  } else {
    if (t < ntiles) load(buf0, t);
    for (; t < ntiles; t += G) process(buf0, t, t + G);
  }
  if (UPDATE) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int cb = wave + 2 * b;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * (lane >> 4) + i;
        if (c < KP)
          sums_part[((int64_t)blockIdx.x * KP + c) * KS_FMAX + cb * 16 + (lane & 15)] =
              (uacc[b][0][i] + uacc[b][1][i]) + (uacc[b][2][i] + uacc[b][3][i]);
      }
    }
    if (wave == 0 && lane < KP) counts_part[(int64_t)blockIdx.x * KP + lane] = ucnt;
  }
}

// One-wave workgroups over 64-row tiles (f = 64): no workgroup barrier at all (a wave's LDS
// operations execute in order), 17.7 KB of LDS per wave, so 8-9 independent waves per CU each
// with its next tile in flight, instead of 4 two-wave workgroups stepping through 3 barriers per
// tile. The wave does the whole update of its tile: 4 feature blocks x 16 row steps of
// v_mfma_f32_16x16x4_f32; the counts come from ballots of the lane's own label.
// AH = 2: two register buffers, the loads of tiles t + G and t + 2 G in flight during tile t (twice
// the bytes in flight per wave; 149 -> ~213 VGPRs, still two waves per SIMD).
template <int KP, bool UPDATE, int AH = 1>
__global__ __launch_bounds__(64, 2) void ks_wave64(const float* __restrict__ X, int64_t n, int64_t ntiles, int64_t ldx,
                                                   const float* __restrict__ Cp, int* __restrict__ labels,
                                                   float* __restrict__ mind, float* __restrict__ sums_part,
                                                   float* __restrict__ counts_part) {
  constexpr int LD = KS_LDMAX;
  __shared__ __attribute__((aligned(16))) float tile[64 * LD];
  __shared__ int lab[64];
  const int lane = threadIdx.x;
  const int c4 = lane & 15, rb = lane >> 4;
  *reinterpret_cast<floatx4*>(tile + lane * LD + KS_FMAX) = (floatx4)(0.f);  // row padding
  floatx4 uacc[4][2];
#pragma unroll
  for (int b = 0; b < 4; ++b) uacc[b][0] = uacc[b][1] = (floatx4)(0.f);
  floatx4 u4[KP <= 8 ? KP / 4 : 1][4];
#pragma unroll
  for (int g = 0; g < (KP <= 8 ? KP / 4 : 1); ++g)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) u4[g][s4] = (floatx4)(0.f);
  float ucnt = 0.f;
  floatx4 buf[16], buf2[AH == 2 ? 16 : 1];
  typedef const floatx4 __attribute__((address_space(1)))* gptr;
  // the partial last tile is read as the LAST 64 rows (n >= 64); its rows below 64 t belong to the
  // previous tile and are excluded (valid) - no branch in the load (a branch cost the loop head its
  // vmcnt(16) and 26 VGPRs)
  auto tile_row0 = [&](int64_t t) __attribute__((always_inline)) { return t * 64 < n - 64 ? t * 64 : n - 64; };
  auto load = [&](floatx4* b, int64_t t) __attribute__((always_inline)) {
    gptr p = (gptr)(X + (tile_row0(t) + rb) * ldx + 4 * c4);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      b[i] = __builtin_nontemporal_load(p);
      p += ldx;  // 4 rows on (4 ldx floats)
      asm volatile("" : "+v"(p));
    }
  };
  float* const st = tile + rb * LD + 4 * c4;
  const floatx4* Cq = reinterpret_cast<const floatx4*>(Cp);
  constexpr int CPI = KP <= 8 ? 2 : 1;
  const int64_t G = gridDim.x;
  // stage tile t from buffer b, refill b with tile t + AH G, then assign (and sum) tile t
  auto body = [&](floatx4* b, int64_t t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) *reinterpret_cast<floatx4*>(st + i * 4 * LD) = b[i];
    // AH = 2: the refill is unconditional (past the end: the last tile again, an L2 hit) so that the
    // compiler's vmcnt at the loop head counts the other buffer's loads as younger (a conditional
    // refill made it wait for all of them)
    if (AH == 2) load(b, t + AH * G < ntiles ? t + AH * G : ntiles - 1);
    else if (t + AH * G < ntiles) load(b, t + AH * G);
    const int64_t row0 = tile_row0(t);
    const bool valid = row0 + lane >= t * 64;
    int bi = 0;
    {
      const float* xr = tile + lane * LD;
      floatx2 acc[KP];
#pragma unroll
      for (int c = 0; c < KP; ++c) acc[c] = (floatx2)(0.f);
      for (int q = 0; q < KS_FMAX / 4; q += CPI) {
        floatx4 cc[CPI][KP];
#pragma unroll
        for (int u = 0; u < CPI; ++u)
#pragma unroll
          for (int c = 0; c < KP; ++c) cc[u][c] = Cq[(q + u) * KP + c];
#pragma unroll
        for (int u = 0; u < CPI; ++u)
          ks_chunk<KP>(cc[u], *reinterpret_cast<const floatx4*>(xr + 4 * (q + u)), acc);
      }
      float best = acc[0][0] + acc[0][1];
#pragma unroll
      for (int c = 1; c < KP; ++c) {
        const float d = acc[c][0] + acc[c][1];
        const bool better = d < best;
        best = better ? d : best;
        bi = better ? c : bi;
      }
      if (valid && labels) labels[row0 + lane] = bi;
      if (valid && mind) mind[row0 + lane] = best;
    }
    if (UPDATE) {
      lab[lane] = valid ? bi : -1;
      if constexpr (KP <= 8) {
        // onehot^T X on v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4 x 4, one row each; layout probed
        // by tools/probes/mfma4x4_probe.hip: A_b[m] / B_b[n] in lane 4 b + m / 4 b + n, D reg m of
        // lane 4 b + n): block b = (feature quad fq = b >> 2, row rr = b & 3), so one MFMA covers 4
        // rows x 16 features x 4 clusters - no padding rows, half (k = 8) or a quarter (k <= 4)
        // of the 16x16x4 form's matrix-core cycles. The 4 row blocks' partials are summed at the end.
        const int q = lane & 3, rr = (lane >> 2) & 3, fq = lane >> 4;
        const float* xb = tile + rr * LD + 4 * fq + q;
#pragma unroll 4
        for (int r0 = 0; r0 < 64; r0 += 4) {
          const int rl = lab[r0 + rr];
          float a[KP / 4];
#pragma unroll
          for (int g = 0; g < KP / 4; ++g) a[g] = rl == 4 * g + q ? 1.f : 0.f;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const float xv = xb[r0 * LD + 16 * s4];
#pragma unroll
            for (int g = 0; g < KP / 4; ++g) u4[g][s4] = __builtin_amdgcn_mfma_f32_4x4x1f32(a[g], xv, u4[g][s4], 0, 0, 0);
          }
        }
      } else {
        const int kq = lane >> 4, c16 = lane & 15;
#pragma unroll 4
        for (int r0 = 0; r0 < 64; r0 += 8) {
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            const int r = r0 + 4 * g + kq;
            const float a = lab[r] == c16 ? 1.f : 0.f;
            const float* xrow = tile + r * LD + c16;
#pragma unroll
            for (int b = 0; b < 4; ++b)
              uacc[b][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, xrow[16 * b], uacc[b][g], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < KP; ++c) {
        const int cnt = __popcll(__ballot(valid && bi == c));
        ucnt += lane == c ? (float)cnt : 0.f;
      }
    }
  };
  int64_t t = blockIdx.x;
  if constexpr (AH == 2) {
    load(buf, t < ntiles ? t : ntiles - 1);  // the launch has at most ntiles workgroups
    load(buf2, t + G < ntiles ? t + G : ntiles - 1);
    // whole pairs in the loop, an odd last tile after it (a break between the two bodies made the
    // loop head a merge point of both buffers' states: full vmcnt waits)
    const int64_t cnt = (ntiles - t + G - 1) / G;
    for (int64_t i = 0; i + 1 < cnt; i += 2, t += 2 * G) {
      body(buf, t);
      body(buf2, t + G);
    }
    if (cnt & 1) body(buf, t);
  } else {
    if (t < ntiles) load(buf, t);
    for (; t < ntiles; t += G) body(buf, t);
  }
  if (UPDATE) {
    if constexpr (KP <= 8) {
      // sum the 4 row blocks (lane bits 2-3), then lanes of row block 0 write cluster 4 g + m,
      // feature 16 s + 4 fq + q
      const int q = lane & 3, rr = (lane >> 2) & 3, fq = lane >> 4;
#pragma unroll
      for (int g = 0; g < KP / 4; ++g)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            float v = u4[g][s4][m];
            v += __shfl_xor(v, 4, 64);
            v += __shfl_xor(v, 8, 64);
            if (rr == 0)
              sums_part[((int64_t)blockIdx.x * KP + 4 * g + m) * KS_FMAX + 16 * s4 + 4 * fq + q] = v;
          }
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 4 * (lane >> 4) + i;
          if (c < KP) sums_part[((int64_t)blockIdx.x * KP + c) * KS_FMAX + b * 16 + (lane & 15)] = uacc[b][0][i] + uacc[b][1][i];
        }
      }
    }
    if (lane < KP) counts_part[(int64_t)blockIdx.x * KP + lane] = ucnt;
  }
}

// this thread's share (partials threadIdx.x + 256 i) of one output's partial sums, in fp64: eight
// independent loads in flight per round (one at a time the loop was latency-bound: 10.5 us for the
// 2049 partials of k = 8, f = 64 in the r5kstrace trace); fixed order for a given nblk
template <int KP>
__device__ __forceinline__ double ks_part_sum(const float* __restrict__ sums_part, const float* __restrict__ counts_part,
                                             int nblk, bool is_sum, int c, int j) {
  const float* base = is_sum ? sums_part + (int64_t)c * KS_FMAX + j : counts_part + c;
  const int64_t stride = is_sum ? (int64_t)KP * KS_FMAX : KP;
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int b = threadIdx.x;
  for (; b + 7 * 256 < nblk; b += 8 * 256) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base[(int64_t)(b + 256 * u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += (double)v[u];
  }
  for (int u = 0; b < nblk; b += 256, ++u) a[u & 7] += (double)base[(int64_t)b * stride];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// sums[c][j] = sum over the workgroups' partials (fp64), counts[c] likewise: one workgroup per
// output, its threads stride over the partials (a thread-per-output loop over ~1000 partials was
// latency-bound at ~0.5 ms)
template <int KP>
__global__ __launch_bounds__(256) void ks_reduce(const float* __restrict__ sums_part,
                                                 const float* __restrict__ counts_part, int nblk, int k, int f,
                                                 float* __restrict__ sums, float* __restrict__ counts) {
  __shared__ double red[4];
  const int e = blockIdx.x;
  const bool is_sum = e < k * f;
  const int c = is_sum ? e / f : e - k * f, j = is_sum ? e - c * f : 0;
  double a = ks_part_sum<KP>(sums_part, counts_part, nblk, is_sum, c, j);
  a = ha_wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = (red[0] + red[1]) + (red[2] + red[3]);
    if (is_sum)
      sums[e] = (float)t;
    else
      counts[c] = (float)t;
  }
}

// new centroids (empty clusters keep theirs), the squared shift (fp64, fixed order) and the next
// pass's padded centroid chunks from the fp64 sums / counts in red; one block
template <int KP>
__device__ __forceinline__ void ks_fin_body(int k, int f, const float* __restrict__ C, int64_t ldc,
                                            float* __restrict__ newC, double* __restrict__ shift,
                                            const double* __restrict__ red, unsigned* __restrict__ arrived,
                                            float* __restrict__ cpad, double* wred) {
  const int kf = k * f;
  double acc = 0.0;
  for (int i = threadIdx.x; i < kf; i += 256) {
    const int ci = i / f, ji = i - ci * f;
    const double cnt = red[kf + ci];
    const float old = C[(int64_t)ci * ldc + ji];
    const float nv = cnt > 0.0 ? (float)(red[i] / cnt) : old;
    newC[i] = nv;
    const double d = (double)old - (double)nv;
    acc = fma(d, d, acc);
  }
  acc = ha_wave_sum_d(acc);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = acc;
  __syncthreads();  // also: newC of every thread of this block is visible below
  if (threadIdx.x == 0) {
    *shift = (wred[0] + wred[1]) + (wred[2] + wred[3]);
    if (arrived) *arrived = 0u;  // ready for the next launch on this workspace
  }
  // the next pass's padded chunks (ks_pad_centroids' layout) from the new centroids
  const int fp = ks_fp(f);
  for (int e2 = threadIdx.x; e2 < KP * (fp + 4); e2 += 256) {
    const int q = e2 / (4 * KP), c2 = (e2 / 4) % KP, j2 = 4 * q + (e2 & 3);
    cpad[e2] = c2 < k ? (j2 < f ? newC[c2 * f + j2] : 0.f) : (j2 == 0 ? __builtin_huge_valf() : 0.f);
  }
}

// The Lloyd epilogue fused into the partial-sum reduction (world of one): every block reduces one
// sum / count like ks_reduce, in fp64, into `red`; the last block to arrive (self-resetting counter)
// forms the new centroids (empty clusters keep theirs), the squared shift (fp64, fixed order) and
// the padded centroid chunks of the NEXT pass in place of this pass's. One launch instead of
// ks_reduce + km_finalize + the next pass's ks_pad_centroids: measured, every extra small launch
// between two passes over the points made the next pass slower (a fit loop with the separate
// finalize alternated 0.58 / 0.71 ms per pass, back-to-back passes ran 0.62 ms; tools/microbench/
// smallk_fitloop2.py).
template <int KP>
__global__ __launch_bounds__(256) void ks_reduce_fin(const float* __restrict__ sums_part,
                                                     const float* __restrict__ counts_part, int nblk, int k, int f,
                                                     const float* __restrict__ C, int64_t ldc, float* __restrict__ newC,
                                                     double* __restrict__ shift, double* __restrict__ red,
                                                     unsigned* __restrict__ arrived, float* __restrict__ cpad) {
  __shared__ double wred[4];
  __shared__ bool last;
  const int e = blockIdx.x;
  const int kf = k * f;
  const bool is_sum = e < kf;
  const int c = is_sum ? e / f : e - kf, j = is_sum ? e - c * f : 0;
  double a = ks_part_sum<KP>(sums_part, counts_part, nblk, is_sum, c, j);
  a = ha_wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    red[e] = (wred[0] + wred[1]) + (wred[2] + wred[3]);
    if (arrived) {
      __threadfence();
      last = atomicAdd(arrived, 1u) == gridDim.x - 1;
    } else {
      last = false;
    }
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  ks_fin_body<KP>(k, f, C, ldc, newC, shift, red, arrived, cpad, wred);
}

// The last step of the Lloyd epilogue as its own one-block launch (after ks_reduce_fin with
// arrived = null): with two tiles of loads in flight per wave (ks_wave64<.., 2>) the pass no longer
// slows down after small launches, and the fused form's per-block agent-scope fence + atomic on one
// counter cost more than this launch (tools/r5/gpu_ksw2.sh, tools/r5/gpu_ksfin.sh)
template <int KP>
__global__ __launch_bounds__(256) void ks_fin(int k, int f, const float* __restrict__ C, int64_t ldc,
                                              float* __restrict__ newC, double* __restrict__ shift,
                                              const double* __restrict__ red, float* __restrict__ cpad) {
  __shared__ double wred[4];
  ks_fin_body<KP>(k, f, C, ldc, newC, shift, red, nullptr, cpad, wred);
}
int ks_kp(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : 16; }

template <int KP, int MODE, bool U>
void ks_launch_generic(int nblk, hipStream_t s, const float* X, int64_t n, int f, int64_t ldx, const float* cpad,
                       int* labels, float* mind, float* sp, float* cp) {
  if (U && f <= 32)
    hipLaunchKernelGGL((ks_step<KP, MODE, U, 2>), dim3(nblk), dim3(KS_ROWS), 0, s, X, n, f, ldx, cpad, labels, mind,
                       sp, cp);
  else
    hipLaunchKernelGGL((ks_step<KP, MODE, U, 4>), dim3(nblk), dim3(KS_ROWS), 0, s, X, n, f, ldx, cpad, labels, mind,
                       sp, cp);
}

// one pass: ks_step64 over the whole tiles when it applies (f = 64, aligned rows) plus the
// generic kernel on the remaining rows as ONE extra partial slot, else the generic kernel alone;
// then the fp64 reduction of the partials
// Fused Lloyd epilogue of ha_ks_lloyd (null: the plain sums / counts reduction)
struct KsFin {
  const float* C;
  int64_t ldc;
  float* newC;
  double* shift;
  double* red;
  unsigned* arrived;
  float* cpad;
};

template <int KP, bool U>
void ks_launch(int mode, int num_cus, hipStream_t s, const float* X, int64_t n, int f, int64_t ldx, const float* cpad,
               int* labels, float* mind, float* sp, float* cp, int k, float* sums, float* counts,
               const KsFin* fin = nullptr) {
  int nblk = 0;
  int64_t done = 0;
  if (mode == KS_ROW4 && f == KS_FMAX) {
    const int64_t full = n / KS_ROWS;
    // HEAT_KS_VARIANT: "w2" (default: one-wave workgroups, 64-row tiles, two tiles of loads in flight
    // per wave: 0.614-0.62 vs 0.616-0.70 ms per pass in the Lloyd-loop variants of
    // smallk_fitloop2.py, tools/r5/gpu_ksw2.sh), "wave" (one tile in flight), "a1" / "a2" (two-wave
    // workgroups, 128-row tiles, one / two tiles of loads in flight). Measured on one box
    // (smallk_ab_r05.jsonl), n = 12.5M, f = 64, fused pass: wave 0.734 / 0.978 / 0.611 ms at
    // k = 8 / 16 / 3 vs a1 0.767 / 1.018 / 0.654 and a2 0.780 / 1.048 / 0.663.
    static const int variant = [] {
      const char* e = getenv("HEAT_KS_VARIANT");
      return !e ? 3 : e[0] == 'w' ? (e[1] == '2' ? 3 : 0) : e[1] == '2' ? 2 : 1;
    }();
    if ((variant == 0 || variant == 3) && n / 64 > 0) {
      // w2 also takes the partial last tile (no tail launch: 13.7 us per pass in the r5kstrace trace)
      const int64_t full64 = variant == 3 ? (n + 63) / 64 : n / 64;
      static const int wpc = [] {  // waves per CU (LDS holds 9 of 17.7 KB)
        const char* e = getenv("HEAT_KS_WPC");
        const int v = e ? atoi(e) : 8;
        return v < 1 ? 1 : v > 9 ? 9 : v;
      }();
      nblk = (int)(full64 < (int64_t)wpc * num_cus ? full64 : (int64_t)wpc * num_cus);
      if (variant == 3)  // HEAT_KS_VARIANT=w2: two tiles of loads in flight per wave
        hipLaunchKernelGGL((ks_wave64<KP, U, 2>), dim3(nblk), dim3(64), 0, s, X, n, full64, ldx, cpad, labels, mind,
                           sp, cp);
      else
        hipLaunchKernelGGL((ks_wave64<KP, U>), dim3(nblk), dim3(64), 0, s, X, full64 * 64, full64, ldx, cpad, labels,
                           mind, sp, cp);
      done = variant == 3 ? n : full64 * 64;
    } else if (full > 0) {
      nblk = (int)(full < 4 * num_cus ? full : 4 * num_cus);
      if (variant == 2)
        hipLaunchKernelGGL((ks_step64<KP, U, 2>), dim3(nblk), dim3(KS_ROWS), 0, s, X, full, ldx, cpad, labels, mind, sp,
                           cp);
      else
        hipLaunchKernelGGL((ks_step64<KP, U, 1>), dim3(nblk), dim3(KS_ROWS), 0, s, X, full, ldx, cpad, labels, mind, sp,
                           cp);
      done = full * KS_ROWS;
    }
  }
  const int64_t rest = n - done;
  if (rest > 0) {
    const int64_t ntiles = (rest + KS_ROWS - 1) / KS_ROWS;
    const int g = done > 0 ? 1 : (int)(ntiles < 4 * num_cus ? ntiles : 4 * num_cus);
    const float* Xr = X + done * ldx;
    int* lr = labels ? labels + done : nullptr;
    float* mr = mind ? mind + done : nullptr;
    float* spr = sp + (int64_t)nblk * KP * KS_FMAX;
    float* cpr = cp + (int64_t)nblk * KP;
    if (mode == KS_ROW4)
      ks_launch_generic<KP, KS_ROW4, U>(g, s, Xr, rest, f, ldx, cpad, lr, mr, spr, cpr);
    else if (mode == KS_FLAT)
      ks_launch_generic<KP, KS_FLAT, U>(g, s, Xr, rest, f, ldx, cpad, lr, mr, spr, cpr);
    else
      ks_launch_generic<KP, KS_SCALAR, U>(g, s, Xr, rest, f, ldx, cpad, lr, mr, spr, cpr);
    nblk += g;
  }
  // HEAT_KS_FIN=fused: the last-arriving reduction block finishes the step (one launch; the default
  // is the reduction and a one-block ks_fin)
  static const bool fin_fused = [] {
    const char* e = getenv("HEAT_KS_FIN");
    return e && e[0] == 'f';
  }();
  if (U && fin && fin_fused) {
    hipLaunchKernelGGL((ks_reduce_fin<KP>), dim3((unsigned)(k * f + k)), dim3(256), 0, s, sp, cp, nblk, k, f, fin->C,
                       fin->ldc, fin->newC, fin->shift, fin->red, fin->arrived, fin->cpad);
  } else if (U && fin) {
    hipLaunchKernelGGL((ks_reduce_fin<KP>), dim3((unsigned)(k * f + k)), dim3(256), 0, s, sp, cp, nblk, k, f, fin->C,
                       fin->ldc, fin->newC, fin->shift, fin->red, (unsigned*)nullptr, fin->cpad);
    hipLaunchKernelGGL((ks_fin<KP>), dim3(1), dim3(256), 0, s, k, f, fin->C, fin->ldc, fin->newC, fin->shift, fin->red,
                       fin->cpad);
  }
  else if (U)
    hipLaunchKernelGGL((ks_reduce<KP>), dim3((unsigned)(k * f + k)), dim3(256), 0, s, sp, cp, nblk, k, f, sums, counts);
}

// partial slots: up to 9 per CU + one for the tail rows of the f = 64 kernels
int ks_slots(int num_cus) { return 9 * num_cus + 1; }

}  // namespace

HA_EXPORT int ha_ks_max_k() { return 16; }
HA_EXPORT int ha_ks_max_f() { return KS_FMAX; }

// Workspace floats: per-workgroup partials (nblk = 4 workgroups per CU) + the padded centroids.
HA_EXPORT int64_t ha_ks_workspace_floats(int k, int num_cus) {
  if (k <= 0 || k > 16 || num_cus <= 0) return -1;
  return (int64_t)ks_slots(num_cus) * ks_kp(k) * (KS_FMAX + 1) + (int64_t)ks_kp(k) * (KS_FMAX + 4);
}

// One pass over X [n, f] (f <= 64, k <= 16): labels (int32, optional), mind (optional) and, when
// sums != nullptr, per-cluster feature sums [k, f] and counts [k] (fp64-reduced, stored fp32).
HA_EXPORT int ha_ks_step(const float* X, int64_t n, int f, int64_t ldx, const float* C, int k, int64_t ldc,
                         int* labels, float* mind, float* sums, float* counts, float* workspace, int num_cus,
                         void* stream) {
  if (k <= 0 || k > 16 || f <= 0 || f > KS_FMAX || ldx < f || ldc < f || num_cus <= 0) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int kp = ks_kp(k);
  const bool al = ((uintptr_t)X & 15) == 0;
  const int mode = (f % 4 == 0 && ldx % 4 == 0 && al) ? KS_ROW4 : (ldx == f && f >= 4 && al) ? KS_FLAT : KS_SCALAR;
  const bool upd = sums != nullptr;
  const int64_t slots = ks_slots(num_cus);
  float* sp = workspace;
  float* cp = workspace + slots * kp * KS_FMAX;
  float* cpad = workspace + slots * kp * (KS_FMAX + 1);
  if (upd && n <= 0) {
    (void)hipMemsetAsync(sums, 0, (size_t)k * f * sizeof(float), s);
    (void)hipMemsetAsync(counts, 0, (size_t)k * sizeof(float), s);
    return ha_launch_status();
  }
  if (n <= 0) return HA_OK;
  hipLaunchKernelGGL(ks_pad_centroids, dim3((unsigned)((kp * (ks_fp(f) + 4) + 255) / 256)), dim3(256), 0, s, C, k, f,
                     ldc, kp, cpad);
#define HA_KS(KP)                                                                                            \
  if (upd)                                                                                                   \
    ks_launch<KP, true>(mode, num_cus, s, X, n, f, ldx, cpad, labels, mind, sp, cp, k, sums, counts);        \
  else                                                                                                       \
    ks_launch<KP, false>(mode, num_cus, s, X, n, f, ldx, cpad, labels, mind, sp, cp, k, sums, counts);
  if (kp == 4) {
    HA_KS(4)
  } else if (kp == 8) {
    HA_KS(8)
  } else {
    HA_KS(16)
  }
#undef HA_KS
  return ha_launch_status();
}

// Workspace floats of ha_ks_lloyd: ha_ks_workspace_floats + the fp64 reduction (k f + k) and the
// arrival counter. Zero it once (the counter self-resets); keep it between the calls of one fit.
HA_EXPORT int64_t ha_ks_lloyd_workspace_floats(int k, int num_cus) {
  const int64_t base = ha_ks_workspace_floats(k, num_cus);
  if (base < 0) return -1;
  return base + 2 * ((int64_t)k * KS_FMAX + k) + 4;
}

// One Lloyd step for few clusters on a world of one (k <= 16, f <= 64): labels (int32, optional),
// newC [k, f] (contiguous) = the means of the assigned points (empty clusters keep their centroid),
// shift = sum (C - newC)^2 (fp64). pad_ready != 0: the workspace already holds the padded chunks of
// C (the previous call's newC, written by its epilogue) - no pad launch.
HA_EXPORT int ha_ks_lloyd(const float* X, int64_t n, int f, int64_t ldx, const float* C, int k, int64_t ldc,
                          int* labels, float* newC, double* shift, float* workspace, int num_cus, int pad_ready,
                          void* stream) {
  if (k <= 0 || k > 16 || f <= 0 || f > KS_FMAX || ldx < f || ldc < f || num_cus <= 0 || n <= 0) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int kp = ks_kp(k);
  const bool al = ((uintptr_t)X & 15) == 0;
  const int mode = (f % 4 == 0 && ldx % 4 == 0 && al) ? KS_ROW4 : (ldx == f && f >= 4 && al) ? KS_FLAT : KS_SCALAR;
  const int64_t slots = ks_slots(num_cus);
  float* sp = workspace;
  float* cp = workspace + slots * kp * KS_FMAX;
  float* cpad = workspace + slots * kp * (KS_FMAX + 1);
  double* red = reinterpret_cast<double*>(workspace + ha_ks_workspace_floats(k, num_cus) + 1);
  red = reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(red) + 7) & ~(uintptr_t)7);
  unsigned* arrived = reinterpret_cast<unsigned*>(red + (int64_t)k * KS_FMAX + k);
  if (!pad_ready)
    hipLaunchKernelGGL(ks_pad_centroids, dim3((unsigned)((kp * (ks_fp(f) + 4) + 255) / 256)), dim3(256), 0, s, C, k,
                       f, ldc, kp, cpad);
  const KsFin fin{C, ldc, newC, shift, red, arrived, cpad};
  if (kp == 4)
    ks_launch<4, true>(mode, num_cus, s, X, n, f, ldx, cpad, labels, nullptr, sp, cp, k, nullptr, nullptr, &fin);
  else if (kp == 8)
    ks_launch<8, true>(mode, num_cus, s, X, n, f, ldx, cpad, labels, nullptr, sp, cp, k, nullptr, nullptr, &fin);
  else
    ks_launch<16, true>(mode, num_cus, s, X, n, f, ldx, cpad, labels, nullptr, sp, cp, k, nullptr, nullptr, &fin);
  return ha_launch_status();
}
