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

#include <type_traits>

namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));

constexpr int KS_ROWS = 128;  // rows per tile = threads per workgroup (2 waves)
constexpr int KS_WAVES = KS_ROWS / 64;
constexpr int KS_FMAX = 64;
constexpr int KS_LDMAX = KS_FMAX + 4;  // padded LDS row stride (words) at f = 64
enum { KS_ROW4 = 0, KS_FLAT = 1, KS_SCALAR = 2 };

// ceil(f / 4) * 4 + 4: 16-byte aligned rows, conflict-free row-per-lane b128 reads
__host__ __device__ inline int ks_ld(int f) { return ((f + 3) / 4) * 4 + 4; }
__host__ __device__ inline int ks_fp(int f) { return ((f + 7) / 8) * 8; }

// padded centroid copy: Cp[c][j] (c < KP, j < FP); rows >= k at +inf, features >= f zero
__global__ __launch_bounds__(256) void ks_pad_centroids(const float* __restrict__ C, int k, int f, int64_t ldc,
                                                        int kp, float* __restrict__ Cp) {
  const int fp = ks_fp(f);
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kp * fp) return;
  const int c = e / fp, j = e - c * fp;
  Cp[e] = c < k ? (j < f ? C[(int64_t)c * ldc + j] : 0.f) : (j == 0 ? __builtin_huge_valf() : 0.f);
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
    // ---- assign: thread = row, centroids as SGPR operands (wave-uniform scalar loads)
    {
      const float* xr = tile + (tid < rows ? tid : 0) * ld;
      floatx2 acc[KP];
#pragma unroll
      for (int c = 0; c < KP; ++c) acc[c] = (floatx2)(0.f);
#pragma unroll 2
      for (int j = 0; j < fp; j += 8) {
        const floatx4 xa = *reinterpret_cast<const floatx4*>(xr + j);
        // xb lies in the row's zero padding when f <= j + 4 (ld >= 4 ceil(f/4) + 4 >= j + 8 then)
        const floatx4 xb = *reinterpret_cast<const floatx4*>(xr + j + 4);
        const floatx2 x0 = {xa[0], xa[1]}, x1 = {xa[2], xa[3]}, x2 = {xb[0], xb[1]}, x3 = {xb[2], xb[3]};
#pragma unroll
        for (int c = 0; c < KP; ++c) {
          const floatx4 ca = *reinterpret_cast<const floatx4*>(Cp + c * fp + j);
          const floatx4 cb = *reinterpret_cast<const floatx4*>(Cp + c * fp + j + 4);
          const floatx2 d0 = x0 - (floatx2){ca[0], ca[1]};
          const floatx2 d1 = x1 - (floatx2){ca[2], ca[3]};
          const floatx2 d2 = x2 - (floatx2){cb[0], cb[1]};
          const floatx2 d3 = x3 - (floatx2){cb[2], cb[3]};
          acc[c] = __builtin_elementwise_fma(d0, d0, acc[c]);
          acc[c] = __builtin_elementwise_fma(d1, d1, acc[c]);
          acc[c] = __builtin_elementwise_fma(d2, d2, acc[c]);
          acc[c] = __builtin_elementwise_fma(d3, d3, acc[c]);
        }
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
  double a = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 256)
    a += is_sum ? (double)sums_part[((int64_t)b * KP + c) * KS_FMAX + j] : (double)counts_part[(int64_t)b * KP + c];
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

int ks_kp(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : 16; }

}  // namespace

HA_EXPORT int ha_ks_max_k() { return 16; }
HA_EXPORT int ha_ks_max_f() { return KS_FMAX; }

// Workspace floats: per-workgroup partials (nblk = 4 workgroups per CU) + the padded centroids.
HA_EXPORT int64_t ha_ks_workspace_floats(int k, int num_cus) {
  if (k <= 0 || k > 16 || num_cus <= 0) return -1;
  return (int64_t)4 * num_cus * ks_kp(k) * (KS_FMAX + 1) + (int64_t)ks_kp(k) * KS_FMAX;
}

// One pass over X [n, f] (f <= 64, k <= 16): labels (int32, optional), mind (optional) and, when
// sums != nullptr, per-cluster feature sums [k, f] and counts [k] (fp64-reduced, stored fp32).
HA_EXPORT int ha_ks_step(const float* X, int64_t n, int f, int64_t ldx, const float* C, int k, int64_t ldc,
                         int* labels, float* mind, float* sums, float* counts, float* workspace, int num_cus,
                         void* stream) {
  if (k <= 0 || k > 16 || f <= 0 || f > KS_FMAX || ldx < f || ldc < f || num_cus <= 0) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int kp = ks_kp(k);
  const int64_t ntiles = (n + KS_ROWS - 1) / KS_ROWS;
  int nblk = 4 * num_cus;
  if (ntiles < nblk) nblk = (int)(ntiles > 0 ? ntiles : 1);
  const bool al = ((uintptr_t)X & 15) == 0;
  const int mode = (f % 4 == 0 && ldx % 4 == 0 && al) ? KS_ROW4 : (ldx == f && f >= 4 && al) ? KS_FLAT : KS_SCALAR;
  const bool upd = sums != nullptr;
  float* sp = workspace;
  float* cp = workspace + (int64_t)4 * num_cus * kp * KS_FMAX;
  float* cpad = workspace + (int64_t)4 * num_cus * kp * (KS_FMAX + 1);
  if (upd && n <= 0) {
    hipMemsetAsync(sums, 0, (size_t)k * f * sizeof(float), s);
    hipMemsetAsync(counts, 0, (size_t)k * sizeof(float), s);
    return ha_launch_status();
  }
  if (n <= 0) return HA_OK;
  hipLaunchKernelGGL(ks_pad_centroids, dim3((unsigned)((kp * ks_fp(f) + 255) / 256)), dim3(256), 0, s, C, k, f, ldc,
                     kp, cpad);
#define HA_KS_L(KP, V, U)                                                                                   \
  if (U && f <= 32)                                                                                         \
    hipLaunchKernelGGL((ks_step<KP, V, U, 2>), dim3(nblk), dim3(KS_ROWS), 0, s, X, n, f, ldx, cpad, labels, mind, sp, \
                       cp);                                                                                 \
  else                                                                                                      \
    hipLaunchKernelGGL((ks_step<KP, V, U, 4>), dim3(nblk), dim3(KS_ROWS), 0, s, X, n, f, ldx, cpad, labels, mind, sp, \
                       cp)
#define HA_KS_M(KP, M)                                                                                      \
  if (upd)                                                                                                  \
    HA_KS_L(KP, M, true);                                                                                   \
  else                                                                                                      \
    HA_KS_L(KP, M, false);
#define HA_KS_KP(KP)                                                                                        \
  if (mode == KS_ROW4) {                                                                                    \
    HA_KS_M(KP, KS_ROW4)                                                                                    \
  } else if (mode == KS_FLAT) {                                                                             \
    HA_KS_M(KP, KS_FLAT)                                                                                    \
  } else {                                                                                                  \
    HA_KS_M(KP, KS_SCALAR)                                                                                  \
  }                                                                                                         \
  if (upd)                                                                                                  \
    hipLaunchKernelGGL((ks_reduce<KP>), dim3((unsigned)(k * f + k)), dim3(256), 0, s, sp, cp, nblk,          \
                       k, f, sums, counts);
  if (kp == 4) {
    HA_KS_KP(4)
  } else if (kp == 8) {
    HA_KS_KP(8)
  } else {
    HA_KS_KP(16)
  }
#undef HA_KS_KP
#undef HA_KS_M
#undef HA_KS_L
  return ha_launch_status();
}
