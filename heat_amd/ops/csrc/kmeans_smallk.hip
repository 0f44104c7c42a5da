// K-means iteration for few clusters (k <= 16, the reference benchmark's k = 8; f <= 64):
// assignment AND centroid sums in one pass over the points.
//
// With k this small the MFMA kernels waste most of a 128-centroid tile on padding and each
// workgroup's short life (stage the centroid image, one tile, store) is latency-bound
// (kmeans_f16x3.hip's filter: 2.3 ms per pass at n = 12.5M, f = 64, k = 8), and the separate
// update re-reads the points (0.8 ms). The arithmetic is 2 n k f flops against n f floats read
// once: the iteration is HBM-bound if the points are read exactly once.
//
// Row-per-lane loads straight from HBM were measured at 1.0 TB/s at f = 64 (64 lanes x 16 B at a
// 256 B stride per instruction re-request every line 8 times and thrash L1/L2), so the points are
// staged: a persistent workgroup (2 waves, 4 per CU) loops over 128-row tiles, loads each tile
// coalesced into LDS
// (row stride f + 1 words: the row-per-thread reads below are bank-conflict free), then
//   assign: thread r owns row r, k difference-form accumulators (sum (x - c)^2, exact fp32, no
//           expansion cancellation) in packed-fp32 pairs, centroids from LDS as wave-wide
//           broadcasts (padding clusters at +inf: no branch in the loop), strict-< argmin (lowest
//           index on ties);
//   update: wave w owns clusters c = w (mod 2), lane j feature j; per 64-row chunk a ballot
//           lists the rows of a cluster and the wave walks only those (4 rows per iteration).
// Each thread issues all of its tile loads before its first LDS write (a load -> wait -> write
// loop kept one 16-byte load in flight per thread: 1.7 TB/s), and the next tile's loads are issued
// right after this tile reached LDS, so they are in flight during its compute.
// Per-workgroup partial sums/counts stay in registers across tiles and are written once; a small
// kernel reduces them in fp64.
#include "common.h"

#include <type_traits>

namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));

constexpr int KS_ROWS = 128;   // rows per tile = threads per workgroup (2 waves)
constexpr int KS_WAVES = KS_ROWS / 64;
constexpr int KS_FMAX = 64;
constexpr int KS_LD = KS_FMAX + 1;

// Staging modes: FLAT (rows contiguous, ldx == f >= 4: the tile is one contiguous span read as
// float4 pieces whatever f is), ROW4 (f % 4 == 0, strided rows), SCALAR (anything else).
enum { KS_FLAT = 0, KS_ROW4 = 1, KS_SCALAR = 2 };

template <int MODE>
struct KsStage {
  typedef typename std::conditional<MODE == KS_SCALAR, float, floatx4>::type piece;
  static constexpr int PER = MODE == KS_SCALAR ? 64 : 16;  // pieces per thread per tile (f = 64)
  static constexpr bool PREFETCH = MODE != KS_SCALAR;    // next tile in registers during compute
};

template <int KP, int MODE, bool UPDATE>
__global__ __launch_bounds__(KS_ROWS, 4) void ks_step(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                  const float* __restrict__ C, int k, int64_t ldc,
                                                  int* __restrict__ labels, float* __restrict__ mind,
                                                  float* __restrict__ sums_part, float* __restrict__ counts_part) {
  using S = KsStage<MODE>;
  typedef typename S::piece piece;
  constexpr int SLOTS = (KP + KS_WAVES - 1) / KS_WAVES;
  constexpr int PER = S::PER;   // (threads == tile rows: pieces per thread do not depend on KS_ROWS)
  __shared__ float tile[KS_ROWS * KS_LD];
  __shared__ __attribute__((aligned(16))) float cl[KP * KS_FMAX];
  __shared__ __attribute__((aligned(16))) int lab[KS_ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t ntiles = (n + KS_ROWS - 1) / KS_ROWS;
  // centroids in LDS (read as wave-wide broadcasts); padding clusters at +inf never win
  for (int e = tid; e < KP * KS_FMAX; e += KS_ROWS) {
    const int c = e / KS_FMAX, j = e - c * KS_FMAX;
    cl[e] = c < k ? (j < f ? C[c * ldc + j] : 0.f) : __builtin_huge_valf();
  }
  float us[SLOTS];
  float uc[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) us[s] = uc[s] = 0.f;

  // piece geometry: a piece is 4 floats (FLAT: of the flat tile, ROW4: of one row) or 1 float
  const int w = MODE == KS_ROW4 ? f >> 2 : f;          // ROW4: pieces per row; else floats per row
  const int step = MODE == KS_FLAT ? 4 * KS_ROWS : KS_ROWS;  // units advanced per piece
  const int qrow = step / w, qrem = step - qrow * w;
  const int start = MODE == KS_FLAT ? 4 * tid : tid;
  const int r_init = start / w, c_init = start - (start / w) * w;
  piece buf[PER];
  auto load = [&](int64_t t) {
    const int64_t row0 = t * KS_ROWS;
    const int rows = (int)(n - row0 < KS_ROWS ? n - row0 : KS_ROWS);
    const float* base = X + row0 * ldx;
    const int tot = MODE == KS_ROW4 ? rows * w : rows * f;   // units in the tile
    int r = r_init, c = c_init;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int u = r * w + c;  // unit index in the tile
      if constexpr (MODE == KS_FLAT) {
        if (u + 3 < tot) {
          buf[i] = *reinterpret_cast<const floatx4*>(base + u);
        } else if (u < tot) {  // tail piece of the last tile: element-wise, never past the data
#pragma unroll
          for (int q = 0; q < 4; ++q) reinterpret_cast<float*>(&buf[i])[q] = u + q < tot ? base[u + q] : 0.f;
        }
      } else if constexpr (MODE == KS_ROW4) {
        if (u < tot) buf[i] = *reinterpret_cast<const floatx4*>(base + (int64_t)r * ldx + 4 * c);
      } else {
        if (u < tot) reinterpret_cast<float*>(&buf[i])[0] = base[(int64_t)r * ldx + c];
      }
      r += qrow;
      c += qrem;
      if (c >= w) {
        c -= w;
        ++r;
      }
    }
  };
  auto store = [&](int rows) {
    const int tot = MODE == KS_ROW4 ? rows * w : rows * f;
    int r = r_init, c = c_init;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int u = r * w + c;
      if (u < tot) {
        if constexpr (MODE == KS_FLAT) {
          int rq = r, cq = c;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (u + q < tot) tile[rq * KS_LD + cq] = reinterpret_cast<const float*>(&buf[i])[q];
            if (++cq == f) {
              cq = 0;
              ++rq;
            }
          }
        } else if constexpr (MODE == KS_ROW4) {
          float* d = tile + r * KS_LD + 4 * c;
#pragma unroll
          for (int q = 0; q < 4; ++q) d[q] = reinterpret_cast<const float*>(&buf[i])[q];
        } else {
          tile[r * KS_LD + c] = reinterpret_cast<const float*>(&buf[i])[0];
        }
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
  if (S::PREFETCH && t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    const int64_t row0 = t * KS_ROWS;
    const int rows = (int)(n - row0 < KS_ROWS ? n - row0 : KS_ROWS);
    if (!S::PREFETCH) load(t);
    store(rows);
    __syncthreads();
    // next tile's loads in flight while this one is processed (software pipelining)
    if (S::PREFETCH && t + gridDim.x < ntiles) load(t + gridDim.x);
    // ---- assign: thread = row; no branches in the centroid loop
    {
      const float* xr = tile + (tid < rows ? tid : 0) * KS_LD;
      floatx2 acc[KP];
#pragma unroll
      for (int c = 0; c < KP; ++c) acc[c] = (floatx2)(0.f);
      int j = 0;
      for (; j + 1 < f; j += 2) {
        const floatx2 x = {xr[j], xr[j + 1]};
#pragma unroll
        for (int c = 0; c < KP; ++c) {
          const floatx2 cv = *reinterpret_cast<const floatx2*>(cl + c * KS_FMAX + j);
          const floatx2 d = x - cv;
          acc[c] = __builtin_elementwise_fma(d, d, acc[c]);
        }
      }
      if (j < f) {
        const float x = xr[j];
#pragma unroll
        for (int c = 0; c < KP; ++c) {
          const float d = x - cl[c * KS_FMAX + j];
          acc[c][0] = fmaf(d, d, acc[c][0]);
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
      // ---- update: wave w owns clusters 2 s + w; per 64-row chunk a ballot lists the cluster's
      // rows and the wave walks only those (4 per iteration), lane = feature
      const float* col = tile + lane;  // lanes >= f read padding; their sums are never used
#pragma unroll
      for (int q = 0; q < SLOTS; ++q) {
        const int cidx = KS_WAVES * q + wave;
        float a = 0.f;
        int cnt = 0;
#pragma unroll
        for (int ch = 0; ch < KS_ROWS / 64; ++ch) {
          uint64_t m = __ballot(lab[ch * 64 + lane] == cidx);
          cnt += __popcll(m);
          while (m) {
            int rr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              rr[i] = m ? (int)__builtin_ctzll(m) : -1;
              m &= m ? m - 1 : 0ull;
            }
            float x[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = rr[i] >= 0 ? col[(ch * 64 + rr[i]) * KS_LD] : 0.f;
            a += (x[0] + x[1]) + (x[2] + x[3]);
          }
        }
        us[q] += a;
        uc[q] += (float)cnt;
      }
    }
    __syncthreads();  // the tile is overwritten next
  }
  if (UPDATE) {
    // partials: sums_part[block][c][64], counts_part[block][c]
#pragma unroll
    for (int q = 0; q < SLOTS; ++q) {
      const int c = KS_WAVES * q + wave;
      if (c < KP) {
        sums_part[((int64_t)blockIdx.x * KP + c) * KS_FMAX + lane] = us[q];
        if (lane == 0) counts_part[(int64_t)blockIdx.x * KP + c] = uc[q];
      }
    }
  }
}

// sums[c][j] = sum over blocks (fp64), counts[c] likewise
template <int KP>
__global__ __launch_bounds__(256) void ks_reduce(const float* __restrict__ sums_part,
                                                 const float* __restrict__ counts_part, int nblk, int k, int f,
                                                 float* __restrict__ sums, float* __restrict__ counts) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < k * f) {
    const int c = e / f, j = e - c * f;
    double a = 0.0;
    for (int b = 0; b < nblk; ++b) a += (double)sums_part[((int64_t)b * KP + c) * KS_FMAX + j];
    sums[e] = (float)a;
  } else if (e < k * f + k) {
    const int c = e - k * f;
    double a = 0.0;
    for (int b = 0; b < nblk; ++b) a += (double)counts_part[(int64_t)b * KP + c];
    counts[c] = (float)a;
  }
}

int ks_kp(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : 16; }

}  // namespace

HA_EXPORT int ha_ks_max_k() { return 16; }
HA_EXPORT int ha_ks_max_f() { return KS_FMAX; }

// Workspace floats for ha_ks_step's per-workgroup partials (nblk = 4 workgroups per CU).
HA_EXPORT int64_t ha_ks_workspace_floats(int k, int num_cus) {
  if (k <= 0 || k > 16 || num_cus <= 0) return -1;
  return (int64_t)4 * num_cus * ks_kp(k) * (KS_FMAX + 1);
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
  const int mode = (ldx == f && f >= 4 && al) ? KS_FLAT : (f % 4 == 0 && ldx % 4 == 0 && al) ? KS_ROW4 : KS_SCALAR;
  const bool upd = sums != nullptr;
  float* sp = workspace;
  float* cp = workspace + (int64_t)nblk * kp * KS_FMAX;
  if (upd && n <= 0) {
    hipMemsetAsync(sums, 0, (size_t)k * f * sizeof(float), s);
    hipMemsetAsync(counts, 0, (size_t)k * sizeof(float), s);
    return ha_launch_status();
  }
  if (n <= 0) return HA_OK;
#define HA_KS_L(KP, M, U)                                                                                   \
  hipLaunchKernelGGL((ks_step<KP, M, U>), dim3(nblk), dim3(KS_ROWS), 0, s, X, n, f, ldx, C, k, ldc, labels, mind, sp, cp)
#define HA_KS_M(KP, M)                                                                                      \
  if (upd)                                                                                                  \
    HA_KS_L(KP, M, true);                                                                                   \
  else                                                                                                      \
    HA_KS_L(KP, M, false);
#define HA_KS_KP(KP)                                                                                        \
  if (mode == KS_FLAT) {                                                                                    \
    HA_KS_M(KP, KS_FLAT)                                                                                    \
  } else if (mode == KS_ROW4) {                                                                             \
    HA_KS_M(KP, KS_ROW4)                                                                                    \
  } else {                                                                                                  \
    HA_KS_M(KP, KS_SCALAR)                                                                                  \
  }                                                                                                         \
  if (upd)                                                                                                  \
    hipLaunchKernelGGL((ks_reduce<KP>), dim3((unsigned)((k * f + k + 255) / 256)), dim3(256), 0, s, sp, cp, nblk, \
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
