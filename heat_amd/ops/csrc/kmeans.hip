// K-means on CDNA4 (gfx950): the counting-sort centroid update (one gather pass over X), replacing
// the reference's k-pass update loop with 2k all-reduces (heat/cluster/kmeans.py:73-100). The
// exact fused assignment lives in kmeans_exact.hip, the fp16x3 one in kmeans_f16x3.hip.
#include "common.h"

#include <stdlib.h>

namespace {

// ---------------------------------------------------------------------------------- update
// Centroid sums by COUNTING SORT instead of scattered float atomics.  Measured on MI355X
// (tools/microbench/ku_bench.hip): LDS float atomics (ds_add_f32) retire at ~1 lane per 3 clocks
// per CU whatever the address pattern, so an LDS-privatised update of 12.5M x 64 points took
// 3.9 ms (0.8 TB/s).  Integer LDS atomics on 4-byte labels are cheap, so:
//   1. ku_hist     per-block label histograms            (labels read once, LDS int atomics)
//   2. ku_scan_blk per-cluster exclusive prefix over blocks
//   3. ku_scan_tot exclusive prefix over clusters -> cluster start offsets, counts
//   4. ku_scatter  row ids into cluster order            (labels read again, 4-byte scatter)
//   5. ku_gather   each workgroup streams a contiguous chunk of the sorted order, gathering
//                  whole 256-byte rows of X and summing in registers; a thread flushes its
//                  running sum with one global atomic when the cluster changes (~2 per thread).
// X is read exactly once, as full rows.  Out-of-range labels are ignored.
constexpr int KU_BLOCK = 1024;     // threads of hist/scatter blocks
constexpr int KU_CHUNK = 2048;     // sorted positions per gather workgroup
constexpr int KU_RU = 8;           // rows in flight per gather thread

__global__ __launch_bounds__(KU_BLOCK) void ku_hist(const int* __restrict__ lab, int64_t n, int k,
                                                    int64_t rows_per_blk, int* __restrict__ hist,
                                                    float* __restrict__ sums, int64_t nsums) {
  extern __shared__ int h[];
  // zero the sums the gather pass accumulates into (instead of a separate memset launch)
  for (int64_t e = (int64_t)blockIdx.x * KU_BLOCK + threadIdx.x; e < nsums; e += (int64_t)gridDim.x * KU_BLOCK)
    sums[e] = 0.f;
  for (int e = threadIdx.x; e < k; e += KU_BLOCK) h[e] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = r0 + rows_per_blk < n ? r0 + rows_per_blk : n;
  for (int64_t i0 = r0 + threadIdx.x; i0 < r1; i0 += 4 * KU_BLOCK) {
    int l[4];  // 4 label loads in flight per thread
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + (int64_t)u * KU_BLOCK;
      l[u] = i < r1 ? lab[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((unsigned)l[u] < (unsigned)k) atomicAdd(&h[l[u]], 1);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < k; e += KU_BLOCK) hist[(int64_t)blockIdx.x * k + e] = h[e];
}

__global__ __launch_bounds__(256) void ku_scan_blk(int* __restrict__ hist, int nblk, int k, int* __restrict__ total) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= k) return;
  int run = 0;
  int b = 0;
  // 8 independent loads in flight per step (the dependent chain is the running sum only)
  for (; b + 8 <= nblk; b += 8) {
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = hist[(int64_t)(b + u) * k + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      hist[(int64_t)(b + u) * k + c] = run;
      run += v[u];
    }
  }
  for (; b < nblk; ++b) {
    const int v = hist[(int64_t)b * k + c];
    hist[(int64_t)b * k + c] = run;
    run += v;
  }
  total[c] = run;
}

__global__ __launch_bounds__(1024) void ku_scan_tot(const int* __restrict__ total, int k, int* __restrict__ cstart,
                                                    float* __restrict__ counts) {
  __shared__ int sh[1024];
  const int per = (k + 1023) / 1024;
  const int t = threadIdx.x;
  int loc = 0;
  for (int j = 0; j < per; ++j) {
    const int c = t * per + j;
    if (c < k) loc += total[c];
  }
  sh[t] = loc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = t >= off ? sh[t - off] : 0;
    __syncthreads();
    sh[t] += v;
    __syncthreads();
  }
  int run = sh[t] - loc;
  for (int j = 0; j < per; ++j) {
    const int c = t * per + j;
    if (c < k) {
      cstart[c] = run;
      counts[c] = (float)total[c];
      run += total[c];
    }
  }
  if (t == 1023) cstart[k] = sh[1023];
}

__global__ __launch_bounds__(KU_BLOCK) void ku_scatter(const int* __restrict__ lab, int64_t n, int k,
                                                       int64_t rows_per_blk, const int* __restrict__ hist,
                                                       const int* __restrict__ cstart, int* __restrict__ order) {
  extern __shared__ int h[];
  for (int e = threadIdx.x; e < k; e += KU_BLOCK) h[e] = cstart[e] + hist[(int64_t)blockIdx.x * k + e];
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = r0 + rows_per_blk < n ? r0 + rows_per_blk : n;
  // 4 rows per thread in flight: the label loads, then the (independent) LDS slot claims, then the
  // stores, instead of one load -> atomic -> store chain per row
  constexpr int U = 4;
  for (int64_t i0 = r0 + threadIdx.x; i0 < r1; i0 += U * KU_BLOCK) {
    int l[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * KU_BLOCK;
      l[u] = i < r1 ? lab[i] : -1;
    }
    int pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) pos[u] = (unsigned)l[u] < (unsigned)k ? atomicAdd(&h[l[u]], 1) : -1;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (pos[u] >= 0) order[pos[u]] = (int)(i0 + (int64_t)u * KU_BLOCK);
  }
}

// 256 threads = 64 columns x 4 row lanes; columns beyond 64 in further passes.
__global__ __launch_bounds__(256) void ku_gather(const float* __restrict__ X, int f, int64_t ldx,
                                                 const int* __restrict__ order, const int* __restrict__ cstart, int k,
                                                 float* __restrict__ sums) {
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t nvalid = cstart[k];
  const int64_t p0 = (int64_t)blockIdx.x * KU_CHUNK;
  const int64_t p1 = p0 + KU_CHUNK < nvalid ? p0 + KU_CHUNK : nvalid;
  const int64_t p = p0 + rl;
  if (p >= p1) return;
  int lo = 0, hi = k - 1;  // cluster of position p: last c with cstart[c] <= p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cstart[mid + 1] > p) hi = mid; else lo = mid + 1;
  }
  for (int cb = 0; cb < f; cb += 64) {
    const int col = cb + c;
    const bool ok = col < f;
    int cur = lo;
    int64_t nb = cstart[cur + 1];
    float acc = 0.f;
    int64_t q = p;
    for (; q + (KU_RU - 1) * 4 < p1; q += KU_RU * 4) {
      int idx[KU_RU];
      float v[KU_RU];
#pragma unroll
      for (int u = 0; u < KU_RU; ++u) idx[u] = order[q + u * 4];
#pragma unroll
      for (int u = 0; u < KU_RU; ++u) v[u] = ok ? X[(int64_t)idx[u] * ldx + col] : 0.f;
#pragma unroll
      for (int u = 0; u < KU_RU; ++u) {
        while (q + u * 4 >= nb) {
          if (ok) atomicAdd(&sums[(int64_t)cur * f + col], acc);
          acc = 0.f;
          ++cur;
          nb = cstart[cur + 1];
        }
        acc += v[u];
      }
    }
    for (; q < p1; q += 4) {
      const float v = ok ? X[(int64_t)order[q] * ldx + col] : 0.f;
      while (q >= nb) {
        if (ok) atomicAdd(&sums[(int64_t)cur * f + col], acc);
        acc = 0.f;
        ++cur;
        nb = cstart[cur + 1];
      }
      acc += v;
    }
    if (ok) atomicAdd(&sums[(int64_t)cur * f + col], acc);
  }
}

// 16-byte variant (f % 4 == 0, 16-byte aligned rows): 256 threads = 16 column groups of 4
// consecutive columns x 16 row lanes, so one wave-wide load covers 4 whole 256-byte rows (f = 64)
// instead of one, with KU_RU4 rows in flight per thread.
// Partial sums of the first KU_LC clusters of the workgroup's chunk are pre-reduced in LDS (one
// global atomic per (cluster, column) per workgroup): with few large clusters the 16 row lanes
// would otherwise all hit the same few addresses (k = 64: 1.17 ms without, vs 0.76 scalar).
constexpr int KU_RU4 = 8;
constexpr int KU_LC = 8;
__device__ __forceinline__ int ku_cluster_of(const int* __restrict__ cstart, int k, int64_t p) {
  int lo = 0, hi = k - 1;  // last c with cstart[c] <= p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cstart[mid + 1] > p) hi = mid; else lo = mid + 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void ku_gather4(const float* __restrict__ X, int f, int64_t ldx,
                                                  const int* __restrict__ order, const int* __restrict__ cstart,
                                                  int k, float* __restrict__ sums) {
  __shared__ float lsum[KU_LC * 64];
  const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int64_t nvalid = cstart[k];
  const int64_t p0 = (int64_t)blockIdx.x * KU_CHUNK;
  const int64_t p1 = p0 + KU_CHUNK < nvalid ? p0 + KU_CHUNK : nvalid;
  if (p0 >= p1) return;  // whole workgroup
  const int64_t p = p0 + rl;
  const int c0 = ku_cluster_of(cstart, k, p0);
  const int lo = p < p1 ? ku_cluster_of(cstart, k, p) : c0;
  for (int cb = 0; cb < f; cb += 64) {
    for (int e = threadIdx.x; e < KU_LC * 64; e += 256) lsum[e] = 0.f;
    __syncthreads();
    const int col = cb + 4 * cg;
    const bool ok = col < f;
    int cur = lo;
    int64_t nb = cstart[cur + 1];
    floatx4 acc = (floatx4)(0.f);
    auto flush = [&]() {
      if (ok) {
        const int lc = cur - c0;
        if (lc < KU_LC) {
#pragma unroll
          for (int q = 0; q < 4; ++q) atomicAdd(&lsum[lc * 64 + 4 * cg + q], acc[q]);
        } else {
          float* d = sums + (int64_t)cur * f + col;
#pragma unroll
          for (int q = 0; q < 4; ++q) atomicAdd(d + q, acc[q]);
        }
      }
      acc = (floatx4)(0.f);
    };
    int64_t q = p;
    for (; q + (KU_RU4 - 1) * 16 < p1; q += KU_RU4 * 16) {
      int idx[KU_RU4];
      floatx4 v[KU_RU4];
#pragma unroll
      for (int u = 0; u < KU_RU4; ++u) idx[u] = order[q + u * 16];
#pragma unroll
      for (int u = 0; u < KU_RU4; ++u)
        v[u] = ok ? *reinterpret_cast<const floatx4*>(X + (int64_t)idx[u] * ldx + col) : (floatx4)(0.f);
#pragma unroll
      for (int u = 0; u < KU_RU4; ++u) {
        while (q + u * 16 >= nb) {
          flush();
          ++cur;
          nb = cstart[cur + 1];
        }
        acc += v[u];
      }
    }
    for (; q < p1; q += 16) {
      const floatx4 v = ok ? *reinterpret_cast<const floatx4*>(X + (int64_t)order[q] * ldx + col) : (floatx4)(0.f);
      while (q >= nb) {
        flush();
        ++cur;
        nb = cstart[cur + 1];
      }
      acc += v;
    }
    flush();
    __syncthreads();
    for (int e = threadIdx.x; e < KU_LC * 64; e += 256) {
      const int c = c0 + e / 64, j = cb + (e & 63);
      const float v = lsum[e];
      if (c < k && j < f && v != 0.f) atomicAdd(&sums[(int64_t)c * f + j], v);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- deterministic update (default)
// The update above is fast but its float atomics (and the atomic slot claims of ku_scatter) make
// the sums depend on timing. The deterministic pipeline keeps its shape and removes every
// order-dependent step:
//   * ku_scatter_det: block b covers the same rows as its ku_hist histogram; its W waves each own a
//     contiguous sub-range (per-wave counts + a prefix over waves in LDS), and each 64-row batch is
//     placed by a bitonic sort of (label, lane) keys across the wave - positions inside a cluster
//     segment follow row order, whatever the scheduling;
//   * ku_gather_det: the sorted positions are cut into ranges of KU_RANGE; a (range, column-group)
//     thread sums its range sequentially and writes the partial of every (cluster, range) segment it
//     touches to its own slot P[cluster + range] (cluster + range is unique along the monotone
//     walk) - no atomics;
//   * ku_reduce_det: sums[c] = the cluster's range partials added in range order (fp64).
constexpr int KU_RANGE = 256;
constexpr int KU_RD = 8;  // rows in flight per gather thread
constexpr int KU_SB = 8;  // label batches loaded together per wave in ku_scatter_det

__global__ __launch_bounds__(1024) void ku_scatter_det(const int* __restrict__ lab, int64_t n, int k,
                                                       int64_t rows_per_blk, int W, const int* __restrict__ hist,
                                                       const int* __restrict__ cstart, int* __restrict__ order) {
  extern __shared__ int cnt[];  // [W][k]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = r0 + rows_per_blk < n ? r0 + rows_per_blk : n;
  const int64_t sub = (r1 - r0 + W - 1) / W;
  const int64_t s0 = r0 + w * sub < r1 ? r0 + w * sub : r1;
  const int64_t s1 = s0 + sub < r1 ? s0 + sub : r1;
  for (int e = tid; e < W * k; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // 8 label loads in flight per lane (one at a time left the pass latency-bound)
  for (int64_t i0 = s0 + lane; i0 < s1; i0 += 64 * KU_SB) {
    int l[KU_SB];
#pragma unroll
    for (int u = 0; u < KU_SB; ++u) l[u] = i0 + 64 * u < s1 ? lab[i0 + 64 * u] : -1;
#pragma unroll
    for (int u = 0; u < KU_SB; ++u)
      if ((unsigned)l[u] < (unsigned)k) atomicAdd(&cnt[w * k + l[u]], 1);  // integer counts: order-free
  }
  __syncthreads();
  for (int c = tid; c < k; c += blockDim.x) {
    int run = cstart[c] + hist[(int64_t)blockIdx.x * k + c];
    for (int v = 0; v < W; ++v) {
      const int t = cnt[v * k + c];
      cnt[v * k + c] = run;
      run += t;
    }
  }
  __syncthreads();
  int* my = cnt + w * k;
  const unsigned long long below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= lane
  for (int64_t g0 = s0; g0 < s1; g0 += 64 * KU_SB) {
  int lg[KU_SB];  // the labels of the next KU_SB batches, loaded together
#pragma unroll
  for (int u = 0; u < KU_SB; ++u) lg[u] = g0 + 64 * u + lane < s1 ? lab[g0 + 64 * u + lane] : -1;
#pragma unroll
  for (int u = 0; u < KU_SB; ++u) {
    const int64_t b0 = g0 + 64 * u;
    if (b0 >= s1) break;
    const int l = lg[u];
    int key = (unsigned)l < (unsigned)k ? (l << 6) | lane : 0x7FFFFFFF;
    // bitonic sort of the 64 keys across the wave (ascending by label, then lane)
#pragma unroll
    for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
      for (int j = kk >> 1; j > 0; j >>= 1) {
        const int other = __shfl_xor(key, j, 64);
        const bool up = (lane & kk) == 0, lower = (lane & j) == 0;
        key = (lower == up) ? min(key, other) : max(key, other);
      }
    }
    const bool valid = key != 0x7FFFFFFF;
    const int sl = key >> 6;
    const int prev = __shfl_up(key, 1, 64);
    const bool start = valid && (lane == 0 || (prev >> 6) != sl);
    const unsigned long long starts = __ballot(start);
    const int mys = 63 - __clzll(starts & below);
    const unsigned long long after = starts & ~below;
    // a run ends at the next start or at the first invalid key (invalid keys sort last); the
    // ballot runs with the whole wave active (inside the branch it would see only the starts)
    const int nvalid = __popcll(__ballot(valid));
    int base = 0;
    if (start) {
      const int end = after ? __ffsll((long long)after) - 1 : nvalid;
      base = my[sl];
      my[sl] = base + (end - lane);
    }
    const int b = __shfl(base, mys < 0 ? 0 : mys, 64);
    if (valid) order[b + (lane - mys)] = (int)(b0 + (key & 63));
  }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void ku_gather_det(const float* __restrict__ X, int f, int64_t ldx,
                                                     const int* __restrict__ order, const int* __restrict__ cstart,
                                                     int k, float* __restrict__ P) {
  const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int64_t nvalid = cstart[k];
  const int64_t rg = (int64_t)blockIdx.x * 16 + rl;
  const int64_t p0 = rg * KU_RANGE;
  if (p0 >= nvalid) return;
  const int64_t p1 = p0 + KU_RANGE < nvalid ? p0 + KU_RANGE : nvalid;
  const int c0 = ku_cluster_of(cstart, k, p0);
  for (int cb = 0; cb < f; cb += 64) {
    const int col = cb + 4 * cg;
    if (col >= f) break;
    int cur = c0;
    int64_t nb = cstart[cur + 1];
    floatx4 acc = (floatx4)(0.f);
    auto flush = [&]() {
      float* d = P + ((int64_t)cur + rg) * f + col;
      if (VEC) {
        *reinterpret_cast<floatx4*>(d) = acc;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (col + q < f) d[q] = acc[q];
      }
      acc = (floatx4)(0.f);
    };
    auto row = [&](int idx) {
      const float* src = X + (int64_t)idx * ldx + col;
      if (VEC) return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(src));  // streamed once
      floatx4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = col + q < f ? src[q] : 0.f;
      return v;
    };
    int64_t q = p0;
    for (; q + KU_RD <= p1; q += KU_RD) {
      int idx[KU_RD];
      floatx4 v[KU_RD];
#pragma unroll
      for (int u = 0; u < KU_RD; ++u) idx[u] = order[q + u];
#pragma unroll
      for (int u = 0; u < KU_RD; ++u) v[u] = row(idx[u]);
#pragma unroll
      for (int u = 0; u < KU_RD; ++u) {
        while (q + u >= nb) {
          flush();
          ++cur;
          nb = cstart[cur + 1];
        }
        acc += v[u];
      }
    }
    for (; q < p1; ++q) {
      const floatx4 v = row(order[q]);
      while (q >= nb) {
        flush();
        ++cur;
        nb = cstart[cur + 1];
      }
      acc += v;
    }
    flush();
  }
}

__global__ __launch_bounds__(256) void ku_reduce_det(const float* __restrict__ P, const int* __restrict__ cstart,
                                                     int k, int f, float* __restrict__ sums) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)k * f) return;
  const int c = (int)(e / f), j = (int)(e % f);
  const int64_t a = cstart[c], b = cstart[c + 1];
  double s = 0.0;
  if (b > a) {
    const int64_t rlo = a / KU_RANGE, rhi = (b - 1) / KU_RANGE;
    int64_t r = rlo;
    for (; r + 8 <= rhi + 1; r += 8) {  // 8 loads in flight, added in range order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = P[((int64_t)c + r + u) * f + j];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)v[u];
    }
    for (; r <= rhi; ++r) s += (double)P[((int64_t)c + r) * f + j];
  }
  sums[e] = (float)s;
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
static void ku_grid(int64_t n, int64_t* nblk, int64_t* rows_per_blk) {
  int64_t rows = 16384;  // >= 16 rows per thread amortises the LDS histogram setup
  int64_t nb = (n + rows - 1) / rows;
  if (nb > 512) {
    nb = 512;
    rows = (n + nb - 1) / nb;
  }
  if (nb < 1) nb = 1;
  *nblk = nb;
  *rows_per_blk = rows;
}

// int32 scratch ha_km_update needs (-1: unsupported k): the order array, histograms, totals and
// segment starts, plus the deterministic gather's (k + ranges) x f float partials.
HA_EXPORT int64_t ha_km_update_workspace(int64_t n, int k, int f, int num_cus) {
  (void)num_cus;
  if (k <= 0 || (int64_t)k * 4 > 150 * 1024 || n >= (int64_t)1 << 31) return -1;
  int64_t nblk, rows;
  ku_grid(n, &nblk, &rows);
  const int64_t nranges = (n + KU_RANGE - 1) / KU_RANGE;
  return n + nblk * k + k + (k + 1) + 4 + (k + nranges) * (int64_t)f;
}

static bool ku_deterministic() {
  static const bool d = [] { const char* e = getenv("HEAT_KU_DETERMINISTIC"); return !e || atoi(e) != 0; }();
  return d;
}

// sums [k][f] and counts [k] are written completely.
HA_EXPORT int ha_km_update(const float* X, int64_t n, int f, int64_t ldx, const int* labels, int k, float* sums,
                           float* counts, int* workspace, int num_cus, void* stream) {
  (void)num_cus;
  hipStream_t s = (hipStream_t)stream;
  if (ha_km_update_workspace(n, k, f, num_cus) < 0) return HA_UNSUPPORTED;
  if (n <= 0) {
    hipMemsetAsync(sums, 0, sizeof(float) * (size_t)k * f, s);
    hipMemsetAsync(counts, 0, sizeof(float) * (size_t)k, s);
    return ha_launch_status();
  }
  int64_t nblk, rows;
  ku_grid(n, &nblk, &rows);
  int* order = workspace;
  int* hist = order + n;
  int* total = hist + nblk * k;
  int* cstart = total + k;
  const size_t lds = (size_t)k * sizeof(int);
  if (lds > 64 * 1024) {
    hipFuncSetAttribute((const void*)ku_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)ku_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  hipLaunchKernelGGL(ku_hist, dim3((unsigned)nblk), dim3(KU_BLOCK), lds, s, labels, n, k, rows, hist, sums,
                     (int64_t)k * f);
  hipLaunchKernelGGL(ku_scan_blk, dim3((k + 255) / 256), dim3(256), 0, s, hist, (int)nblk, k, total);
  hipLaunchKernelGGL(ku_scan_tot, dim3(1), dim3(1024), 0, s, total, k, cstart, counts);
  if (ku_deterministic()) {
    // waves per scatter block: their per-wave counts ([W][k] ints) must fit in LDS
    int W = 16;
    while (W > 1 && (size_t)W * k * sizeof(int) > 128 * 1024) W >>= 1;
    const size_t lds_det = (size_t)W * k * sizeof(int);
    if (lds_det > 64 * 1024)
      hipFuncSetAttribute((const void*)ku_scatter_det, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_det);
    hipLaunchKernelGGL(ku_scatter_det, dim3((unsigned)nblk), dim3(64 * W), lds_det, s, labels, n, k, rows, W, hist,
                       cstart, order);
    // partials after cstart[k + 1] (16-byte aligned)
    int64_t off = (int64_t)((cstart + k + 1) - workspace);
    off = (off + 3) & ~(int64_t)3;
    float* P = reinterpret_cast<float*>(workspace + off);
    const int64_t nranges = (n + KU_RANGE - 1) / KU_RANGE;
    const unsigned gblk = (unsigned)((nranges + 15) / 16);
    if (f % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0)
      hipLaunchKernelGGL(ku_gather_det<true>, dim3(gblk), dim3(256), 0, s, X, f, ldx, order, cstart, k, P);
    else
      hipLaunchKernelGGL(ku_gather_det<false>, dim3(gblk), dim3(256), 0, s, X, f, ldx, order, cstart, k, P);
    hipLaunchKernelGGL(ku_reduce_det, dim3((unsigned)(((int64_t)k * f + 255) / 256)), dim3(256), 0, s, P, cstart, k,
                       f, sums);
    return ha_launch_status();
  }
  hipLaunchKernelGGL(ku_scatter, dim3((unsigned)nblk), dim3(KU_BLOCK), lds, s, labels, n, k, rows, hist, cstart,
                     order);
  static const bool g4 = [] { const char* e = getenv("HEAT_KU_GATHER4"); return !e || atoi(e) != 0; }();
  if (g4 && f % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0)
    hipLaunchKernelGGL(ku_gather4, dim3((unsigned)((n + KU_CHUNK - 1) / KU_CHUNK)), dim3(256), 0, s, X, f, ldx,
                       order, cstart, k, sums);
  else
    hipLaunchKernelGGL(ku_gather, dim3((unsigned)((n + KU_CHUNK - 1) / KU_CHUNK)), dim3(256), 0, s, X, f, ldx,
                       order, cstart, k, sums);
  return ha_launch_status();
}
