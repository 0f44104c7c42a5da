// Exact rescoring of kNN candidate lists (reference hot loop
// heat/classification/kneighborsclassifier.py:117-136 - distances + topk): for every query q and
// its candidate rows idx[q][0 .. c) of T (-1 = none), the exact difference-form squared distance
// sum_j (Q[q][j] - T[i][j])^2 in fp32 (one sequential fused chain over the features, the same for
// every run), then the k smallest in (distance, index) order.
//
// The certified one-term kNN pass (kmeans_f16x3.hip: h1_topk) hands over 16 or 32 candidates per
// query; rescoring them with torch (gather the rows, broadcast subtract, square, sum, lexicographic
// top-k) made four passes over a [nq, c, f] intermediate (~25 ms at 1e6 x 16 x 128). Here it is one
// pass: a group of 32 lanes per query, lane l owns candidate l (its row read with 16-byte loads, the
// query row broadcast), and a 32-lane bitonic sort of the packed (distance bits, index) key orders
// the candidates; lanes s < k write result s.
#include "common.h"

namespace {

constexpr int RS_GROUP = 32;  // lanes per query (candidates per query <= 32)

template <bool VEC, typename IDX>
__global__ __launch_bounds__(256) void knn_rescore(const float* __restrict__ Q, int64_t ldq,
                                                   const float* __restrict__ T, int64_t ldt, int64_t nt,
                                                   int64_t nq, int f, const IDX* __restrict__ cand, int c, int k,
                                                   float* __restrict__ dist, int64_t* __restrict__ out_idx) {
  const int lane = threadIdx.x & 63;
  const int l = lane & (RS_GROUP - 1);
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / RS_GROUP;
  if (q >= nq) return;  // the whole 32-lane group leaves together (q is uniform in the group)
  int64_t i = l < c ? (int64_t)cand[q * c + l] : -1;
  if (i >= nt) i = -1;  // defensive: an out-of-range candidate is "none", never read
  float d = __builtin_huge_valf();
  if (i >= 0) {
    const float* qr = Q + q * ldq;
    const float* tr = T + i * ldt;
    float acc = 0.f;
    int j = 0;
    if constexpr (VEC) {
      for (; j + 4 <= f; j += 4) {
        const floatx4 a = *reinterpret_cast<const floatx4*>(qr + j);
        const floatx4 b = *reinterpret_cast<const floatx4*>(tr + j);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float e = a[u] - b[u];
          acc = fmaf(e, e, acc);
        }
      }
    }
    for (; j < f; ++j) {
      const float e = qr[j] - tr[j];
      acc = fmaf(e, e, acc);
    }
    d = acc;
  }
  // (distance, index) key: d >= 0 (or +inf / NaN), so its bits order like the value; "none" (-1)
  // sorts after every real candidate of equal distance
  uint64_t key = ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)(i >= 0 ? (uint32_t)i : 0xFFFFFFFFu);
#pragma unroll
  for (int size = 2; size <= RS_GROUP; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t other = (uint64_t)__shfl_xor((unsigned long long)key, stride, 64);
      const bool ascending = (l & size) == 0 || size == RS_GROUP;
      const bool lower = (l & stride) == 0;
      const uint64_t lo = key < other ? key : other, hi = key < other ? other : key;
      key = (lower == ascending) ? lo : hi;
    }
  }
  if (l < k) {
    const uint32_t ib = (uint32_t)key;
    const bool ok = ib != 0xFFFFFFFFu;
    dist[q * k + l] = ok ? __uint_as_float((uint32_t)(key >> 32)) : __builtin_huge_valf();
    out_idx[q * k + l] = ok ? (int64_t)ib : -1;
  }
}

}  // namespace

// dist [nq, k] fp32 / out_idx [nq, k] int64: the k <= c <= 32 nearest of each query's candidate
// rows cand [nq, c] (int32 when idx64 == 0, else int64; -1 = none) by exact fp32 difference-form
// squared distance, equal distances by index. Q [nq, f] (ldq), T [nt, f] (ldt) fp32 row-major.
HA_EXPORT int ha_knn_rescore(const float* Q, int64_t ldq, const float* T, int64_t ldt, int64_t nt, int64_t nq, int f,
                             const void* cand, int idx64, int c, int k, float* dist, int64_t* out_idx, void* stream) {
  if (nq < 0 || nt < 0 || f <= 0 || c < 1 || c > RS_GROUP || k < 1 || k > c || ldq < f || ldt < f) return HA_BAD_ARG;
  if (nt >= (int64_t)0xFFFFFFFF) return HA_UNSUPPORTED;  // indices travel in the key's low 32 bits
  if (nq == 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = f % 4 == 0 && ldq % 4 == 0 && ldt % 4 == 0 && (((uintptr_t)Q | (uintptr_t)T) & 15) == 0;
  const int64_t threads = nq * RS_GROUP;
  const dim3 grid((unsigned)((threads + 255) / 256));
#define HA_RS(V, I)                                                                                          \
  hipLaunchKernelGGL((knn_rescore<V, I>), grid, dim3(256), 0, s, Q, ldq, T, ldt, nt, nq, f, (const I*)cand, c, k, \
                     dist, out_idx)
  if (vec) {
    if (idx64) HA_RS(true, int64_t);
    else HA_RS(true, int);
  } else {
    if (idx64) HA_RS(false, int64_t);
    else HA_RS(false, int);
  }
#undef HA_RS
  return ha_launch_status();
}
