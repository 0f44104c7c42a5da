// Counter-based Threefry RNG, bit-exact with the reference's 8-round variant
// (heat/core/random.py:864-1062; counter layout 55-200; float conversion 220-245; Kundu normal
// transform 248-265; biased randint 556-560) - fused into ONE kernel: counter -> 8 rounds ->
// uint->float / normal / integer, instead of ~40 elementwise torch launches per call.
//
// Global element e of the flat random stream uses counter pair g = e >> 1 (component e & 1).
// 32-bit variant: V = counter + g (mod 2^64), x0 = hi32(V), x1 = lo32(V), key = seed & 0x7FFFFFFF.
// 64-bit variant: V = counter + g (mod 2^128), x0 = hi64(V), x1 = lo64(V), key = seed.
#include "common.h"

namespace {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

__device__ __forceinline__ void tf32(uint32_t& x0, uint32_t& x1, uint32_t k) {
  const uint32_t ks0 = k, ks1 = k, ks2 = 466688986u ^ k ^ k;
  x0 += ks0;
  x1 += ks1;
  x0 += x1; x1 = rotl32(x1, 13); x1 ^= x0;
  x0 += x1; x1 = rotl32(x1, 15); x1 ^= x0;
  x0 += x1; x1 = rotl32(x1, 26); x1 ^= x0;
  x0 += x1; x1 = rotl32(x1, 6); x1 ^= x0;
  x0 += ks1;
  x1 += ks2 + 1u;
  x0 += x1; x1 = rotl32(x1, 17); x1 ^= x0;
  x0 += x1; x1 = rotl32(x1, 29); x1 ^= x0;
  x0 += x1; x1 = rotl32(x1, 16); x1 ^= x0;
  x0 += x1; x1 = rotl32(x1, 24); x1 ^= x0;
  x0 += ks0;
  x1 += ks1 + 3u;
}

__device__ __forceinline__ void tf64(uint64_t& x0, uint64_t& x1, uint64_t k) {
  const uint64_t ks0 = k, ks1 = k, ks2 = 2004413935125273122ull ^ k ^ k;
  x0 += ks0;
  x1 += ks1;
  x0 += x1; x1 = rotl64(x1, 16); x1 ^= x0;
  x0 += x1; x1 = rotl64(x1, 42); x1 ^= x0;
  x0 += x1; x1 = rotl64(x1, 12); x1 ^= x0;
  x0 += x1; x1 = rotl64(x1, 31); x1 ^= x0;
  x0 += ks1;
  x1 += ks2 + 1ull;
  x0 += x1; x1 = rotl64(x1, 16); x1 ^= x0;
  x0 += x1; x1 = rotl64(x1, 32); x1 ^= x0;
  x0 += x1; x1 = rotl64(x1, 24); x1 ^= x0;
  x0 += x1; x1 = rotl64(x1, 21); x1 ^= x0;
  x0 += ks0;
  x1 += ks1 + 3ull;
}

// distribution codes
enum { DIST_UNIFORM = 0, DIST_NORMAL = 1, DIST_INT = 2 };

__device__ __forceinline__ float kundu_f(float u) {
  const float inner = 1.f - powf(u, 0.0775f);
  const float tiny = 1.17549435e-38f;
  return (logf(-logf(inner + tiny) + tiny) - 1.0821f) * (1.0f / 0.3807f);
}

// Fast single-precision Kundu transform. u^0.0775 = exp2(0.0775 log2 u) and the two logs go
// through the hardware v_log_f32 / v_exp_f32 (~1 ulp) instead of the precise powf / logf (tens of
// instructions each), which held randn at 0.75 TB/s. The transform amplifies an error of w = u^0.0775
// by 1 / (1 - w): where 1 - u < 2^-5 the value comes from a table (2^18 entries, 1 MB, L2-resident;
// u only takes the values k 2^-23) that the HOST computes with its own torch formula and uploads
// once per device (ha_threefry_set_kundu_table), so the result equals the host path exactly where
// the rounding of u^0.0775 decides it, and within a few ulp elsewhere.
constexpr int KUNDU_TAB_BITS = 18;
__device__ float g_kundu_tab[1 << KUNDU_TAB_BITS];  // [i] = kundu(u) at u = (2^23 - 1 - i) 2^-23
static bool g_tab_ready[64] = {};

__device__ __forceinline__ float kundu_fast(uint32_t v23) {
  // the table value is loaded for EVERY element (lanes outside the table read entry 0, one line
  // shared by the wave): a branch around the load put its latency on the path of ~86 % of the
  // waves (3 % of lanes need it) and held randn at 2.5 TB/s
  const uint32_t mi = 8388607u - v23;  // 2^23 (1 - u) - 1
  const bool in_tab = mi < (1u << KUNDU_TAB_BITS);
  const float tabv = g_kundu_tab[in_tab ? mi : 0u];
  // kundu(u) = (ln(-ln(1 - u^0.0775 + tiny) + tiny) - 1.0821) / 0.3807 with the constants folded
  // (VALU-bound kernel: every instruction counts):
  //   w = exp2(0.0775 log2 u)                     (u = 0: -inf -> w = 0; NOT fma(0.0775, log2 v23,
  //       -0.0775 * 23): the rounded constant shifts w by a systematic ~1e-7, which 1 / (1 - w)
  //       amplifies into a 1.7e-6 bias of the sample mean, measured)
  //   ln(l1 + tiny) = ln(ln 2) + ln 2 log2(t),   t = -log2(1 - w) + tiny / ln 2
  //   kundu = KA log2(t) + KB,   KA = ln 2 / 0.3807,   KB = (ln(ln 2) - 1.0821) / 0.3807
  // (1 - w + tiny == 1 - w outside the table range, where w < 1 - 2^-6)
  const float KA = 0.69314718056f / 0.3807f, KB = (-0.36651292058f - 1.0821f) / 0.3807f;
  const float u = (float)v23 * (1.0f / 8388608.0f);
  const float w = __builtin_amdgcn_exp2f(0.0775f * __builtin_amdgcn_logf(u));
  const float t = 1.69587987e-38f - __builtin_amdgcn_logf(1.f - w);
  const float r = fmaf(KA, __builtin_amdgcn_logf(t), KB);
  return in_tab ? tabv : r;
}

__device__ __forceinline__ double kundu_d(double u) {
  const double inner = 1.0 - pow(u, 0.0775);
  const double tiny = 2.2250738585072014e-308;
  return (log(-log(inner + tiny) + tiny) - 1.0821) * (1.0 / 0.3807);
}

template <int DIST>
__device__ __forceinline__ void tf_convert32(uint32_t v, void* out, int64_t i, int64_t low, int64_t span) {
  if constexpr (DIST == DIST_INT) {
    int32_t sv = (int32_t)v;
    int32_t a = sv < 0 ? (int32_t)(0u - (uint32_t)sv) : sv;  // torch abs (wraps at INT_MIN)
    int64_t r = (int64_t)a % span;
    if (r < 0) r += span;
    reinterpret_cast<int32_t*>(out)[i] = (int32_t)(r + low);
  } else {
    const uint32_t v23 = v & 0x7FFFFFu;
    reinterpret_cast<float*>(out)[i] = DIST == DIST_NORMAL ? kundu_fast(v23) : (float)v23 * (1.0f / 8388608.0f);
  }
}

// out: local block of n elements; global element index of out[0] is e0. One counter pair per
// thread per grid-stride step; a pair whose two elements are both in range and 8-byte aligned
// (e0 even) is written with one 8-byte store. DIST is a template parameter so each launch is one
// straight-line loop (the run-time switch kept the 64-bit modulo of the integer path in every
// iteration's code).
template <int DIST>
__global__ __launch_bounds__(256) void tf_fill32(void* __restrict__ out, int64_t e0, int64_t n, uint64_t counter_lo,
                                                 uint32_t key, int64_t low, int64_t span) {
  const int64_t p0 = e0 >> 1;
  const int64_t p1 = (e0 + n + 1) >> 1;
  const bool even = (e0 & 1) == 0;
  for (int64_t p = p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < p1;
       p += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t V = counter_lo + (uint64_t)p;
    uint32_t x0 = (uint32_t)(V >> 32), x1 = (uint32_t)V;
    tf32(x0, x1, key);
    const int64_t i = 2 * p - e0;
    if (DIST != DIST_INT && even && i >= 0 && i + 1 < n) {
      float2 o;
      const uint32_t a = x0 & 0x7FFFFFu, b = x1 & 0x7FFFFFu;
      o.x = DIST == DIST_NORMAL ? kundu_fast(a) : (float)a * (1.0f / 8388608.0f);
      o.y = DIST == DIST_NORMAL ? kundu_fast(b) : (float)b * (1.0f / 8388608.0f);
      *reinterpret_cast<float2*>(reinterpret_cast<float*>(out) + i) = o;
    } else {
      if (i >= 0 && i < n) tf_convert32<DIST>(x0, out, i, low, span);
      if (i + 1 >= 0 && i + 1 < n) tf_convert32<DIST>(x1, out, i + 1, low, span);
    }
  }
}

// Fast path of tf_fill32 for uniform / normal output when e0 is even and out is 16-byte aligned:
// each thread turns TWO consecutive counter pairs into 4 consecutive elements with one 16-byte
// store, halving the per-element loop, index and store-issue overhead (the normal transform keeps
// this kernel VALU-bound).
template <int DIST>
__global__ __launch_bounds__(256) void tf_fill32q(float* __restrict__ out, int64_t e0, int64_t n, uint64_t counter_lo,
                                                  uint32_t key) {
  const int64_t nq = (n + 3) >> 2;
  const uint64_t c0 = counter_lo + (uint64_t)(e0 >> 1);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t V0 = c0 + 2 * (uint64_t)q, V1 = V0 + 1;
    uint32_t a0 = (uint32_t)(V0 >> 32), a1 = (uint32_t)V0, b0 = (uint32_t)(V1 >> 32), b1 = (uint32_t)V1;
    tf32(a0, a1, key);
    tf32(b0, b1, key);
    const uint32_t v[4] = {a0 & 0x7FFFFFu, a1 & 0x7FFFFFu, b0 & 0x7FFFFFu, b1 & 0x7FFFFFu};
    floatx4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = DIST == DIST_NORMAL ? kundu_fast(v[c]) : (float)v[c] * (1.0f / 8388608.0f);
    const int64_t i = 4 * q;
    if (i + 3 < n) {
      *reinterpret_cast<floatx4*>(out + i) = o;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (i + c < n) out[i + c] = o[c];
    }
  }
}

__global__ __launch_bounds__(256) void tf_fill64(void* __restrict__ out, int64_t e0, int64_t n, uint64_t counter_lo,
                                                 uint64_t counter_hi, uint64_t key, int dist, int64_t low,
                                                 int64_t span) {
  const int64_t p0 = e0 >> 1;
  const int64_t p1 = (e0 + n + 1) >> 1;
  for (int64_t p = p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < p1;
       p += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = counter_lo + (uint64_t)p;
    const uint64_t hi = counter_hi + (lo < counter_lo ? 1ull : 0ull);
    uint64_t x0 = hi, x1 = lo;
    tf64(x0, x1, key);
    const uint64_t comp[2] = {x0, x1};
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t e = 2 * p + c;
      const int64_t i = e - e0;
      if (i < 0 || i >= n) continue;
      const uint64_t v = comp[c];
      if (dist == DIST_INT) {
        int64_t s = (int64_t)v;
        int64_t a = s < 0 ? (int64_t)(0ull - (uint64_t)s) : s;
        int64_t r = a % span;
        if (r < 0) r += span;
        reinterpret_cast<int64_t*>(out)[i] = r + low;
      } else {
        const double u = (double)(v & 0x1FFFFFFFFFFFFFull) * (1.0 / 9007199254740992.0);
        reinterpret_cast<double*>(out)[i] = dist == DIST_NORMAL ? kundu_d(u) : u;
      }
    }
  }
}

}  // namespace

HA_EXPORT int ha_threefry_kundu_table_size() { return 1 << KUNDU_TAB_BITS; }

// host_tab: ha_threefry_kundu_table_size() floats, [i] = kundu((2^23 - 1 - i) 2^-23), for the
// current device (synchronous copy)
HA_EXPORT int ha_threefry_set_kundu_table(const float* host_tab, int count) {
  if (!host_tab || count != (1 << KUNDU_TAB_BITS)) return HA_BAD_ARG;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return HA_LAUNCH;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_kundu_tab), host_tab, sizeof(float) * count) != hipSuccess) return HA_LAUNCH;
  g_tab_ready[dev] = true;
  return HA_OK;
}

// bits: 32 or 64. For bits == 32 only counter_lo (the counter mod 2^64) is used.
HA_EXPORT int ha_threefry_fill(void* out, int64_t e0, int64_t n, uint64_t counter_lo, uint64_t counter_hi, uint64_t seed,
                               int bits, int dist, double low, double span, void* stream) {
  if (n <= 0) return HA_OK;
  const int64_t pairs = ((e0 + n + 1) >> 1) - (e0 >> 1);
  int64_t blocks = (pairs + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipStream_t s = (hipStream_t)stream;
  if (bits == 32 && dist == DIST_NORMAL) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_tab_ready[dev]) return HA_UNSUPPORTED;
  }
  if (bits == 32) {
    const uint32_t key = (uint32_t)(seed & 0x7FFFFFFFull);
    if (dist != DIST_INT && (e0 & 1) == 0 && ((uintptr_t)out & 15) == 0) {
      int64_t qb = ((n + 3) / 4 + 255) / 256;
      if (qb > 65536) qb = 65536;
      if (dist == DIST_NORMAL)
        hipLaunchKernelGGL(tf_fill32q<DIST_NORMAL>, dim3((unsigned)qb), dim3(256), 0, s, (float*)out, e0, n, counter_lo,
                           key);
      else
        hipLaunchKernelGGL(tf_fill32q<DIST_UNIFORM>, dim3((unsigned)qb), dim3(256), 0, s, (float*)out, e0, n,
                           counter_lo, key);
    } else if (dist == DIST_NORMAL)
      hipLaunchKernelGGL(tf_fill32<DIST_NORMAL>, dim3((unsigned)blocks), dim3(256), 0, s, out, e0, n, counter_lo, key,
                         (int64_t)low, (int64_t)span);
    else if (dist == DIST_INT)
      hipLaunchKernelGGL(tf_fill32<DIST_INT>, dim3((unsigned)blocks), dim3(256), 0, s, out, e0, n, counter_lo, key,
                         (int64_t)low, (int64_t)span);
    else
      hipLaunchKernelGGL(tf_fill32<DIST_UNIFORM>, dim3((unsigned)blocks), dim3(256), 0, s, out, e0, n, counter_lo, key,
                         (int64_t)low, (int64_t)span);
  } else if (bits == 64) {
    hipLaunchKernelGGL(tf_fill64, dim3((unsigned)blocks), dim3(256), 0, s, out, e0, n, counter_lo, counter_hi, seed,
                       dist, (int64_t)low, (int64_t)span);
  } else {
    return HA_BAD_ARG;
  }
  return ha_launch_status();
}
