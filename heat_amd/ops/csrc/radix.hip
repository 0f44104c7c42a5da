// hipcc-flags: -fno-slp-vectorize
// Stable LSD radix sort of rows of 32-bit keys (float32 / int32) with their positions - the local
// phase of the distributed sample sort (core/_sample_sort.py) and ht.sort on one device
// (reference: torch.sort inside manipulations.py:2258-2509).
//
// A key is mapped to an order-preserving uint32 (floats: sign-magnitude flip, NaN canonicalised
// to the largest value, -0.0 to +0.0 so the two zeros tie as in torch.sort; descending = bitwise
// NOT), the payload is the element's flat index. Four 8-bit digit passes sort by key; a (C, n)
// batch then takes ceil(log2(C) / 8) more passes on the row number (payload / n), which - LSD
// passes being stable - leaves every row sorted by key with ties in position order. The values are
// gathered from the input by payload at the end (bit-exact, -0.0 and NaN payloads preserved).
//
// One pass = three kernels over tiles of 4096 elements (256 threads x 16 items):
//   rs_hist     per-tile 256-bin histogram in LDS -> hist[digit][tile]
//   rs_scan     one workgroup per digit: exclusive scan of its row of tile counts, row total
//   rs_scatter  per tile: a stable rank of every element (within a wave from eight ballots - lanes
//               with the same digit = AND of the per-bit ballot masks - and wave-private running
//               counters in LDS; waves own contiguous quarters of the tile, so only two block
//               barriers), the tile sorted by digit in LDS, then every digit's run written to its
//               global place (base of the digit = a 256-entry scan of the totals + the tile's
//               offset) by consecutive threads.
#include "common.h"

namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;

__device__ __forceinline__ unsigned rs_key_f32(unsigned b, int desc) {
  if ((b & 0x7F800000u) == 0x7F800000u && (b & 0x007FFFFFu)) b = 0x7FC00000u;  // NaN: one, largest
  if (b == 0x80000000u) b = 0u;                                                  // -0.0 ties +0.0
  unsigned k = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return desc ? ~k : k;
}

__global__ __launch_bounds__(RS_THREADS) void rs_init(const void* __restrict__ x, int dtype, int64_t N, int desc,
                                                      unsigned* __restrict__ keys, int* __restrict__ pay) {
  const int64_t i = (int64_t)blockIdx.x * RS_THREADS + threadIdx.x;
  if (i >= N) return;
  const unsigned b = reinterpret_cast<const unsigned*>(x)[i];
  unsigned k;
  if (dtype == 0) {
    k = rs_key_f32(b, desc);
  } else {
    k = b ^ 0x80000000u;
    if (desc) k = ~k;
  }
  keys[i] = k;
  pay[i] = (int)i;
}

__device__ __forceinline__ unsigned rs_digit(unsigned key, int pay, int shift, int mode, int rowlen) {
  return mode == 0 ? (key >> shift) & 255u : ((unsigned)(pay / rowlen) >> shift) & 255u;
}

__global__ __launch_bounds__(RS_THREADS) void rs_hist(const unsigned* __restrict__ keys, const int* __restrict__ pay,
                                                      int64_t N, int shift, int mode, int rowlen,
                                                      unsigned* __restrict__ hist, int ntiles) {
  __shared__ unsigned h[256];
  const int tid = threadIdx.x;
  h[tid] = 0u;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int i = 0; i < RS_ITEMS; ++i) {
    const int64_t idx = base + i * RS_THREADS + tid;
    if (idx < N) atomicAdd(&h[rs_digit(keys[idx], mode ? pay[idx] : 0, shift, mode, rowlen)], 1u);
  }
  __syncthreads();
  hist[(int64_t)tid * ntiles + blockIdx.x] = h[tid];
}

// exclusive scan of one 256-value block in LDS; returns this thread's exclusive prefix and the total
__device__ __forceinline__ unsigned rs_block_scan(unsigned v, unsigned* s, unsigned& total) {
  const int tid = threadIdx.x;
  s[tid] = v;
  __syncthreads();
#pragma unroll
  for (int o = 1; o < RS_THREADS; o <<= 1) {
    const unsigned add = tid >= o ? s[tid - o] : 0u;
    __syncthreads();
    s[tid] += add;
    __syncthreads();
  }
  total = s[RS_THREADS - 1];
  const unsigned excl = s[tid] - v;
  __syncthreads();
  return excl;
}

__global__ __launch_bounds__(RS_THREADS) void rs_scan(unsigned* __restrict__ hist, int ntiles,
                                                      unsigned* __restrict__ totals) {
  __shared__ unsigned s[RS_THREADS];
  unsigned* row = hist + (int64_t)blockIdx.x * ntiles;
  unsigned carry = 0u;
  for (int c0 = 0; c0 < ntiles; c0 += RS_THREADS) {
    const int i = c0 + threadIdx.x;
    const unsigned v = i < ntiles ? row[i] : 0u;
    unsigned tot;
    const unsigned ex = rs_block_scan(v, s, tot);
    if (i < ntiles) row[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

__global__ __launch_bounds__(RS_THREADS) void rs_scatter(const unsigned* __restrict__ keys, const int* __restrict__ pay,
                                                         int64_t N, int shift, int mode, int rowlen,
                                                         const unsigned* __restrict__ hist, int ntiles,
                                                         const unsigned* __restrict__ totals,
                                                         unsigned* __restrict__ okeys, int* __restrict__ opay) {
  __shared__ unsigned s[RS_THREADS];
  __shared__ unsigned gbase[256];   // global start of each digit's run of this tile
  __shared__ unsigned tdo[256];     // start of each digit's run inside the tile
  __shared__ unsigned wc[4][256];   // per-wave running counts, then per-wave offsets
  __shared__ unsigned sk[RS_TILE];  // the tile, locally sorted by digit
  __shared__ int sp[RS_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  {
    unsigned tot;
    const unsigned ex = rs_block_scan(totals[tid], s, tot);
    gbase[tid] = ex + hist[(int64_t)tid * ntiles + blockIdx.x];
#pragma unroll
    for (int w = 0; w < 4; ++w) wc[w][tid] = 0u;
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  // wave w owns the contiguous quarter [w * 1024, (w + 1) * 1024) of the tile, item by item: the
  // element order is (wave, item, lane), so ranks taken in that order are stable
  unsigned kr[RS_ITEMS], rk[RS_ITEMS];
  int pr[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const int64_t e = base + wave * (RS_ITEMS * 64) + i * 64 + lane;
    kr[i] = e < N ? keys[e] : 0u;
    pr[i] = e < N ? pay[e] : 0;
  }
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const bool valid = base + wave * (RS_ITEMS * 64) + i * 64 + lane < N;
    const unsigned d = rs_digit(kr[i], pr[i], shift, mode, rowlen);
    uint64_t match = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool on = (d >> bit) & 1u;
      const uint64_t bb = __ballot(on);
      match &= on ? bb : ~bb;
    }
    const unsigned r = __popcll(match & lt);
    rk[i] = wc[wave][d] + r;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (valid && r == 0u) wc[wave][d] += (unsigned)__popcll(match);  // one leader per digit group
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  __syncthreads();
  {
    const unsigned c0 = wc[0][tid], c1 = wc[1][tid], c2 = wc[2][tid], c3 = wc[3][tid];
    wc[0][tid] = 0u;
    wc[1][tid] = c0;
    wc[2][tid] = c0 + c1;
    wc[3][tid] = c0 + c1 + c2;
    unsigned tot;
    tdo[tid] = rs_block_scan(c0 + c1 + c2 + c3, s, tot);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    if (base + wave * (RS_ITEMS * 64) + i * 64 + lane < N) {
      const unsigned d = rs_digit(kr[i], pr[i], shift, mode, rowlen);
      const unsigned lp = tdo[d] + wc[wave][d] + rk[i];
      sk[lp] = kr[i];
      sp[lp] = pr[i];
    }
  }
  __syncthreads();
  // write the digit runs out: consecutive threads -> consecutive addresses within a run
  const int cnt = (int)(N - base < RS_TILE ? N - base : RS_TILE);
  for (int j = tid; j < cnt; j += RS_THREADS) {
    const unsigned k = sk[j];
    const int pl = sp[j];
    const unsigned d = rs_digit(k, pl, shift, mode, rowlen);
    const int64_t pos = (int64_t)gbase[d] + (j - (int)tdo[d]);
    if (pos < N) {  // always true for consistent counts; never write out of bounds
      okeys[pos] = k;
      opay[pos] = pl;
    }
  }
}

__global__ __launch_bounds__(RS_THREADS) void rs_finish(const void* __restrict__ x, const int* __restrict__ pay,
                                                        int64_t N, int rowlen, void* __restrict__ vals,
                                                        int64_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * RS_THREADS + threadIdx.x;
  if (i >= N) return;
  const int p = pay[i];
  reinterpret_cast<unsigned*>(vals)[i] = reinterpret_cast<const unsigned*>(x)[p];
  idx[i] = p % rowlen;
}

}  // namespace

// Workspace bytes for ha_radix_sort_rows over N elements.
HA_EXPORT int64_t ha_radix_workspace_bytes(int64_t N) {
  const int64_t ntiles = (N + RS_TILE - 1) / RS_TILE;
  return N * 16 + ntiles * 256 * 4 + 256 * 4 + 64;
}

// Stable sort of every row of x (rows x rowlen, contiguous; dtype 0 = float32, 1 = int32):
// vals (same dtype) and idx (int64 positions within the row). desc: descending. N < 2^31.
HA_EXPORT int ha_radix_sort_rows(const void* x, int dtype, int64_t rows, int64_t rowlen, int desc, void* vals,
                                 int64_t* idx, void* workspace, void* stream) {
  const int64_t N = rows * rowlen;
  if (N <= 0) return HA_OK;
  if (N >= (int64_t)INT32_MAX || rowlen <= 0 || (dtype != 0 && dtype != 1)) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int ntiles = (int)((N + RS_TILE - 1) / RS_TILE);
  char* w = (char*)workspace;
  unsigned* ka = (unsigned*)w;
  int* pa = (int*)(w + N * 4);
  unsigned* kb = (unsigned*)(w + N * 8);
  int* pb = (int*)(w + N * 12);
  unsigned* hist = (unsigned*)(w + N * 16);
  unsigned* totals = hist + (int64_t)ntiles * 256;
  const unsigned eblocks = (unsigned)((N + RS_THREADS - 1) / RS_THREADS);
  hipLaunchKernelGGL(rs_init, dim3(eblocks), dim3(RS_THREADS), 0, s, x, dtype, N, desc, ka, pa);
  int row_bits = 0;
  while (row_bits < 31 && ((int64_t)1 << row_bits) < rows) ++row_bits;
  const int passes = 4 + (rows > 1 ? (row_bits + 7) / 8 : 0);
  for (int ps = 0; ps < passes; ++ps) {
    const int mode = ps < 4 ? 0 : 1;
    const int shift = ps < 4 ? 8 * ps : 8 * (ps - 4);
    hipLaunchKernelGGL(rs_hist, dim3(ntiles), dim3(RS_THREADS), 0, s, ka, pa, N, shift, mode, (int)rowlen, hist,
                       ntiles);
    hipLaunchKernelGGL(rs_scan, dim3(256), dim3(RS_THREADS), 0, s, hist, ntiles, totals);
    hipLaunchKernelGGL(rs_scatter, dim3(ntiles), dim3(RS_THREADS), 0, s, ka, pa, N, shift, mode, (int)rowlen, hist,
                       ntiles, totals, kb, pb);
    unsigned* tk = ka;
    ka = kb;
    kb = tk;
    int* tp = pa;
    pa = pb;
    pb = tp;
  }
  hipLaunchKernelGGL(rs_finish, dim3(eblocks), dim3(RS_THREADS), 0, s, x, pa, N, (int)rowlen, vals, idx);
  return ha_launch_status();
}
