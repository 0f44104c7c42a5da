// Single-pass statistical moments (count, mean, M2) on CDNA4: the HBM-bound core of
// mean/var/std (reference heat/core/statistics.py:726-835 mean, 1634-1769 var).
//
// Each thread accumulates SHIFTED sums (x-K, (x-K)^2) in fp32 over its elements (K = a value of
// the same data, so the sums do not cancel), converts them to (n, mean, M2) in fp64 and the
// partial triples are merged with Chan's formula (fp64) across the wave, the workgroup and,
// outside this file, across workgroup partials and ranks.  Loads are 16-byte vectorised and
// non-temporal (the data is streamed once: MI355X_MICROARCH measures 6.5-6.8 TB/s for nt streams
// vs ~6.3 for the default policy).
#include "common.h"

#include <stdlib.h>

namespace {

struct Trip {
  double n, mean, m2;
};

__device__ __forceinline__ Trip trip_from_shifted(double n, float K, float s1, float s2) {
  Trip t;
  t.n = n;
  if (n > 0) {
    const double d1 = s1, d2 = s2;
    t.mean = (double)K + d1 / n;
    double m2 = d2 - d1 * d1 / n;
    t.m2 = m2 > 0 ? m2 : 0.0;
  } else {
    t.mean = 0.0;
    t.m2 = 0.0;
  }
  return t;
}

__device__ __forceinline__ Trip chan(const Trip& a, const Trip& b) {
  if (a.n == 0) return b;
  if (b.n == 0) return a;
  Trip r;
  r.n = a.n + b.n;
  const double d = b.mean - a.mean;
  r.mean = a.mean + d * (b.n / r.n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / r.n);
  return r;
}

__device__ __forceinline__ Trip wave_merge(Trip t) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Trip u;
    u.n = __shfl_xor(t.n, o, 64);
    u.mean = __shfl_xor(t.mean, o, 64);
    u.m2 = __shfl_xor(t.m2, o, 64);
    t = chan(t, u);
  }
  return t;
}

// Final outputs of a reduction (the fused epilogue, K6): kind 0 = the (n, mean, M2) triple in
// fp64 (input of a cross-rank merge), 1 = mean, 2 = var = M2 / (n - ddof), 3 = std, as fp32.
__device__ __forceinline__ void mom_emit(const Trip& t, int kind, double ddof, void* out, int64_t i) {
  if (kind == 0) {
    double* o = reinterpret_cast<double*>(out) + i * 3;
    o[0] = t.n;
    o[1] = t.mean;
    o[2] = t.m2;
    return;
  }
  double v = t.mean;
  if (kind >= 2) {
    v = t.m2 / (t.n - ddof);
    if (kind == 3) v = sqrt(v);
  }
  reinterpret_cast<float*>(out)[i] = (float)v;
}

// This block's partials are stored write-through (ha_store_wt) by the threads that own them; each
// of those waves drained them (s_waitcnt vmcnt(0)) before the barrier here. Lane 0 takes a ticket
// on the per-output arrival counter (agent-scope atomic, no release fence: see common.h); true in
// every thread of the block that arrived last, after ONE agent acquire, which also resets the
// counter for the next launch on this workspace.
__device__ __forceinline__ bool mom_last_arrival(unsigned* __restrict__ cnt, unsigned expected) {
  __shared__ bool last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((ha_gu32*)(cnt), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const bool l = t == expected - 1;
    if (l) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store((ha_gu32*)(cnt), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = l;
  }
  __syncthreads();
  return last;
}

__device__ __forceinline__ Trip mom_load(const double* p) { return Trip{p[0], p[1], p[2]}; }

// Chan merge of the triples p[q * stride], q in [q0, q1), in q order; 8 triples loaded per round
// (the loads are independent of the merge chain, so 8 are in flight instead of one).
__device__ __forceinline__ Trip mom_merge_strided(const double* p, int q0, int q1, int64_t stride) {
  Trip t = {0.0, 0.0, 0.0};
  int q = q0;
  for (; q + 8 <= q1; q += 8) {
    Trip v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = mom_load(p + (int64_t)(q + u) * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) t = chan(t, v[u]);
  }
  for (; q < q1; ++q) t = chan(t, mom_load(p + (int64_t)q * stride));
  return t;
}

// Chan merge of one triple per thread over a 256-thread block (wave butterflies, then the 4 wave
// results in wave order); the result is valid in thread 0. sh: 4 x 3 doubles of LDS.
__device__ __forceinline__ Trip mom_block_merge(Trip t, double (*sh)[3]) {
  t = wave_merge(t);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sh[w][0] = t.n;
    sh[w][1] = t.mean;
    sh[w][2] = t.m2;
  }
  __syncthreads();
  Trip acc = {sh[0][0], sh[0][1], sh[0][2]};
  for (int k = 1; k < 4; ++k) acc = chan(acc, Trip{sh[k][0], sh[k][1], sh[k][2]});
  return acc;
}

// rows: x[r * ld + i], i in [0, len).  Grid.x = nrows * nchunks; part[(r*nchunks + c)*3 + {0,1,2}]
__global__ __launch_bounds__(256) void mom_rows(const float* __restrict__ x, int64_t nrows, int64_t len,
                                                int64_t ld, int nchunks, int G, double* __restrict__ part,
                                                void* __restrict__ out, int kind, double ddof,
                                                unsigned* __restrict__ arrive) {
  const int64_t g = blockIdx.x;
  const int64_t r = g / nchunks;
  const int c = (int)(g % nchunks);
  const int64_t per = (len + nchunks - 1) / nchunks;
  int64_t c0 = (int64_t)c * per;
  int64_t c1 = c0 + per < len ? c0 + per : len;
  const float* row = x + r * ld;
  const int tid = threadIdx.x;
  float s1 = 0.f, s2 = 0.f;
  double cnt = 0;
  float K = c0 < c1 ? row[c0] : 0.f;
  const bool vec = ((reinterpret_cast<uintptr_t>(row) & 15) == 0);
  if (c0 < c1) {
    int64_t i0 = c0;
    if (vec) {
      // scalar head up to 16-byte alignment, then float4 body
      const int64_t a0 = (c0 + 3) & ~(int64_t)3;
      const int64_t head_end = a0 < c1 ? a0 : c1;
      for (int64_t i = c0 + tid; i < head_end; i += 256) {
        const float d = row[i] - K;
        s1 += d;
        s2 = fmaf(d, d, s2);
        cnt += 1;
      }
      i0 = head_end;
      const int64_t nv = (c1 - i0) / 4;
      const floatx4* v4 = reinterpret_cast<const floatx4*>(row + i0);
      int64_t q = tid;
      for (; q + 3 * 256 < nv; q += 4 * 256) {
        floatx4 a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = __builtin_nontemporal_load(v4 + q + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = a[u][e] - K;
            s1 += d;
            s2 = fmaf(d, d, s2);
          }
        }
        cnt += 16;
      }
      for (; q < nv; q += 256) {
        const floatx4 a = v4[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = a[e] - K;
          s1 += d;
          s2 = fmaf(d, d, s2);
        }
        cnt += 4;
      }
      i0 += nv * 4;
    }
    for (int64_t i = i0 + tid; i < c1; i += 256) {
      const float d = row[i] - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
      cnt += 1;
    }
  }
  Trip t = trip_from_shifted(cnt, K, s1, s2);
  t = wave_merge(t);
  __shared__ double sh[4][3];
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    sh[w][0] = t.n;
    sh[w][1] = t.mean;
    sh[w][2] = t.m2;
  }
  __syncthreads();
  if (tid == 0) {
    Trip acc = {sh[0][0], sh[0][1], sh[0][2]};
    for (int k = 1; k < 4; ++k) acc = chan(acc, Trip{sh[k][0], sh[k][1], sh[k][2]});
    if (out != nullptr && nchunks == 1) {
      mom_emit(acc, kind, ddof, out, r);
    } else {
      double* o = part + g * 3;
      if (out != nullptr) {  // handed to the row's last block
        ha_store_wt(o, acc.n);
        ha_store_wt(o + 1, acc.mean);
        ha_store_wt(o + 2, acc.m2);
      } else {
        o[0] = acc.n;
        o[1] = acc.mean;
        o[2] = acc.m2;
      }
    }
  }
  if (out == nullptr || nchunks == 1) return;
  // fused epilogue, a two-level tree: the last-arriving block of each group of G consecutive
  // chunks merges the group (one partial per thread, fixed lane order), the last group merges the
  // group partials. One counter for all chunks serialised ~2K same-address atomics (+40 us on a
  // 0.64 ms pass); a group's G adds spread over ~sqrt(nchunks) counters.
  const int ngroups = (nchunks + G - 1) / G, grp = c / G;
  unsigned* ctr = arrive + r * (ngroups + 1);
  const int q0 = grp * G, q1 = q0 + G < nchunks ? q0 + G : nchunks;
  if (!mom_last_arrival(ctr + grp, (unsigned)(q1 - q0))) return;
  double* gpart = part + nrows * nchunks * 3;
  Trip m = q0 + tid < q1 ? mom_load(part + (r * nchunks + q0 + tid) * 3) : Trip{0.0, 0.0, 0.0};
  m = mom_block_merge(m, sh);
  if (tid == 0) {
    double* o = gpart + (r * ngroups + grp) * 3;
    ha_store_wt(o, m.n);
    ha_store_wt(o + 1, m.mean);
    ha_store_wt(o + 2, m.m2);
  }
  if (!mom_last_arrival(ctr + ngroups, (unsigned)ngroups)) return;
  m = tid < ngroups ? mom_load(gpart + (r * ngroups + tid) * 3) : Trip{0.0, 0.0, 0.0};
  m = mom_block_merge(m, sh);
  if (tid == 0) mom_emit(m, kind, ddof, out, r);
}

// Short rows (nchunks == 1, len <= 16K): one wave per row, 4 rows per workgroup.  All lanes share
// the shift K = row[0], so the shifted sums are plain wave sums (no per-lane Chan merges, which
// made the block-per-row kernel ~4x slower than HBM on 1e6 x 1000 inputs).
__global__ __launch_bounds__(256) void mom_rows_wave(const float* __restrict__ x, int64_t nrows, int64_t len,
                                                     int64_t ld, double* __restrict__ part, void* __restrict__ out,
                                                     int kind, double ddof) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const float* row = x + r * ld;
  const float K = row[0];
  float s1 = 0.f, s2 = 0.f;
  // scalar head up to 16-byte alignment
  int64_t a0 = (int64_t)((4 - ((reinterpret_cast<uintptr_t>(row) >> 2) & 3)) & 3);
  if (a0 > len) a0 = len;
  if (lane < a0) {
    const float d = row[lane] - K;
    s1 += d;
    s2 = fmaf(d, d, s2);
  }
  const int64_t nv = (len - a0) / 4;
  const floatx4* v4 = reinterpret_cast<const floatx4*>(row + a0);
  int64_t q = lane;
  for (; q + 3 * 64 < nv; q += 4 * 64) {
    floatx4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = __builtin_nontemporal_load(v4 + q + u * 64);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = a[u][e] - K;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
  }
  for (; q < nv; q += 64) {
    const floatx4 a = v4[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = a[e] - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
  }
  for (int64_t i = a0 + nv * 4 + lane; i < len; i += 64) {
    const float d = row[i] - K;
    s1 += d;
    s2 = fmaf(d, d, s2);
  }
  s1 = ha_wave_sum(s1);
  s2 = ha_wave_sum(s2);
  if (lane == 0) {
    const Trip t = trip_from_shifted((double)len, K, s1, s2);
    if (out != nullptr) {
      mom_emit(t, kind, ddof, out, r);
    } else {
      part[r * 3 + 0] = t.n;
      part[r * 3 + 1] = t.mean;
      part[r * 3 + 2] = t.m2;
    }
  }
}

// Short aligned rows (4 <= len <= 1024, 16-byte aligned rows): a grid of a few workgroups per CU,
// each wave walking rows r, r + nwaves, ... with the NEXT row's loads (<= 4 x 16 B per lane) issued
// before the current row is reduced - one launch-free pipeline instead of a workgroup per 4 rows
// (1e6 x 1000 axis 1: the per-row kernel left HBM at 5.6 TB/s, dispatch-bound on 250K workgroups).
__device__ __forceinline__ void mom_row_loads(const float* row, int nv, int lane, floatx4 (&a)[4]) {
  const floatx4* v4 = reinterpret_cast<const floatx4*>(row);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = lane + 64 * u;
    a[u] = q < nv ? __builtin_nontemporal_load(v4 + q) : (floatx4)(0.f);
  }
}

__global__ __launch_bounds__(256) void mom_rows_pipe(const float* __restrict__ x, int64_t nrows, int64_t len,
                                                     int64_t ld, double* __restrict__ part, void* __restrict__ out,
                                                     int kind, double ddof) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nv = (int)(len / 4), rem = (int)(len - 4 * (int64_t)nv);
  floatx4 cur[4], nxt[4];
  float tcur = 0.f, tnxt = 0.f;  // the scalar tail element of this lane (lane < rem)
  if (r < nrows) {
    mom_row_loads(x + r * ld, nv, lane, cur);
    if (lane < rem) tcur = x[r * ld + 4 * nv + lane];
  }
  for (; r < nrows; r += nw) {
    const int64_t rn = r + nw;
    if (rn < nrows) {
      mom_row_loads(x + rn * ld, nv, lane, nxt);
      if (lane < rem) tnxt = x[rn * ld + 4 * nv + lane];
    }
    // the row is in registers: shift by its fp32 mean (one extra wave sum, no memory traffic) -
    // a shift by row[0] lost ~10x in M2 when row[0] sat far in a tail (var of 5e4 rows of
    // N(100, 9): 3e-6 relative)
    float sm = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (lane + 64 * u < nv) sm += (cur[u][0] + cur[u][1]) + (cur[u][2] + cur[u][3]);
    if (lane < rem) sm += tcur;
    const float K = ha_wave_sum(sm) / (float)len;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (lane + 64 * u < nv) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = cur[u][e] - K;
          s1 += d;
          s2 = fmaf(d, d, s2);
        }
      }
    }
    if (lane < rem) {
      const float d = tcur - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
    s1 = ha_wave_sum(s1);
    s2 = ha_wave_sum(s2);
    if (lane == 0) {
      const Trip t = trip_from_shifted((double)len, K, s1, s2);
      if (out != nullptr) {
        mom_emit(t, kind, ddof, out, r);
      } else {
        part[r * 3 + 0] = t.n;
        part[r * 3 + 1] = t.mean;
        part[r * 3 + 2] = t.m2;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
    tcur = tnxt;
  }
}

// columns: x[i * ld + col], reduce over i in [0, len).  Each thread owns VEC consecutive
// columns; grid = (ceil(ncols / (256*VEC)), nchunks).  part[(c*ncols + col)*3 + {0,1,2}]
template <int VEC>
__global__ __launch_bounds__(256) void mom_cols(const float* __restrict__ x, int64_t len, int64_t ncols,
                                                int64_t ld, int nchunks, int G, double* __restrict__ part,
                                                void* __restrict__ out, int kind, double ddof,
                                                unsigned* __restrict__ cnt) {
  const int64_t col0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
  const int c = blockIdx.y;
  const int64_t per = (len + nchunks - 1) / nchunks;
  const int64_t r0 = (int64_t)c * per;
  const int64_t r1 = r0 + per < len ? r0 + per : len;
  if (col0 < ncols) {
  float K[VEC], s1[VEC], s2[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    s1[e] = 0.f;
    s2[e] = 0.f;
    K[e] = 0.f;
  }
  if (r0 < r1) {
    if (VEC == 4) {
      const floatx4 k4 = *reinterpret_cast<const floatx4*>(x + r0 * ld + col0);
#pragma unroll
      for (int e = 0; e < VEC; ++e) K[e] = k4[e];
    } else {
      K[0] = x[r0 * ld + col0];
    }
  }
  int64_t i = r0;
  // 16 rows (256 B per thread) in flight: ~128 KB per CU at 2 workgroups per CU (8 rows left the
  // few-chunk grid short of bytes in flight; more chunks instead cost partials and merge depth)
  if (VEC == 4) {
    for (; i + 15 < r1; i += 16) {
      floatx4 a[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) a[u] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(x + (i + u) * ld + col0));
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = a[u][e] - K[e];
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
    }
  }
  for (; i + 3 < r1; i += 4) {
    if (VEC == 4) {
      floatx4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(x + (i + u) * ld + col0));
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = a[u][e] - K[e];
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
    } else {
      float a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = x[(i + u) * ld + col0];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float d = a[u] - K[0];
        s1[0] += d;
        s2[0] = fmaf(d, d, s2[0]);
      }
    }
  }
  for (; i < r1; ++i) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float d = x[i * ld + col0 + e] - K[e];
      s1[e] += d;
      s2[e] = fmaf(d, d, s2[e]);
    }
  }
  const double n = (double)(r1 > r0 ? r1 - r0 : 0);
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int64_t col = col0 + e;
    if (col < ncols) {
      const Trip t = trip_from_shifted(n, K[e], s1[e], s2[e]);
      if (out != nullptr && nchunks == 1) {
        mom_emit(t, kind, ddof, out, col);
      } else {
        double* o = part + ((int64_t)c * ncols + col) * 3;
        if (out != nullptr) {  // handed to the group's last block
          ha_store_wt(o, t.n);
          ha_store_wt(o + 1, t.mean);
          ha_store_wt(o + 2, t.m2);
        } else {
          o[0] = t.n;
          o[1] = t.mean;
          o[2] = t.m2;
        }
      }
    }
  }
  }
  if (out == nullptr || nchunks == 1) return;
  // fused epilogue as a two-level tree (a serial merge of ~2K partials per column in ONE block
  // was latency-bound: 1e6 x 1000 axis 0 took 2x the HBM time): the last-arriving block of each
  // group of G consecutive chunks merges the group's partials (chunk order) into gpart, the last
  // group merges the group partials (group order) - deterministic whatever the arrival order.
  const int ngroups = (nchunks + G - 1) / G, grp = c / G;
  unsigned* ctr = cnt + (int64_t)blockIdx.x * (ngroups + 1);
  const int q0 = grp * G, q1 = q0 + G < nchunks ? q0 + G : nchunks;
  if (!mom_last_arrival(ctr + grp, (unsigned)(q1 - q0))) return;
  double* gpart = part + (int64_t)nchunks * ncols * 3;
  if (col0 < ncols) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int64_t col = col0 + e;
      if (col < ncols) {
        const Trip t = mom_merge_strided(part + col * 3, q0, q1, ncols * 3);
        double* o = gpart + ((int64_t)grp * ncols + col) * 3;
        ha_store_wt(o, t.n);
        ha_store_wt(o + 1, t.mean);
        ha_store_wt(o + 2, t.m2);
      }
    }
  }
  if (!mom_last_arrival(ctr + ngroups, (unsigned)ngroups)) return;
  if (col0 >= ncols) return;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int64_t col = col0 + e;
    if (col < ncols) mom_emit(mom_merge_strided(gpart + col * 3, 0, ngroups, ncols * 3), kind, ddof, out, col);
  }
}

}  // namespace

// Chunks per merge group of the fused epilogues (ceil(sqrt(nchunks)): both tree levels short).
static int mom_group(int nchunks) {
  int g = 1;
  while (g * g < nchunks) ++g;
  return g;
}

// Workspace of ha_moments_rows' fused epilogue (nchunks > 1): doubles of part, zeroed counters.
HA_EXPORT void ha_moments_rows_workspace(int64_t nrows, int nchunks, int64_t* part_doubles, int64_t* counters) {
  const int g = mom_group(nchunks > 0 ? nchunks : 1);
  const int64_t ngroups = (nchunks + g - 1) / g;
  *part_doubles = nrows * (nchunks + (nchunks > 1 ? ngroups : 0)) * 3;
  *counters = nchunks > 1 ? nrows * (ngroups + 1) : 0;
}

// (n, mean, M2) of each row x[r * ld + i], i < len. out == null: per-chunk partial triples into
// part[(r nchunks + c) 3 + {0, 1, 2}]; else the final value per row (kind: 0 triple fp64, 1 mean,
// 2 var, 3 std as fp32) into out - chunks merged by a two-level tree of last-arriving blocks
// (part / cnt sized by ha_moments_rows_workspace; the counters zeroed, reset by the kernel).
HA_EXPORT int ha_moments_rows(const float* x, int64_t nrows, int64_t len, int64_t ld, int nchunks, double* part,
                              void* out, int kind, double ddof, unsigned* cnt, void* stream) {
  if (nrows <= 0) return HA_OK;
  if (nchunks < 1 || nchunks > 65536 || (out != nullptr && nchunks > 1 && cnt == nullptr)) return HA_BAD_ARG;
  static const bool pipe = [] { const char* e = getenv("HEAT_MOM_ROWS_PIPE"); return !e || atoi(e) != 0; }();
  if (pipe && nchunks == 1 && len >= 4 && len <= 1024 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t want = (int64_t)ncu * 8, need = (nrows + 3) / 4;
    const int64_t blocks = want < need ? want : need;
    hipLaunchKernelGGL(mom_rows_pipe, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, nrows, len, ld,
                       part, out, kind, ddof);
    return ha_launch_status();
  }
  if (nchunks == 1 && len > 0 && len <= 16384) {
    const int64_t blocks = (nrows + 3) / 4;
    if (blocks > 0x7fffffffLL) return HA_UNSUPPORTED;
    hipLaunchKernelGGL(mom_rows_wave, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, nrows, len, ld,
                       part, out, kind, ddof);
    return ha_launch_status();
  }
  const int64_t grid = nrows * nchunks;
  if (grid > 0x7fffffffLL) return HA_UNSUPPORTED;
  hipLaunchKernelGGL(mom_rows, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, x, nrows, len, ld, nchunks,
                     mom_group(nchunks),
                     part, out, kind, ddof, cnt);
  return ha_launch_status();
}

// (n, mean, M2) of each column x[i * ld + col], i < len; out / kind as ha_moments_rows. With out
// and nchunks > 1, part needs (nchunks + ceil(nchunks / G)) * ncols * 3 doubles and cnt
// ceil(ncols / 256) * (ceil(nchunks / G) + 1) zeroed counters (ha_moments_cols_counters), G as
// mom_group.
HA_EXPORT int ha_moments_cols(const float* x, int64_t len, int64_t ncols, int64_t ld, int nchunks, double* part,
                              void* out, int kind, double ddof, unsigned* cnt, void* stream) {
  if (ncols <= 0) return HA_OK;
  if (nchunks < 1 || nchunks > 65535 || (out != nullptr && nchunks > 1 && cnt == nullptr)) return HA_BAD_ARG;
  const bool vec = (ncols % 4 == 0) && (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  if (vec) {
    const int64_t gx = (ncols / 4 + 255) / 256;
    hipLaunchKernelGGL(mom_cols<4>, dim3((unsigned)gx, nchunks), dim3(256), 0, (hipStream_t)stream, x, len, ncols,
                       ld, nchunks, mom_group(nchunks), part, out, kind, ddof, cnt);
  } else {
    const int64_t gx = (ncols + 255) / 256;
    hipLaunchKernelGGL(mom_cols<1>, dim3((unsigned)gx, nchunks), dim3(256), 0, (hipStream_t)stream, x, len, ncols,
                       ld, nchunks, mom_group(nchunks), part, out, kind, ddof, cnt);
  }
  return ha_launch_status();
}

// Workspace of ha_moments_cols' fused epilogue: doubles of part (first) and counters (second).
HA_EXPORT void ha_moments_cols_workspace(int64_t ncols, int nchunks, int64_t* part_doubles, int64_t* counters) {
  const int g = mom_group(nchunks > 0 ? nchunks : 1);
  const int64_t ngroups = (nchunks + g - 1) / g;
  *part_doubles = (nchunks + (nchunks > 1 ? ngroups : 0)) * ncols * 3;
  *counters = ((ncols + 255) / 256) * (ngroups + 1);
}
