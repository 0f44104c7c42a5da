// K-means on CDNA4 (gfx950): fused assignment (distance GEMM + running argmin, the n x k distance
// matrix is never materialised) and a one-pass centroid update with LDS-privatised sums.
//
// Replaces the reference's cdist + argmin (heat/cluster/_kcluster.py:196-209) and its k-pass
// update loop with 2k all-reduces (heat/cluster/kmeans.py:73-100).
//
// Assignment = exact fp32 on the f32-input MFMA (v_mfma_f32_32x32x2_f32, bit-for-bit an fmaf
// chain, no TF32 on gfx950).  Orientation: centroids are the MFMA A (row) operand and points the B
// (column) operand, so an accumulator lane holds ONE point and 16 centroids: the running argmin
// is lane-local, and one __shfl_xor(32) merges the two half-waves at the very end.
//
// The K (feature) dimension is permuted: at k-step s the lane half h works on feature h*F2+s, so a
// lane's B fragment is F2 CONTIGUOUS floats of its point's row (16-byte loads) and the packed
// centroid image in LDS is read with conflict-free lane-linear ds_read_b128.
#include "common.h"

namespace {

template <int FPAD>
struct KMCfg {
  static constexpr int F2 = FPAD / 2;     // k-steps (each MFMA consumes 2 features)
  static constexpr int S4 = F2 / 4;       // float4 groups per lane-half row
  static constexpr int CB = FPAD >= 128 ? 64 : 128;  // centroids per LDS chunk
  static constexpr int NPB = FPAD >= 128 ? 1 : 2;    // 32-point blocks per wave
  static constexpr int CHUNK = CB * FPAD;            // floats of packed centroids per chunk
  static constexpr int PTS_PER_WG = 4 * NPB * 32;    // 4 waves per workgroup
};

// Packed centroid image: [chunk][cb][s4][lane][4] with lane = h*32 + j:
//   value = C[chunk*CB + cb*32 + j][h*F2 + 4*s4 + t]
template <int FPAD>
__global__ void km_pack_centroids(const float* __restrict__ C, int k, int f, int64_t ldc,
                                  float* __restrict__ frag, float* __restrict__ cnorm, int kpad) {
  using K = KMCfg<FPAD>;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)kpad * (FPAD / 4);
  if (tid < total) {
    const int c = (int)(tid / (FPAD / 4));
    const int q = (int)(tid % (FPAD / 4));
    const int col = 4 * q;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (c < k && col < f) v = *reinterpret_cast<const floatx4*>(C + (int64_t)c * ldc + col);
    const int h = col / K::F2, s4 = (col % K::F2) / 4;
    const int chunk = c / K::CB, cb = (c % K::CB) / 32, j = c % 32;
    const int lane = h * 32 + j;
    const int64_t dst = ((((int64_t)chunk * (K::CB / 32) + cb) * K::S4 + s4) * 64 + lane) * 4;
    *reinterpret_cast<floatx4*>(frag + dst) = v;
  }
  if (tid < kpad) {
    const int c = (int)tid;
    float s = 0.f;
    if (c < k) {
      for (int i = 0; i < f; ++i) {
        const float x = C[(int64_t)c * ldc + i];
        s = fmaf(x, x, s);
      }
      cnorm[c] = s;
    } else {
      cnorm[c] = __builtin_huge_valf();  // padded centroids are never the minimum
    }
  }
}

template <int FPAD>
__global__ __launch_bounds__(256, 2) void km_assign(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                   const float* __restrict__ frag,
                                                   const float* __restrict__ cnorm, int nchunks,
                                                   int* __restrict__ labels, float* __restrict__ mind) {
  using K = KMCfg<FPAD>;
  constexpr int F2 = K::F2, S4 = K::S4, CB = K::CB, NPB = K::NPB, CHUNK = K::CHUNK;
  constexpr int BUF = CHUNK + CB;                 // packed centroids + their norms
  constexpr int STG = CHUNK / 4 / 256;            // float4 staged per thread per chunk
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * K::PTS_PER_WG + (int64_t)wave * (NPB * 32);

  // ---- B fragments: this lane's half row of its points, kept in registers for all centroids
  float xb[NPB][F2];
  float xsq[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    int64_t row = pbase + pb * 32 + j;
    row = row < n ? row : n - 1;
    const float* xr = X + row * ldx + h * F2;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < S4; ++q) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (h * F2 + 4 * q < f) v = *reinterpret_cast<const floatx4*>(xr + 4 * q);
      xb[pb][4 * q + 0] = v[0];
      xb[pb][4 * q + 1] = v[1];
      xb[pb][4 * q + 2] = v[2];
      xb[pb][4 * q + 3] = v[3];
      s = fmaf(v[0], v[0], s);
      s = fmaf(v[1], v[1], s);
      s = fmaf(v[2], v[2], s);
      s = fmaf(v[3], v[3], s);
    }
    xsq[pb] = s;
  }

  float best[NPB];
  int bidx[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    best[pb] = __builtin_huge_valf();
    bidx[pb] = 0;
  }

  // ---- stage chunk 0
  {
    const floatx4* src = reinterpret_cast<const floatx4*>(frag);
    floatx4* dst = reinterpret_cast<floatx4*>(smem);
#pragma unroll
    for (int i = 0; i < STG; ++i) dst[tid + 256 * i] = src[tid + 256 * i];
    if (tid < CB / 4)
      reinterpret_cast<floatx4*>(smem + CHUNK)[tid] = reinterpret_cast<const floatx4*>(cnorm)[tid];
  }
  __syncthreads();

  for (int ch = 0; ch < nchunks; ++ch) {
    const bool more = ch + 1 < nchunks;
    // issue the next chunk's loads early (register staging, written after compute)
    floatx4 stg[STG];
    floatx4 stn = {0.f, 0.f, 0.f, 0.f};
    if (more) {
      const floatx4* src = reinterpret_cast<const floatx4*>(frag + (int64_t)(ch + 1) * CHUNK);
#pragma unroll
      for (int i = 0; i < STG; ++i) stg[i] = src[tid + 256 * i];
      if (tid < CB / 4) stn = reinterpret_cast<const floatx4*>(cnorm + (ch + 1) * CB)[tid];
    }
    const float* buf = smem + (ch & 1) * BUF;
#pragma unroll 1
    for (int cb = 0; cb < CB / 32; ++cb) {
      floatx16 acc[NPB];
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[pb] = (floatx16)(0.f);
#pragma unroll
      for (int s4 = 0; s4 < S4; ++s4) {
        const floatx4 a = *reinterpret_cast<const floatx4*>(buf + ((cb * S4 + s4) * 64 + lane) * 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
          for (int pb = 0; pb < NPB; ++pb)
            acc[pb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], xb[pb][4 * s4 + t], acc[pb], 0, 0, 0);
        }
      }
      // epilogue: d = |c|^2 - 2 x.c ; accumulator row = (reg&3) + 8*(reg>>2) + 4*h
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const floatx4 cn = *reinterpret_cast<const floatx4*>(buf + CHUNK + cb * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int cidx = ch * CB + cb * 32 + 8 * g + 4 * h + t;
#pragma unroll
          for (int pb = 0; pb < NPB; ++pb) {
            const float d = fmaf(-2.f, acc[pb][4 * g + t], cn[t]);
            if (d < best[pb]) {
              best[pb] = d;
              bidx[pb] = cidx;
            }
          }
        }
      }
    }
    if (more) {
      floatx4* dst = reinterpret_cast<floatx4*>(smem + ((ch + 1) & 1) * BUF);
#pragma unroll
      for (int i = 0; i < STG; ++i) dst[tid + 256 * i] = stg[i];
      if (tid < CB / 4) reinterpret_cast<floatx4*>(smem + ((ch + 1) & 1) * BUF + CHUNK)[tid] = stn;
    }
    __syncthreads();
  }

  // ---- merge the two half-waves (same point, disjoint centroid rows) and write
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const float ob = __shfl_xor(best[pb], 32, 64);
    const int oi = __shfl_xor(bidx[pb], 32, 64);
    const float xs = xsq[pb] + __shfl_xor(xsq[pb], 32, 64);
    if (ob < best[pb] || (ob == best[pb] && oi < bidx[pb])) {
      best[pb] = ob;
      bidx[pb] = oi;
    }
    const int64_t row = pbase + pb * 32 + j;
    if (h == 0 && row < n) {
      labels[row] = bidx[pb];
      if (mind) mind[row] = fmaxf(best[pb] + xs, 0.f);
    }
  }
}

// One pass over the points: per-(centroid, column) sums in LDS (ds_add_f32), counts in LDS,
// flushed once per workgroup with coalesced global float atomics (256 contiguous bytes per
// wave instruction).  Grid = (row ranges, column blocks of FC columns).  1024 threads and 8 rows
// per thread in flight keep ~64 KB of loads outstanding per CU (the kernel is HBM-bound; at one
// workgroup per CU the first version was latency-bound at ~0.8 TB/s).
constexpr int KU_THREADS = 1024;
constexpr int KU_UNROLL = 8;
template <int FC>
__global__ __launch_bounds__(KU_THREADS) void km_update(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                        const int* __restrict__ labels, int k, int64_t rows_per_wg,
                                                        float* __restrict__ sums, float* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* lsum = lds;                    // [k][FC]
  float* lcnt = lds + (int64_t)k * FC;  // [k]
  const int tid = threadIdx.x;
  for (int e = tid; e < k * FC + k; e += KU_THREADS) lds[e] = 0.f;
  __syncthreads();
  const int cblk = blockIdx.y;
  const int c0 = cblk * FC;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r1 = r0 + rows_per_wg < n ? r0 + rows_per_wg : n;
  constexpr int RP = KU_THREADS / FC;  // rows handled per pass by the block
  const int c = tid % FC, rs = tid / FC;
  const bool colok = c0 + c < f;
  const bool counter = (cblk == 0) && (c == 0);
  int64_t i = r0 + rs;
  for (; i + (KU_UNROLL - 1) * RP < r1; i += KU_UNROLL * RP) {
    int lab[KU_UNROLL];
    float v[KU_UNROLL];
#pragma unroll
    for (int u = 0; u < KU_UNROLL; ++u) {
      const int64_t r = i + u * RP;
      lab[u] = labels[r];
      v[u] = colok ? X[r * ldx + c0 + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < KU_UNROLL; ++u) {
      atomicAdd(&lsum[lab[u] * FC + c], v[u]);
      if (counter) atomicAdd(&lcnt[lab[u]], 1.f);
    }
  }
  for (; i < r1; i += RP) {
    const int lab = labels[i];
    const float v = colok ? X[i * ldx + c0 + c] : 0.f;
    atomicAdd(&lsum[lab * FC + c], v);
    if (counter) atomicAdd(&lcnt[lab], 1.f);
  }
  __syncthreads();
  for (int e = tid; e < k * FC; e += KU_THREADS) {
    const int kk = e / FC, cc = e % FC;
    const float v = lsum[e];
    if (v != 0.f && c0 + cc < f) atomicAdd(&sums[(int64_t)kk * f + c0 + cc], v);
  }
  if (cblk == 0) {
    for (int e = tid; e < k; e += KU_THREADS) {
      const float v = lcnt[e];
      if (v != 0.f) atomicAdd(&counts[e], v);
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
HA_EXPORT int ha_km_workspace_floats(int k, int f, int* fpad_out, int* kpad_out) {
  int fpad = f <= 16 ? 16 : f <= 32 ? 32 : f <= 64 ? 64 : f <= 128 ? 128 : -1;
  if (fpad < 0) return -1;
  const int cb = fpad >= 128 ? 64 : 128;
  const int kpad = (k + cb - 1) / cb * cb;
  *fpad_out = fpad;
  *kpad_out = kpad;
  return kpad * fpad + kpad;  // packed image + norms
}

HA_EXPORT int ha_km_assign(const float* X, int64_t n, int f, int64_t ldx, const float* C, int k, int64_t ldc,
                           float* workspace, int* labels, float* mind, void* stream) {
  if (n <= 0) return HA_OK;
  if (f % 4 != 0 || ldx % 4 != 0 || ldc % 4 != 0 || k <= 0) return HA_BAD_ARG;
  int fpad, kpad;
  if (ha_km_workspace_floats(k, f, &fpad, &kpad) < 0) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  float* frag = workspace;
  float* cnorm = workspace + (int64_t)kpad * fpad;
  const int64_t packthreads = (int64_t)kpad * (fpad / 4) > kpad ? (int64_t)kpad * (fpad / 4) : kpad;
  const int pblocks = (int)((packthreads + 255) / 256);
#define HA_KM_CASE(FP)                                                                                  \
  case FP: {                                                                                            \
    using KC = KMCfg<FP>;                                                                               \
    hipLaunchKernelGGL(km_pack_centroids<FP>, dim3(pblocks), dim3(256), 0, s, C, k, f, ldc, frag, cnorm, \
                       kpad);                                                                           \
    const int nchunks = kpad / KC::CB;                                                                  \
    const int64_t nwg = (n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG;                                      \
    const size_t lds = 2 * (size_t)(KC::CHUNK + KC::CB) * sizeof(float);                               \
    hipFuncSetAttribute((const void*)km_assign<FP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    hipLaunchKernelGGL(km_assign<FP>, dim3((unsigned)nwg), dim3(256), lds, s, X, n, f, ldx, frag, cnorm, \
                       nchunks, labels, mind);                                                          \
    break;                                                                                              \
  }
  switch (fpad) {
    HA_KM_CASE(16)
    HA_KM_CASE(32)
    HA_KM_CASE(64)
    HA_KM_CASE(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_KM_CASE
  return ha_launch_status();
}

// Largest power-of-two column block whose [k][FC] sums + [k] counts fit in LDS.
HA_EXPORT int ha_km_update_fc(int k, int f) {
  const int64_t budget = 160 * 1024 - 1024;
  int fc = 64;
  while (fc >= 4 && (int64_t)k * (fc + 1) * 4 > budget) fc >>= 1;
  if (fc < 4) return -1;
  while (fc > 4 && fc / 2 >= f) fc >>= 1;
  return fc;
}

// sums [k][f] and counts [k] must be zeroed by the caller (stream-ordered memset).
HA_EXPORT int ha_km_update(const float* X, int64_t n, int f, int64_t ldx, const int* labels, int k, float* sums,
                           float* counts, int num_cus, void* stream) {
  if (n <= 0) return HA_OK;
  const int fc = ha_km_update_fc(k, f);
  if (fc < 0) return HA_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int ncb = (f + fc - 1) / fc;
  const size_t lds = ((size_t)k * fc + k) * sizeof(float);
  // one resident workgroup per CU (LDS-bound); enough row ranges to cover the chip
  int64_t wgs_per_cb = (int64_t)num_cus * (lds <= 72 * 1024 ? 2 : 1) / ncb;
  if (wgs_per_cb < 1) wgs_per_cb = 1;
  int64_t rows = (n + wgs_per_cb - 1) / wgs_per_cb;
  if (rows < 512) rows = 512;
  const int64_t npt = (n + rows - 1) / rows;
  dim3 grid((unsigned)npt, (unsigned)ncb);
#define HA_KU(FC_) hipFuncSetAttribute((const void*)km_update<FC_>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
  switch (fc) { case 4: HA_KU(4); break; case 8: HA_KU(8); break; case 16: HA_KU(16); break; case 32: HA_KU(32); break; case 64: HA_KU(64); break; }
#undef HA_KU
  switch (fc) {
    case 4: hipLaunchKernelGGL(km_update<4>, grid, dim3(KU_THREADS), lds, s, X, n, f, ldx, labels, k, rows, sums, counts); break;
    case 8: hipLaunchKernelGGL(km_update<8>, grid, dim3(KU_THREADS), lds, s, X, n, f, ldx, labels, k, rows, sums, counts); break;
    case 16: hipLaunchKernelGGL(km_update<16>, grid, dim3(KU_THREADS), lds, s, X, n, f, ldx, labels, k, rows, sums, counts); break;
    case 32: hipLaunchKernelGGL(km_update<32>, grid, dim3(KU_THREADS), lds, s, X, n, f, ldx, labels, k, rows, sums, counts); break;
    case 64: hipLaunchKernelGGL(km_update<64>, grid, dim3(KU_THREADS), lds, s, X, n, f, ldx, labels, k, rows, sums, counts); break;
    default: return HA_UNSUPPORTED;
  }
  return ha_launch_status();
}
