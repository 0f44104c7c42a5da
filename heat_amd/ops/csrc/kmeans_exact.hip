// hipcc-flags: -fno-slp-vectorize
// Exact k-means assignment on CDNA4 (gfx950): distance GEMM + running argmin fused, the n x k
// distance matrix is never materialised (replaces the reference's cdist + argmin,
// heat/cluster/_kcluster.py:196-209).
//
// Exact fp32 on the f32-input MFMA (v_mfma_f32_32x32x2_f32, bit-for-bit an fmaf chain, no TF32 on
// gfx950).  Orientation: centroids are the MFMA A (row) operand and points the B (column) operand,
// so an accumulator lane holds ONE point and 16 centroids: the running argmin is lane-local, and
// one __shfl_xor(32) merges the two half-waves at the very end.
//
// The K (feature) dimension is permuted: at k-step s the lane half h works on feature h*F2+s, so a
// lane's B fragment is F2 CONTIGUOUS floats of its point's row (16-byte loads) and the packed
// centroid image in LDS is read with conflict-free lane-linear ds_read_b128.
// Built with -fno-slp-vectorize: SLP-packed f32 VALU (v_pk_fma_f32) issued beside MFMAs costs
// several times the issue slot of scalar ops on gfx950 (see kmeans_f16x3.hip).
#include "common.h"

#include <stdlib.h>

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

// Exact assignment with the structure of the fp16x3 kernel (kmeans_f16x3.hip: h3_assign_p) -
//  * the packed centroid chunks are staged by LDS-DMA (global_load_lds_dwordx4, lane-linear 1 KB
//    pieces) into two LDS buffers (no register staging);
//  * the tiles of a chunk are unrolled with ping-pong accumulators: the argmin epilogue of tile
//    t-1 is issued in the MFMA gaps of tile t (sched_group_barrier).
// Measured against round 3's register-staged, unpipelined kernel (bench.py exact path, k = 1024,
// 1.25e7 x 64): 13.37 vs 13.38 ms (122 TFLOP/s either way, ~85 % of gemm_f32t's rate): the exact
// assignment is bound by the f32 MFMA rate, not by its staging or epilogue. Kept for its lower
// register use (193 VGPRs at FPAD 64) and the shared structure with the fp16x3 kernel.
template <int FPAD>
__global__ __launch_bounds__(256, 2) void km_assign_p(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                     const float* __restrict__ frag,
                                                     const float* __restrict__ cnorm, int nchunks,
                                                     int* __restrict__ labels, float* __restrict__ mind) {
  using K = KMCfg<FPAD>;
  constexpr int F2 = K::F2, S4 = K::S4, CB = K::CB, NPB = K::NPB, CHUNK = K::CHUNK;
  constexpr int BUF = CHUNK + CB;                  // floats: packed centroids + their norms
  constexpr int PIECES = CHUNK * 4 / 1024;         // 1 KB DMA pieces per chunk
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * K::PTS_PER_WG + (int64_t)wave * (NPB * 32);

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
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        xb[pb][4 * q + t] = v[t];
        s = fmaf(v[t], v[t], s);
      }
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
  floatx16 acc[2][NPB];
  const float* pcn = nullptr;  // LDS norms of the tile whose epilogue is pending
  int pt = -1;                 // its first centroid
  auto epilogue = [&](const floatx16 (&ac)[NPB], const float* cnb, int cbase) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const floatx4 cn = *reinterpret_cast<const floatx4*>(cnb + 8 * g + 4 * h);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int cidx = cbase + 8 * g + 4 * h + t;
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) {
          const float d = fmaf(-2.f, ac[pb][4 * g + t], cn[t]);
          const bool lt = d < best[pb];
          best[pb] = lt ? d : best[pb];
          bidx[pb] = lt ? cidx : bidx[pb];
        }
      }
    }
  };
  for (int ch = 0; ch < nchunks; ++ch) {
    {
      const char* src = reinterpret_cast<const char*>(frag + (int64_t)ch * CHUNK) + lane * 16;
      unsigned char* dst = reinterpret_cast<unsigned char*>(smem + (ch & 1) * BUF);
#pragma unroll
      for (int pc = wave; pc < PIECES; pc += 4)
        __builtin_amdgcn_global_load_lds(src + pc * 1024, (__attribute__((address_space(3))) void*)(dst + pc * 1024),
                                         16, 0, 0);
      if (wave == 0 && lane < CB / 4)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(cnorm + ch * CB) + lane * 16,
                                         (__attribute__((address_space(3))) void*)(dst + CHUNK * 4), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    const float* buf = smem + (ch & 1) * BUF;
#pragma unroll
    for (int cb = 0; cb < CB / 32; ++cb) {
      const int cur = cb & 1;  // CB/32 is even: the ping-pong slot is compile-time
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
      for (int s4 = 0; s4 < S4; ++s4) {
        const floatx4 a = *reinterpret_cast<const floatx4*>(buf + ((cb * S4 + s4) * 64 + lane) * 4);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int pb = 0; pb < NPB; ++pb)
            acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], xb[pb][4 * s4 + t], acc[cur][pb], 0, 0, 0);
      }
      if (pt >= 0) epilogue(acc[cur ^ 1], pcn, pt);
#pragma unroll
      for (int i = 0; i < S4 * 4 * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // then up to 3 VALU
      }
      pt = ch * CB + cb * 32;
      pcn = buf + CHUNK + cb * 32;
    }
    __syncthreads();  // every wave is done with the buffer before the chunk after next is staged
  }
  if (pt >= 0) epilogue(acc[((CB / 32) - 1) & 1], pcn, pt);

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

}  // namespace

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
    hipFuncSetAttribute((const void*)km_assign_p<FP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    hipLaunchKernelGGL(km_assign_p<FP>, dim3((unsigned)nwg), dim3(256), lds, s, X, n, f, ldx, frag, cnorm, \
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

