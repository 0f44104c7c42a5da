// Pairwise L2-family distances by quadratic expansion on the FP16 matrix cores with a 3-term
// split (the reference's quadratic_expansion=True path, heat/spatial/distance.py:46-63, 86-102).
//
// Each operand is packed once per call into fp16 hi/lo planes of its rows scaled by a power of two
// s (max |x_i| in [0.5, 1)), plus the exact fp32 squared norm and 1/s (cdist_pack).  Then
//     x.y = (hi_x.hi_y + hi_x.lo_y + lo_x.hi_y) / (s_x s_y)        (three MFMAs, fp32 accumulate)
// with ~fp32-GEMM accuracy, at 16x the per-instruction rate of the f32-input MFMA, and
//     d2 = max(|x|^2 + |y|^2 - 2 x.y, 0)  -> sqrt | identity | exp(-scale d2).
//
// Output tile 128 x 128 per 256-thread workgroup (4 waves x 64 x 64 = 2 x 2 blocks of
// v_mfma_f32_32x32x16_f16).  Features advance in chunks of 32 (2 k-steps); both operand chunks are
// staged through LDS in fragment order (lane-linear conflict-free ds_read_b128); the next chunk's
// global loads are in flight (in registers) during the MFMAs, 3 workgroups per CU.  Workgroups are mapped so that
// the ones resident on one XCD sweep a contiguous band of tile rows (shared X panels in that
// XCD's L2).  The distance matrix is written with non-temporal stores (it is streamed, never
// re-read by this kernel).
#include "common.h"

namespace {

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

constexpr int TM = 128, TN = 128, KC = 32;
constexpr int IMG_H = 4 * 2 * 2 * 64 * 8;  // halfs per operand chunk image: [rb][s][hl][lane][8]

// one wave per row: planes[row][0:fpad] = hi, [fpad:2 fpad] = lo, aux[row] = {|x|^2, 1/s}
__global__ __launch_bounds__(256) void cdist_pack(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                  int fpad, _Float16* __restrict__ planes,
                                                  float2* __restrict__ aux) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = X + row * ldx;
  float mx = 0.f, ss = 0.f;
  for (int c = lane; c < f; c += 64) {
    const float v = xr[c];
    mx = fmaxf(mx, fabsf(v));
    ss = fmaf(v, v, ss);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    ss += __shfl_xor(ss, o, 64);
  }
  int e = 0;
  if (mx > 0.f && mx < __builtin_huge_valf()) frexpf(mx, &e);
  const float s = ldexpf(1.f, -e);
  _Float16* pr = planes + row * (2 * (int64_t)fpad);
  for (int g = lane; g < fpad / 8; g += 64) {
    halfx8 hi, lo;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = g * 8 + i;
      const float v = c < f ? xr[c] * s : 0.f;
      const _Float16 hv = (_Float16)v;
      hi[i] = hv;
      lo[i] = (_Float16)(v - (float)hv);
    }
    *reinterpret_cast<halfx8*>(pr + g * 8) = hi;
    *reinterpret_cast<halfx8*>(pr + fpad + g * 8) = lo;
  }
  if (lane == 0) aux[row] = make_float2(ss, 1.f / s);
}

// piece q (0..1023) of a 128-row x 32-feature x {hi,lo} chunk: source row-major, LDS fragment order
__device__ __forceinline__ void piece_addr(int q, int& r, int& src_off, int& dst_off, int fpad) {
  r = q >> 3;
  const int g = q & 7;
  const int hl = g >> 2, gg = g & 3;
  const int h = gg >> 1, s = gg & 1;
  src_off = hl * fpad + 8 * gg;  // + chunk*32, within the row
  const int rb = r >> 5, j = r & 31;
  dst_off = ((((rb * 2 + s) * 2 + hl) * 64) + h * 32 + j) * 8;
}

template <int MODE>
__device__ __forceinline__ float epi(float d2, float scale) {
  if (MODE == 0) return __builtin_amdgcn_sqrtf(d2);  // v_sqrt_f32 (1 ulp), no denormal rescaling
  if (MODE == 1) return d2;
  return __expf(-d2 * scale);
}

// ABL (timing ablations in tools/microbench only): 1 = no stores, 2 = no MFMAs
template <int MODE, int ABL = 0>
__global__ __launch_bounds__(256, 3) void cdist_h3(const _Float16* __restrict__ PX, const float2* __restrict__ AX,
                                                  int64_t m, const _Float16* __restrict__ PY,
                                                  const float2* __restrict__ AY, int64_t n, int fpad,
                                                  float* __restrict__ C, int64_t ldc, float scale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  _Float16* img = reinterpret_cast<_Float16*>(smem);          // [op][IMG_H]
  float* rowv = reinterpret_cast<float*>(smem + 2 * IMG_H * 2);  // xn[128], isx[128], yn[128], isy[128]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;

  // XCD-aware tile order: workgroup b runs on XCD b % 8; give each XCD a contiguous band of tiles
  const int64_t tiles_n = (n + TN - 1) / TN;
  const int64_t tiles = ((m + TM - 1) / TM) * tiles_n;
  const int64_t per_xcd = (tiles + 7) / 8;
  const int64_t b = blockIdx.x;
  const int64_t t = (b % 8) * per_xcd + b / 8;  // a bijection of [0, 8 per_xcd)
  if (t >= tiles) return;                          // padding of the last band
  // grouped order inside the band: GROUP tile-rows advance together, so the ~64 workgroups
  // resident on one XCD cover an 8 x 8 block of tiles and share 8 X and 8 Y panels in its L2
  // (row-major order would need 1 X and 64 distinct Y panels)
  constexpr int64_t GROUP = 8;
  const int64_t tiles_m = (m + TM - 1) / TM;
  const int64_t grp = t / (GROUP * tiles_n);
  const int64_t first = grp * GROUP;
  const int64_t gsz = tiles_m - first < GROUP ? tiles_m - first : GROUP;
  const int64_t in = t - grp * GROUP * tiles_n;
  const int64_t row0 = (first + in % gsz) * TM, col0 = (in / gsz) * TN;

  if (tid < 128) {
    const int64_t r = row0 + tid;
    const float2 a = r < m ? AX[r] : make_float2(0.f, 0.f);
    rowv[tid] = a.x;
    rowv[128 + tid] = a.y;
  } else {
    const int64_t c = col0 + tid - 128;
    const float2 a = c < n ? AY[c] : make_float2(0.f, 0.f);
    rowv[256 + tid - 128] = a.x;
    rowv[384 + tid - 128] = a.y;
  }

  const int nch = fpad / KC;
  halfx8 stg[8];
  int dsto[8];
  // issue the global loads of chunk `ch` into registers
  auto load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int op = i >> 2;
      const int q = tid + 256 * (i & 3);
      int r, so, dso;
      piece_addr(q, r, so, dso, fpad);
      dsto[i] = op * IMG_H + dso;
      const int64_t gr = (op == 0 ? row0 : col0) + r;
      const int64_t lim = op == 0 ? m : n;
      const _Float16* P = op == 0 ? PX : PY;
      halfx8 v = (halfx8)((_Float16)0.f);
      if (gr < lim) v = *reinterpret_cast<const halfx8*>(P + gr * (2 * (int64_t)fpad) + ch * KC + so);
      stg[i] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<halfx8*>(img + dsto[i]) = stg[i];
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = (floatx16)(0.f);
  const int wr = wave >> 1, wc = wave & 1;

  // one LDS buffer (3 workgroups per CU fit): the next chunk waits in registers during the MFMAs
  load(0);
  store();
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const _Float16* ix = img;
    const _Float16* iy = ix + IMG_H;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      halfx8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int rb = 2 * wr + u;
        ah[u] = *reinterpret_cast<const halfx8*>(ix + (((rb * 2 + s) * 2 + 0) * 64 + lane) * 8);
        al[u] = *reinterpret_cast<const halfx8*>(ix + (((rb * 2 + s) * 2 + 1) * 64 + lane) * 8);
        const int cb = 2 * wc + u;
        bh[u] = *reinterpret_cast<const halfx8*>(iy + (((cb * 2 + s) * 2 + 0) * 64 + lane) * 8);
        bl[u] = *reinterpret_cast<const halfx8*>(iy + (((cb * 2 + s) * 2 + 1) * 64 + lane) * 8);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          if (ABL == 2) {
            acc[u][v][0] += (float)ah[u][0] * (float)bh[v][0];
            continue;
          }
          acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[u], bh[v], acc[u][v], 0, 0, 0);
          acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[u], bl[v], acc[u][v], 0, 0, 0);
          acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[u], bh[v], acc[u][v], 0, 0, 0);
        }
    }
    if (ch + 1 < nch) {
      __syncthreads();
      store();
      __syncthreads();
    }
  }

  // epilogue: lane holds column j of each 32x32 block, rows (r&3) + 8(r>>2) + 4h
  const bool interior = row0 + TM <= m && col0 + TN <= n;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int cl = (2 * wc + v) * 32 + j;
    const int64_t col = col0 + cl;
    const float ynv = rowv[256 + cl], m2isy = -2.f * rowv[384 + cl];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rbase = (2 * wr + u) * 32 + 4 * h;
      float* cp = C + (row0 + rbase) * ldc + col;
      float o[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = rbase + (r & 3) + 8 * (r >> 2);
        const float d2 = fmaxf(fmaf(m2isy * rowv[128 + rl], acc[u][v][r], rowv[rl] + ynv), 0.f);
        o[r] = epi<MODE>(d2, scale);
      }
      if (ABL == 1) {
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) t += o[r];
        if (t == 1234.5f) cp[0] = t;  // keep the epilogue alive
      } else if (interior) {
#pragma unroll
        for (int r = 0; r < 16; ++r) __builtin_nontemporal_store(o[r], cp + ((r & 3) + 8 * (r >> 2)) * ldc);
      } else if (col < n) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (row0 + rbase + (r & 3) + 8 * (r >> 2) < m)
            __builtin_nontemporal_store(o[r], cp + ((r & 3) + 8 * (r >> 2)) * ldc);
      }
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
HA_EXPORT int ha_cdist_h3_fpad(int f) { return f <= 0 ? -1 : (f + KC - 1) / KC * KC; }

// planes: n * 2 * fpad halfs; aux: n float2 {|x|^2, 1/s}
HA_EXPORT int ha_cdist_h3_pack(const float* X, int64_t n, int f, int64_t ldx, void* planes, void* aux,
                               void* stream) {
  if (n <= 0) return HA_OK;
  const int fpad = ha_cdist_h3_fpad(f);
  if (fpad < 0) return HA_BAD_ARG;
  hipLaunchKernelGGL(cdist_pack, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, X, n, f, ldx,
                     fpad, (_Float16*)planes, (float2*)aux);
  return ha_launch_status();
}

// mode: 0 euclidean, 1 squared euclidean, 2 gaussian exp(-scale d2)
HA_EXPORT int ha_cdist_h3(const void* PX, const void* AX, int64_t m, const void* PY, const void* AY, int64_t n,
                          int f, float* C, int64_t ldc, int mode, float scale, void* stream) {
  if (m <= 0 || n <= 0) return HA_OK;
  const int fpad = ha_cdist_h3_fpad(f);
  if (fpad < 0 || mode < 0 || mode > 2) return HA_BAD_ARG;
  const int64_t tiles = ((m + TM - 1) / TM) * ((n + TN - 1) / TN);
  const int64_t per_xcd = (tiles + 7) / 8;
  const size_t lds = 2 * IMG_H * 2 + 512 * 4;
#define HA_CD(MODE_)                                                                                          \
  case MODE_:                                                                                                 \
    hipFuncSetAttribute((const void*)cdist_h3<MODE_>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);  \
    hipLaunchKernelGGL(cdist_h3<MODE_>, dim3((unsigned)(per_xcd * 8)), dim3(256), lds, (hipStream_t)stream,   \
                       (const _Float16*)PX, (const float2*)AX, m, (const _Float16*)PY, (const float2*)AY, n, fpad, \
                       C, ldc, scale);                                                                        \
    break;
  switch (mode) {
    HA_CD(0)
    HA_CD(1)
    HA_CD(2)
  }
#undef HA_CD
  return ha_launch_status();
}
