// Pairwise L2-family distances by quadratic expansion on the FP16 matrix cores with a 3-term
// split (the reference's quadratic_expansion=True path, heat/spatial/distance.py:46-63, 86-102).
//
// Each operand is packed once per call into fp16 hi/lo planes of its rows scaled by a power of two
// s (max |x_i| in [0.5, 1)), plus the exact fp32 squared norm and 1/s (cdist_pack).  Then
//     x.y = (hi_x.hi_y + hi_x.lo_y + lo_x.hi_y) / (s_x s_y)        (three MFMAs, fp32 accumulate)
// with ~fp32-GEMM accuracy, at 16x the per-instruction rate of the f32-input MFMA, and
//     d2 = max(|x|^2 + |y|^2 - 2 x.y, 0)  -> sqrt | identity | exp(-scale d2).
//
// Packed layout ("fragment-blocked"): rows are padded to a multiple of 128 with zero rows and
// stored per 32-row block as [block][kstep = fpad/16][hl][lane 64][8 halfs]: the 1 KB a wave
// feeds to one v_mfma_f32_32x32x16_f16 operand (lane = 32 h + j holds row j, features
// 16 kstep + 8 h .. +8) is contiguous, so every operand load is a lane-linear 16-byte access.
//
// Kernels (128 x 128 output tiles, 4 waves):
//  * cdist_p (fpad <= 128, the common case): a workgroup keeps one 128-row X panel resident in
//    LDS and sweeps a run of column tiles; each wave owns 32 columns of every tile and streams its
//    Y fragments straight from global memory into registers, issuing the NEXT tile's fragment
//    right after consuming the current one (one tile of prefetch, no barrier in the loop).  Y
//    traffic per output is 4*fpad/128 bytes and X is read once per run.
//  * cdist_t (any fpad): both operands staged through one LDS buffer in 32-feature chunks with
//    the next chunk in flight in registers.
// Workgroups are mapped XCD-aware (blocks resident on one XCD sweep the same column tiles, shared
// through that XCD's L2).  Distances are written with non-temporal stores (streamed output).
#include "common.h"

#include <type_traits>

namespace {

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

constexpr int TM = 128, TN = 128, KC = 32;  // KC: feature padding granularity of the planes
constexpr int FRAG_H = 512;                 // halfs per 1 KB operand fragment (64 lanes x 8)

__host__ __device__ inline int64_t padded_rows(int64_t n) { return (n + TM - 1) / TM * TM; }

// one wave per (padded) row: hi/lo fragments of the row into the blocked layout, aux = {|x|^2, 1/s}
__global__ __launch_bounds__(256) void cdist_pack(const float* __restrict__ X, int64_t n, int f, int64_t ldx,
                                                  int fpad, _Float16* __restrict__ planes,
                                                  float2* __restrict__ aux) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= padded_rows(n)) return;
  const bool live = row < n;
  const float* xr = X + (live ? row : 0) * ldx;
  float mx = 0.f, ss = 0.f;
  if (live)
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
  const int ksg = fpad / 16;
  _Float16* blk = planes + (row >> 5) * (int64_t)ksg * 2 * FRAG_H;
  const int j = (int)(row & 31);
  for (int g = lane; g < fpad / 8; g += 64) {
    halfx8 hi, lo;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = g * 8 + i;
      const float v = live && c < f ? xr[c] * s : 0.f;
      const _Float16 hv = (_Float16)v;
      hi[i] = hv;
      lo[i] = (_Float16)(v - (float)hv);
    }
    const int ks = g >> 1, h = g & 1;
    _Float16* d = blk + (int64_t)ks * 2 * FRAG_H + ((h << 5) | j) * 8;
    *reinterpret_cast<halfx8*>(d) = hi;
    *reinterpret_cast<halfx8*>(d + FRAG_H) = lo;
  }
  if (lane == 0) aux[row] = live ? make_float2(ss, 1.f / s) : make_float2(0.f, 0.f);
}

template <int MODE>
__device__ __forceinline__ float epi(float d2, float scale) {
  if (MODE == 0) return __builtin_amdgcn_sqrtf(d2);  // v_sqrt_f32 (1 ulp), no denormal rescaling
  if (MODE == 1) return d2;
  return __expf(-d2 * scale);
}

// acc[u] (32 x 32 block u of rows, this wave's 32 columns at col) -> C with the fused epilogue.
// Lane holds column j, rows (r&3) + 8(r>>2) + 4h of each block.
template <int MODE, int NU, bool NT = true>
__device__ __forceinline__ void store_blocks(const floatx16 (&acc)[NU], const float* rowv, int rb0, int64_t row0,
                                             int64_t m, int64_t col, int64_t n, float ynv, float m2isy, float* C,
                                             int64_t ldc, float scale, int h, bool interior) {
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int rbase = (rb0 + u) * 32 + 4 * h;
    float* cp = C + (row0 + rbase) * ldc + col;
    float o[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = rbase + (r & 3) + 8 * (r >> 2);
      const float d2 = fmaxf(fmaf(m2isy * rowv[128 + rl], acc[u][r], rowv[rl] + ynv), 0.f);
      o[r] = epi<MODE>(d2, scale);
    }
    if (interior) {
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

// ------------------------------------------------------------------ panel-resident kernel, fpad <= 128
// ABL (timing ablation in tools/microbench only): 1 = no stores
template <int MODE, int KS, int ABL = 0>
__global__ __launch_bounds__(256, 2) void cdist_p(const _Float16* __restrict__ PX, const float2* __restrict__ AX,
                                                  int64_t m, const _Float16* __restrict__ PY,
                                                  const float2* __restrict__ AY, int64_t n, float* __restrict__ C,
                                                  int64_t ldc, float scale, int run) {
  constexpr int PANEL_H = 4 * KS * 2 * FRAG_H;  // 128 rows x 16 KS features x {hi, lo}
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  _Float16* xs = reinterpret_cast<_Float16*>(smem);
  float* rowv = reinterpret_cast<float*>(smem + PANEL_H * 2);  // xn[128], isx[128]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;

  // block b runs on XCD b % 8; the blocks of one XCD take consecutive t = consecutive row panels of
  // one column run, so they stream the same Y tiles (one L2 fill per XCD)
  const int64_t panels = (m + TM - 1) / TM, tiles_n = (n + TN - 1) / TN;
  const int64_t runs = (tiles_n + run - 1) / run;
  const int64_t total = panels * runs, per_xcd = (total + 7) / 8;
  const int64_t b = blockIdx.x;
  const int64_t t = (b % 8) * per_xcd + b / 8;
  if (t >= total) return;
  const int64_t rp = t % panels, cr = t / panels;
  const int64_t row0 = rp * TM;
  const int64_t c_begin = cr * run, c_end = c_begin + run < tiles_n ? c_begin + run : tiles_n;

  // resident X panel (contiguous in the blocked layout) and its row values
  {
    const halfx8* src = reinterpret_cast<const halfx8*>(PX + rp * (int64_t)PANEL_H);
    halfx8* dst = reinterpret_cast<halfx8*>(xs);
#pragma unroll
    for (int i = tid; i < PANEL_H / 8; i += 256) dst[i] = src[i];
    if (tid < 128) {
      const float2 a = AX[row0 + tid];
      rowv[tid] = a.x;
      rowv[128 + tid] = a.y;
    }
  }

  // this wave's Y fragments of column tile c: 32-row block 4c + wave
  auto yfrag = [&](int64_t c, int ks, int hl) {
    return *reinterpret_cast<const halfx8*>(PY + ((c * 4 + wave) * KS + ks) * (2 * FRAG_H) + hl * FRAG_H + lane * 8);
  };
  halfx8 y[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    y[ks][0] = yfrag(c_begin, ks, 0);
    y[ks][1] = yfrag(c_begin, ks, 1);
  }
  float2 ya = AY[c_begin * TN + wave * 32 + j];
  __syncthreads();

  for (int64_t c = c_begin; c < c_end; ++c) {
    const bool more = c + 1 < c_end;
    const int64_t cn = more ? c + 1 : c;  // the last tile re-reads itself: no branches around loads
    // the X fragments are loop-invariant; an opaque per-iteration base keeps the compiler from
    // hoisting all of them (4 x KS x 2 x 4 VGPRs) out of the loop
    int xoff = lane * 8;
    asm volatile("" : "+v"(xoff));
    const _Float16* xl = xs + xoff;
    floatx16 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = (floatx16)(0.f);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const halfx8 bh = y[ks][0], bl = y[ks][1];
      y[ks][0] = yfrag(cn, ks, 0);  // next tile's fragments into the slots just consumed
      y[ks][1] = yfrag(cn, ks, 1);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const halfx8 ah = *reinterpret_cast<const halfx8*>(xl + ((u * KS + ks) * 2 + 0) * FRAG_H);
        const halfx8 al = *reinterpret_cast<const halfx8*>(xl + ((u * KS + ks) * 2 + 1) * FRAG_H);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[u], 0, 0, 0);
      }
    }
    const float2 yc = ya;
    ya = AY[cn * TN + wave * 32 + j];
    const int64_t col = c * TN + wave * 32 + j;
    if (ABL == 1) {
      float s = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[u][r];
      if (s == 1234.5f) C[col] = s;  // keep the MFMAs alive
      continue;
    }
    // epilogue. Row values come from LDS through the laundered base (hoisting them would pin
    // 128 VGPRs), and the store address is a wave-uniform row pointer (SGPRs, bumped 8 rows at a
    // time) plus one 32-bit per-lane byte offset, so no 64-bit per-store addresses are kept.
    const float ynv = yc.x, m2isy = -2.f * yc.y;
    const float* rv = rowv + (xoff >> 3) - lane + 4 * h;  // == rowv + 4h, opaque to LICM
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    int64_t ld4 = ldc * 4;
    asm volatile("" : "+s"(ld4));  // per-iteration, so the row offsets are not hoisted into spilled SGPRs
    char* p = reinterpret_cast<char*>(C + row0 * ldc + c * TN + wv * 32);
    const uint32_t lb = (uint32_t)(4 * h * ld4 + j * 4);
    const bool interior = row0 + TM <= m && (c + 1) * TN <= n;
    int rows_left = (int)((m - row0 < TM ? m - row0 : TM) - 4 * h);
    asm volatile("" : "+v"(rows_left));  // keep the 64 row predicates out of the loop preheader
    auto tile_out = [&](auto edge) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = u * 32 + 8 * q;  // + 4h + rr
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const float d2 = fmaxf(fmaf(m2isy * rv[128 + rl + rr], acc[u][4 * q + rr], rv[rl + rr] + ynv), 0.f);
            const float o = epi<MODE>(d2, scale);
            float* dst = reinterpret_cast<float*>(p + rr * ld4 + lb);
            if (!decltype(edge)::value || (col < n && rl + rr < rows_left)) __builtin_nontemporal_store(o, dst);
          }
          p += 8 * ld4;
        }
      }
    };
    if (interior) tile_out(std::false_type{});
    else tile_out(std::true_type{});
  }
}

// ---------------------------------------------------------------------- LDS-staged tile kernel, any fpad
template <int MODE>
__global__ __launch_bounds__(256, 3) void cdist_t(const _Float16* __restrict__ PX, const float2* __restrict__ AX,
                                                  int64_t m, const _Float16* __restrict__ PY,
                                                  const float2* __restrict__ AY, int64_t n, int fpad,
                                                  float* __restrict__ C, int64_t ldc, float scale) {
  constexpr int IMG_H = 4 * 2 * 2 * FRAG_H;  // one 32-feature chunk of 128 rows: [rb][s][hl][lane][8]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  _Float16* img = reinterpret_cast<_Float16*>(smem);             // [op][IMG_H]
  float* rowv = reinterpret_cast<float*>(smem + 2 * IMG_H * 2);  // xn[128], isx[128], yn[128], isy[128]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5;

  // XCD-aware tile order: workgroup b runs on XCD b % 8; give each XCD a contiguous band of tiles,
  // grouped 8 tile-rows at a time so the workgroups resident on one XCD share 8 X and 8 Y panels
  const int64_t tiles_n = (n + TN - 1) / TN, tiles_m = (m + TM - 1) / TM;
  const int64_t tiles = tiles_m * tiles_n;
  const int64_t per_xcd = (tiles + 7) / 8;
  const int64_t b = blockIdx.x;
  const int64_t t = (b % 8) * per_xcd + b / 8;  // a bijection of [0, 8 per_xcd)
  if (t >= tiles) return;
  constexpr int64_t GROUP = 8;
  const int64_t grp = t / (GROUP * tiles_n);
  const int64_t first = grp * GROUP;
  const int64_t gsz = tiles_m - first < GROUP ? tiles_m - first : GROUP;
  const int64_t in = t - grp * GROUP * tiles_n;
  const int64_t row0 = (first + in % gsz) * TM, col0 = (in / gsz) * TN;

  if (tid < 128) {
    const float2 a = AX[row0 + tid];
    rowv[tid] = a.x;
    rowv[128 + tid] = a.y;
  } else {
    const float2 a = AY[col0 + tid - 128];
    rowv[256 + tid - 128] = a.x;
    rowv[384 + tid - 128] = a.y;
  }

  const int ksg = fpad / 16, nch = fpad / KC;
  // chunk ch of an operand = k-steps 2ch, 2ch+1 of its four 32-row blocks: 16 fragments, copied
  // lane-linearly (piece q: fragment q/64, lane q%64)
  halfx8 stg[8];
  auto load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int op = i >> 2, q = tid + 256 * (i & 3);
      const int fr = q >> 6, l = q & 63;
      const int rb = fr >> 2, s = (fr >> 1) & 1, hl = fr & 1;
      const int64_t blk = (op == 0 ? row0 : col0) / 32 + rb;
      const _Float16* P = op == 0 ? PX : PY;
      stg[i] = *reinterpret_cast<const halfx8*>(P + ((blk * ksg + 2 * ch + s) * 2 + hl) * FRAG_H + l * 8);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      *reinterpret_cast<halfx8*>(img + (i >> 2) * IMG_H + (tid + 256 * (i & 3)) * 8) = stg[i];
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = (floatx16)(0.f);
  const int wr = wave >> 1, wc = wave & 1;

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
        const int rb = 2 * wr + u, cb = 2 * wc + u;
        ah[u] = *reinterpret_cast<const halfx8*>(ix + ((rb * 2 + s) * 2 + 0) * FRAG_H + lane * 8);
        al[u] = *reinterpret_cast<const halfx8*>(ix + ((rb * 2 + s) * 2 + 1) * FRAG_H + lane * 8);
        bh[u] = *reinterpret_cast<const halfx8*>(iy + ((cb * 2 + s) * 2 + 0) * FRAG_H + lane * 8);
        bl[u] = *reinterpret_cast<const halfx8*>(iy + ((cb * 2 + s) * 2 + 1) * FRAG_H + lane * 8);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
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

  const bool interior = row0 + TM <= m && col0 + TN <= n;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int cl = (2 * wc + v) * 32 + (lane & 31);
    const floatx16 a2[2] = {acc[0][v], acc[1][v]};
    store_blocks<MODE, 2>(a2, rowv, 2 * wr, row0, m, col0 + cl, n, rowv[256 + cl], -2.f * rowv[384 + cl], C, ldc,
                          scale, h, interior);
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
HA_EXPORT int ha_cdist_h3_fpad(int f) { return f <= 0 ? -1 : (f + KC - 1) / KC * KC; }

HA_EXPORT int64_t ha_cdist_h3_rows(int64_t n) { return n <= 0 ? 0 : padded_rows(n); }

// planes: ha_cdist_h3_rows(n) * 2 * fpad halfs (blocked layout); aux: ha_cdist_h3_rows(n) float2
HA_EXPORT int ha_cdist_h3_pack(const float* X, int64_t n, int f, int64_t ldx, void* planes, void* aux,
                               void* stream) {
  if (n <= 0) return HA_OK;
  const int fpad = ha_cdist_h3_fpad(f);
  if (fpad < 0) return HA_BAD_ARG;
  hipLaunchKernelGGL(cdist_pack, dim3((unsigned)(padded_rows(n) / 4)), dim3(256), 0, (hipStream_t)stream, X, n, f,
                     ldx, fpad, (_Float16*)planes, (float2*)aux);
  return ha_launch_status();
}

// column tiles per workgroup of cdist_p: long runs amortise the X panel, short runs balance the tail
static int cdist_run(int64_t m, int64_t n) {
  const int64_t tiles = ((m + TM - 1) / TM) * ((n + TN - 1) / TN);
  int64_t r = tiles / 4096;
  return (int)(r < 1 ? 1 : r > 16 ? 16 : r);
}

template <int MODE, int KS>
static void launch_p(const void* PX, const void* AX, int64_t m, const void* PY, const void* AY, int64_t n, float* C,
                     int64_t ldc, float scale, hipStream_t stream) {
  const int run = cdist_run(m, n);
  const int64_t panels = (m + TM - 1) / TM, runs = ((n + TN - 1) / TN + run - 1) / run;
  const int64_t per_xcd = (panels * runs + 7) / 8;
  const size_t lds = 4 * KS * 2 * FRAG_H * 2 + 256 * 4;
  hipFuncSetAttribute((const void*)cdist_p<MODE, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((cdist_p<MODE, KS>), dim3((unsigned)(per_xcd * 8)), dim3(256), lds, stream, (const _Float16*)PX,
                     (const float2*)AX, m, (const _Float16*)PY, (const float2*)AY, n, C, ldc, scale, run);
}

template <int MODE>
static void launch_t(const void* PX, const void* AX, int64_t m, const void* PY, const void* AY, int64_t n, int fpad,
                     float* C, int64_t ldc, float scale, hipStream_t stream) {
  const int64_t tiles = ((m + TM - 1) / TM) * ((n + TN - 1) / TN);
  const int64_t per_xcd = (tiles + 7) / 8;
  const size_t lds = 2 * (4 * 2 * 2 * FRAG_H) * 2 + 512 * 4;
  hipFuncSetAttribute((const void*)cdist_t<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(cdist_t<MODE>, dim3((unsigned)(per_xcd * 8)), dim3(256), lds, stream, (const _Float16*)PX,
                     (const float2*)AX, m, (const _Float16*)PY, (const float2*)AY, n, fpad, C, ldc, scale);
}

template <int MODE>
static void launch(const void* PX, const void* AX, int64_t m, const void* PY, const void* AY, int64_t n, int fpad,
                   float* C, int64_t ldc, float scale, hipStream_t stream) {
  switch (fpad) {
    case 32: launch_p<MODE, 2>(PX, AX, m, PY, AY, n, C, ldc, scale, stream); break;
    case 64: launch_p<MODE, 4>(PX, AX, m, PY, AY, n, C, ldc, scale, stream); break;
    case 96: launch_p<MODE, 6>(PX, AX, m, PY, AY, n, C, ldc, scale, stream); break;
    case 128: launch_p<MODE, 8>(PX, AX, m, PY, AY, n, C, ldc, scale, stream); break;
    default: launch_t<MODE>(PX, AX, m, PY, AY, n, fpad, C, ldc, scale, stream);
  }
}

// mode: 0 euclidean, 1 squared euclidean, 2 gaussian exp(-scale d2); PX/PY from ha_cdist_h3_pack
// (row offsets into a packed operand must be multiples of 128)
HA_EXPORT int ha_cdist_h3(const void* PX, const void* AX, int64_t m, const void* PY, const void* AY, int64_t n,
                          int f, float* C, int64_t ldc, int mode, float scale, void* stream) {
  if (m <= 0 || n <= 0) return HA_OK;
  const int fpad = ha_cdist_h3_fpad(f);
  if (fpad < 0 || mode < 0 || mode > 2) return HA_BAD_ARG;
  const hipStream_t s = (hipStream_t)stream;
  if (mode == 0) launch<0>(PX, AX, m, PY, AY, n, fpad, C, ldc, scale, s);
  else if (mode == 1) launch<1>(PX, AX, m, PY, AY, n, fpad, C, ldc, scale, s);
  else launch<2>(PX, AX, m, PY, AY, n, fpad, C, ldc, scale, s);
  return ha_launch_status();
}
