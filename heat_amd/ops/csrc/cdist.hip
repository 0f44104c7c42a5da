// Pairwise distances on CDNA4 (gfx950): the hot path of heat.spatial (reference
// heat/spatial/distance.py: _euclidian 16 / _euclidian_fast 31 / _gaussian 66 / _manhattan 105).
//
// L2 family: one fp32-MFMA (v_mfma_f32_32x32x2_f32) GEMM tile of X.Y^T per 128x128 output block
// with a fused epilogue  d2 = |x|^2 + |y|^2 - 2 x.y, clamp >= 0, then sqrt (euclidean), nothing
// (squared) or exp(-d2 / (2 sigma^2)) (gaussian / rbf).  Row norms are computed while staging.
// As in the k-means kernel the K dimension is permuted (half h of the wave owns features
// h*16 + s of each 32-feature chunk), so operand fragments are contiguous 16-byte LDS reads.
//
// L1: VALU tile kernel (|x - y| has no matrix-core form), 64x64 outputs per workgroup, no
// m x n x f intermediate (the reference's _manhattan_fast materialises one).
#include "common.h"

#include <cmath>
#include <cstdlib>

namespace {

constexpr int BM = 128, BN = 128, KB = 32;   // output tile, features per LDS chunk
constexpr int S4 = KB / 2 / 4;               // float4 groups per half per chunk (=4)

enum { MODE_EUCLID = 0, MODE_SQEUCLID = 1, MODE_GAUSS = 2 };

// LDS image of one 128-row operand chunk: [rb (4)][s4 (4)][lane (64)][4]
__device__ __forceinline__ int frag_off(int rb, int s4, int lane) { return ((rb * S4 + s4) * 64 + lane) * 4; }

__device__ __forceinline__ void stage(const float* __restrict__ src, int64_t nrows, int f, int64_t ld, int64_t row0,
                                      int k0, float* __restrict__ dst, float* __restrict__ nrm, int tid) {
  // 128 rows x 32 features = 1024 float4, 4 per thread
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int q = tid + 256 * it;        // float4 index in fragment order
    const int lane = q & 63;
    const int s4 = (q >> 6) & (S4 - 1);
    const int rb = q >> 8;
    const int j = lane & 31, h = lane >> 5;
    const int64_t row = row0 + rb * 32 + j;
    const int col = k0 + h * (KB / 2) + 4 * s4;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < nrows && col < f) v = *reinterpret_cast<const floatx4*>(src + row * ld + col);
    *reinterpret_cast<floatx4*>(dst + frag_off(rb, s4, lane)) = v;
    float ss = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    // 8 float4 per row per chunk (2 halves x 4 groups): reduce into the row's norm
    atomicAdd(&nrm[rb * 32 + j], ss);
  }
}

__global__ __launch_bounds__(256, 2) void cdist_l2(const float* __restrict__ X, int64_t m, const float* __restrict__ Y,
                                                  int64_t n, int f, int64_t ldx, int64_t ldy, float* __restrict__ C,
                                                  int64_t ldc, int mode, float scale) {
  __shared__ __attribute__((aligned(16))) float sx[BM * KB];
  __shared__ __attribute__((aligned(16))) float sy[BN * KB];
  __shared__ float xn[BM];
  __shared__ float yn[BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5;
  // XCD-friendly order: consecutive workgroups walk along a row of tiles (they share X rows)
  const int64_t tiles_n = (n + BN - 1) / BN;
  const int64_t tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int64_t row0 = tm * BM, col0 = tn * BN;
  const int wr = wave >> 1, wc = wave & 1;  // wave owns a 64x64 quadrant: row blocks 2wr..2wr+1
  if (tid < BM) xn[tid] = 0.f;
  if (tid >= 128 && tid < 128 + BN) yn[tid - 128] = 0.f;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (floatx16)(0.f);
  __syncthreads();
  for (int k0 = 0; k0 < f; k0 += KB) {
    stage(X, m, f, ldx, row0, k0, sx, xn, tid);
    stage(Y, n, f, ldy, col0, k0, sy, yn, tid);
    __syncthreads();
#pragma unroll
    for (int s4 = 0; s4 < S4; ++s4) {
      floatx4 a[2], b[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        a[u] = *reinterpret_cast<const floatx4*>(sx + frag_off(2 * wr + u, s4, lane));
        b[u] = *reinterpret_cast<const floatx4*>(sy + frag_off(2 * wc + u, s4, lane));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int v = 0; v < 2; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][t], b[v][t], acc[u][v], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: lane owns column j of each 32x32 block, rows (reg&3) + 8*(reg>>2) + 4*h
  const int j = lane & 31;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int cl = (2 * wc + v) * 32 + j;
    const int64_t col = col0 + cl;
    const float ynv = yn[cl];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (2 * wr + u) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t row = row0 + rl;
        float d2 = fmaxf(fmaf(-2.f, acc[u][v][r], xn[rl] + ynv), 0.f);
        float out;
        if (mode == MODE_EUCLID) out = sqrtf(d2);
        else if (mode == MODE_SQEUCLID) out = d2;
        else out = __expf(-d2 * scale);
        if (row < m && col < n) C[row * ldc + col] = out;
      }
    }
  }
}

// Difference-based (exact) distances on the VALU, 64x64 outputs per workgroup: thread (tr, tc)
// owns rows tr + 16u and the 4 CONSECUTIVE columns 4tc..4tc+3, so the Y operand is one aligned
// ds_read_b128 per feature, the squared-difference accumulation runs on packed fp32
// (v_pk_add_f32 / v_pk_fma_f32: two pairs per instruction) and the output rows leave as 16-byte
// stores (16 lanes = 256 contiguous bytes).  XCD-banded tile order as in the MFMA kernels.
// Measured alternative (SUSY 40k x 18): 128 x 128 tiles with 8 x 8 outputs per thread (x and y as
// ds_read_b128, a quarter of the LDS cycles per output) ran 2.21 ms vs 2.25 ms, 1.80 ms with the
// stores removed: the loop is VALU-bound (packed fp32 gives no issue-rate gain over 2 scalar ops
// here), not LDS-bound, so the simpler 64 x 64 kernel stays.
// OP 0: sum |x-y| ; OP 1: sqrt(sum (x-y)^2) ; OP 2: sum (x-y)^2 ; OP 3: exp(-scale * sum (x-y)^2)
constexpr int LB = 64, LK = 32, LYS = LB + 4;
typedef float floatx2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void cdist_vk(const float* __restrict__ X, int64_t m, const float* __restrict__ Y,
                                                int64_t n, int f, int64_t ldx, int64_t ldy, float* __restrict__ C,
                                                int64_t ldc, float scale, int64_t per_xcd, int vec_out) {
  __shared__ float sx[LK][LB + 1];
  __shared__ __attribute__((aligned(16))) float sy[LK][LYS];
  const int tid = threadIdx.x;
  const int64_t tiles_n = (n + LB - 1) / LB;
  const int64_t tiles = ((m + LB - 1) / LB) * tiles_n;
  const int64_t t = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (t >= tiles) return;
  const int64_t row0 = (t / tiles_n) * LB, col0 = (t % tiles_n) * LB;
  const int tr = tid / 16, tc = tid % 16;
  floatx2 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a) acc[a][0] = acc[a][1] = (floatx2)(0.f);
  for (int k0 = 0; k0 < f; k0 += LK) {
    for (int e = tid; e < LB * LK; e += 256) {
      const int r = e / LK, c = e % LK;
      const int64_t gr = row0 + r, gc = col0 + r;
      sx[c][r] = (gr < m && k0 + c < f) ? X[gr * ldx + k0 + c] : 0.f;
      sy[c][r] = (gc < n && k0 + c < f) ? Y[gc * ldy + k0 + c] : 0.f;
    }
    __syncthreads();
    const int kk = (f - k0) < LK ? (f - k0) : LK;
    for (int k = 0; k < kk; ++k) {
      const floatx4 b = *reinterpret_cast<const floatx4*>(&sy[k][4 * tc]);
      const floatx2 b01 = {b[0], b[1]}, b23 = {b[2], b[3]};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float av = sx[k][tr + 16 * u];
        const floatx2 a2 = {av, av};
        const floatx2 d0 = a2 - b01, d1 = a2 - b23;
        if (OP == 0) {
          acc[u][0] += __builtin_elementwise_abs(d0);
          acc[u][1] += __builtin_elementwise_abs(d1);
        } else {
          acc[u][0] = __builtin_elementwise_fma(d0, d0, acc[u][0]);
          acc[u][1] = __builtin_elementwise_fma(d1, d1, acc[u][1]);
        }
      }
    }
    __syncthreads();
  }
  const int64_t col = col0 + 4 * tc;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t row = row0 + tr + 16 * u;
    if (row >= m) continue;
    float o[4] = {acc[u][0][0], acc[u][0][1], acc[u][1][0], acc[u][1][1]};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      if (OP == 1) o[v] = __builtin_amdgcn_sqrtf(o[v]);
      else if (OP == 3) o[v] = __expf(-o[v] * scale);
    }
    float* cp = C + row * ldc + col;
    if (vec_out && col + 3 < n) {
      const floatx4 ov = {o[0], o[1], o[2], o[3]};
      __builtin_nontemporal_store(ov, reinterpret_cast<floatx4*>(cp));
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (col + v < n) cp[v] = o[v];
    }
  }
}

// Exact kernel, round 5: 128 x 128 outputs per workgroup, 8 x 8 per thread (rows 4 tr + {0..3,
// 64..67}, columns 4 tc + {0..3, 64..67}: four ds_read_b128 per feature feed 64 difference pairs).
// The staging issues ALL of a chunk's global loads before the first LDS write (the kernel above
// waits for each load before issuing the next: its SUSY 40k x 18 run was bound by that serial
// load latency, 2.25 ms of which 1.80 ms without the stores): a thread loads 4 consecutive rows
// of one feature column (32 lanes = one 128-byte run of a row) and writes them transposed as one
// ds_write_b128. Squared differences on packed fp32 (x broadcast by op_sel), |x - y| on scalar
// v_sub + v_add with the abs modifier (no abs on packed ops).
constexpr int VB = 128, VK = 32, VS = VB + 4;  // tile, features per chunk, LDS row stride

// SYM (Y = X, m = n): only the tiles on or above the diagonal are launched (row-major order of the
// upper triangle), and an off-diagonal tile is also stored mirrored at (col, row): every distance
// pair is computed once (the reference's Y = None path, heat/spatial/distance.py:237, 265-362).
template <int OP, bool SYM>
__global__ __launch_bounds__(256, 2) void cdist_vx(const float* __restrict__ X, int64_t m, const float* __restrict__ Y,
                                                   int64_t n, int f, int64_t ldx, int64_t ldy, float* __restrict__ C,
                                                   int64_t ldc, float scale, int64_t per_xcd, int vec_out) {
  __shared__ __attribute__((aligned(16))) float sx[VK * VS];
  __shared__ __attribute__((aligned(16))) float sy[VK * VS];
  const int tid = threadIdx.x;
  const int64_t tiles_n = (n + VB - 1) / VB;
  const int64_t tiles = SYM ? tiles_n * (tiles_n + 1) / 2 : ((m + VB - 1) / VB) * tiles_n;
  const int64_t t = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (t >= tiles) return;
  int64_t row0, col0;
  if (SYM) {
    // t -> (i, j >= i): row i holds tiles_n - i tiles; invert the prefix sums with the quadratic
    // formula, then correct the rounding
    const double T = (double)tiles_n;
    int64_t i = (int64_t)((2.0 * T + 1.0 - sqrt((2.0 * T + 1.0) * (2.0 * T + 1.0) - 8.0 * (double)t)) / 2.0);
    auto first = [&](int64_t r) { return r * tiles_n - r * (r - 1) / 2; };
    while (i > 0 && first(i) > t) --i;
    while (first(i + 1) <= t) ++i;
    row0 = i * VB;
    col0 = (i + (t - first(i))) * VB;
  } else {
    row0 = (t / tiles_n) * VB;
    col0 = (t % tiles_n) * VB;
  }
  const int tr = tid >> 4, tc = tid & 15;
  // staging role: feature column sc, 4-row groups sq + 8 u (u = 0..3) of the 32 groups
  const int sc = tid & 31, sq = tid >> 5;
  floatx2 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (floatx2)(0.f);
  // buffer descriptors over this tile's rows (the range check returns 0 past the last valid row):
  // one 32-bit per-lane offset, the per-load row offsets are scalars
  const int xrows = (int)(m - row0 < VB ? m - row0 : VB), yrows = (int)(n - col0 < VB ? n - col0 : VB);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X + row0 * ldx), (short)0, (int)(((int64_t)(xrows - 1) * ldx + f) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Y + col0 * ldy), (short)0, (int)(((int64_t)(yrows - 1) * ldy + f) * 4), 0x00020000);
  for (int k0 = 0; k0 < f; k0 += VK) {
    floatx4 vx[4], vy[4];
    const bool cin = k0 + sc < f;
    const int ox = (int)((4 * sq * ldx + k0 + sc) * 4), oy = (int)((4 * sq * ldy + k0 + sc) * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 32 * u + j;
        const float a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, ox, (int)(r * ldx * 4), 0));
        const float b = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, oy, (int)(r * ldy * 4), 0));
        vx[u][j] = cin ? a : 0.f;
        vy[u][j] = cin ? b : 0.f;
      }
    }
    if (k0 > 0) __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      *reinterpret_cast<floatx4*>(sx + sc * VS + 4 * (sq + 8 * u)) = vx[u];
      *reinterpret_cast<floatx4*>(sy + sc * VS + 4 * (sq + 8 * u)) = vy[u];
    }
    __syncthreads();
    const int kk = (f - k0) < VK ? (f - k0) : VK;
    for (int k = 0; k < kk; ++k) {
      const floatx4 xa = *reinterpret_cast<const floatx4*>(sx + k * VS + 4 * tr);
      const floatx4 xb = *reinterpret_cast<const floatx4*>(sx + k * VS + 64 + 4 * tr);
      const floatx4 ya = *reinterpret_cast<const floatx4*>(sy + k * VS + 4 * tc);
      const floatx4 yb = *reinterpret_cast<const floatx4*>(sy + k * VS + 64 + 4 * tc);
      const float xv[8] = {xa[0], xa[1], xa[2], xa[3], xb[0], xb[1], xb[2], xb[3]};
      const floatx2 yv[4] = {{ya[0], ya[1]}, {ya[2], ya[3]}, {yb[0], yb[1]}, {yb[2], yb[3]}};
#pragma unroll
      for (int a = 0; a < 8; ++a) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (OP == 0) {
            acc[a][b][0] += __builtin_fabsf(xv[a] - yv[b][0]);
            acc[a][b][1] += __builtin_fabsf(xv[a] - yv[b][1]);
          } else {
            const floatx2 d = (floatx2){xv[a], xv[a]} - yv[b];
            acc[a][b] = __builtin_elementwise_fma(d, d, acc[a][b]);
          }
        }
      }
    }
  }
  auto fin = [&](float v) {
    if (OP == 1) return __builtin_amdgcn_sqrtf(v);
    if (OP == 3) return __expf(-v * scale);
    return v;
  };
  if (SYM && row0 != col0) {
    // the mirrored tile (col block, row block): thread's column 4 tc + j + 64 h becomes a row
    // holding its 8 values at columns 4 tr + {0..3} and 64 + 4 tr + {0..3}
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t row = col0 + 64 * h + 4 * tc + j;
        if (row >= n) continue;
        float o[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) o[a] = fin(acc[a][2 * h + (j >> 1)][j & 1]);
        float* rp = C + row * ldc + row0 + 4 * tr;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int64_t col = row0 + 4 * tr + 64 * half;
          if (vec_out && col + 3 < m) {
            __builtin_nontemporal_store((floatx4){o[4 * half], o[4 * half + 1], o[4 * half + 2], o[4 * half + 3]},
                                        reinterpret_cast<floatx4*>(rp + 64 * half));
          } else {
#pragma unroll
            for (int v = 0; v < 4; ++v)
              if (col + v < m) rp[64 * half + v] = o[4 * half + v];
          }
        }
      }
  }
  if (vec_out && row0 + VB <= m && col0 + VB <= n) {
    // whole tile (wave-uniform): 16 unguarded 16-byte stores per thread, no per-element branches
    // (the guarded form below costs ~400 VALU per thread, a quarter of the kernel's VALU work)
    float* base = C + (row0 + 4 * tr) * ldc + col0 + 4 * tc;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      float* rp = base + (int64_t)((a & 3) + 64 * (a >> 2)) * ldc;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        __builtin_nontemporal_store((floatx4){fin(acc[a][2 * h][0]), fin(acc[a][2 * h][1]), fin(acc[a][2 * h + 1][0]),
                                              fin(acc[a][2 * h + 1][1])},
                                    reinterpret_cast<floatx4*>(rp + 64 * h));
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int64_t row = row0 + 4 * tr + (a & 3) + 64 * (a >> 2);
    if (row >= m) continue;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t col = col0 + 64 * h + 4 * tc;
      float o[4] = {acc[a][2 * h][0], acc[a][2 * h][1], acc[a][2 * h + 1][0], acc[a][2 * h + 1][1]};
#pragma unroll
      for (int v = 0; v < 4; ++v) o[v] = fin(o[v]);
      float* cp = C + row * ldc + col;
      if (vec_out && col + 3 < n) {
        __builtin_nontemporal_store((floatx4){o[0], o[1], o[2], o[3]}, reinterpret_cast<floatx4*>(cp));
      } else {
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (col + v < n) cp[v] = o[v];
      }
    }
  }
}

}  // namespace

// mode: 0 euclidean, 1 squared euclidean, 2 gaussian (exp(-d2*scale)) - MFMA quadratic expansion;
//       3 manhattan; 4 / 5 / 6 = exact (difference-based) euclidean / squared / gaussian on the VALU
HA_EXPORT int ha_cdist(const float* X, int64_t m, const float* Y, int64_t n, int f, int64_t ldx, int64_t ldy, float* C,
                       int64_t ldc, int mode, float scale, void* stream) {
  if (m <= 0 || n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  static const bool vk64 = [] { const char* e = getenv("HEAT_CDIST_VK64"); return e && atoi(e) != 0; }();
  // mode bit 8: symmetric (Y is X, m == n): compute-once upper-triangle tiles, exact kernels only
  const bool sym = (mode & 256) != 0;
  mode &= 255;
  if (sym && (mode < 3 || X != Y || m != n || ldx != ldy)) return HA_BAD_ARG;
  // cdist_vx addresses a 128-row tile with 32-bit byte offsets
  const bool fits = (int64_t)VB * (ldx > ldy ? ldx : ldy) * 4 < 0x7fffffffLL;
  if (mode >= 3 && (!vk64 || sym) && fits) {
    const int64_t tn = (n + VB - 1) / VB;
    const int64_t tiles = sym ? tn * (tn + 1) / 2 : ((m + VB - 1) / VB) * tn;
    const int64_t per_xcd = (tiles + 7) / 8;
    if (per_xcd * 8 > 0x7fffffffLL) return HA_UNSUPPORTED;
    const int vec = ((ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
    const dim3 g((unsigned)(per_xcd * 8)), b(256);
#define HA_VX(OPV)                                                                                            \
  if (sym)                                                                                                   \
    hipLaunchKernelGGL((cdist_vx<OPV, true>), g, b, 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, scale, per_xcd, vec); \
  else                                                                                                       \
    hipLaunchKernelGGL((cdist_vx<OPV, false>), g, b, 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, scale, per_xcd, vec);
    switch (mode) {
      case 3: HA_VX(0) break;
      case 4: HA_VX(1) break;
      case 5: HA_VX(2) break;
      case 6: HA_VX(3) break;
      default: return HA_BAD_ARG;
    }
#undef HA_VX
    return ha_launch_status();
  }
  if (sym) return HA_UNSUPPORTED;
  if (mode >= 3) {  // round-4 64 x 64 kernel (HEAT_CDIST_VK64=1, A/B only)
    const int64_t tiles = ((m + LB - 1) / LB) * ((n + LB - 1) / LB);
    const int64_t per_xcd = (tiles + 7) / 8;
    if (per_xcd * 8 > 0x7fffffffLL) return HA_UNSUPPORTED;
    const int vec = ((ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
    const dim3 g((unsigned)(per_xcd * 8)), b(256);
    switch (mode) {
      case 3: hipLaunchKernelGGL(cdist_vk<0>, g, b, 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, scale, per_xcd, vec); break;
      case 4: hipLaunchKernelGGL(cdist_vk<1>, g, b, 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, scale, per_xcd, vec); break;
      case 5: hipLaunchKernelGGL(cdist_vk<2>, g, b, 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, scale, per_xcd, vec); break;
      case 6: hipLaunchKernelGGL(cdist_vk<3>, g, b, 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, scale, per_xcd, vec); break;
      default: return HA_BAD_ARG;
    }
    return ha_launch_status();
  }
  if (f % 4 != 0 || ldx % 4 != 0 || ldy % 4 != 0) return HA_BAD_ARG;
  const int64_t tiles = ((m + BM - 1) / BM) * ((n + BN - 1) / BN);
  if (tiles > 0x7fffffffLL) return HA_UNSUPPORTED;
  hipLaunchKernelGGL(cdist_l2, dim3((unsigned)tiles), dim3(256), 0, s, X, m, Y, n, f, ldx, ldy, C, ldc, mode, scale);
  return ha_launch_status();
}
