// Lloyd-step epilogue in ONE launch: new centroids from the (all-reduced) sums and counts, empty
// clusters keep their centroid, and the squared centroid shift. Replaces ~12 small torch kernels
// (casts, cat, clamp, divide, where, difference, square, sum) whose launch gaps cost ~0.1 ms per
// 5 ms k-means step.
//   newC[c, j] = counts[c] > 0 ? (float)(sums[c, j] / counts[c]) : C[c, j]
//   shift      = sum (C[c, j] - newC[c, j])^2      (fp64)
// Sums and counts are fp64 (the packed all-reduce buffer [sums | counts] of a distributed step) or
// fp32 (the update kernel's own output on a world of one: no cast/pack kernels in between).
// The shift is reduced without atomics on one address and without a memset launch: every block
// writes its partial, and the last block to finish (a self-resetting arrival counter in `ws`)
// adds them in a fixed order, so the result is also deterministic.
#include "common.h"

namespace {

constexpr int FIN_MAX_BLOCKS = 256;

template <typename T>
__global__ __launch_bounds__(256) void km_finalize(const T* __restrict__ sums, const T* __restrict__ counts, int k,
                                                   int f, const float* __restrict__ C, int64_t ldc,
                                                   float* __restrict__ newC, double* __restrict__ shift,
                                                   double* __restrict__ part, unsigned* __restrict__ arrived) {
  const int kf = k * f;
  double acc = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < kf; i += gridDim.x * 256) {
    const int c = i / f, j = i - c * f;
    const double cnt = (double)counts[c];
    const float old = C[(int64_t)c * ldc + j];
    const float nv = cnt > 0.0 ? (float)((double)sums[i] / cnt) : old;
    newC[i] = nv;
    const double d = (double)old - (double)nv;
    acc = fma(d, d, acc);
  }
  acc = ha_wave_sum_d(acc);
  __shared__ double wpart[4];
  __shared__ bool last;
  if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = wpart[0] + wpart[1] + wpart[2] + wpart[3];
    __threadfence();
    last = atomicAdd(arrived, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (threadIdx.x < 64) {
    double s = 0.0;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += 64) s += part[b];
    s = ha_wave_sum_d(s);
    if (threadIdx.x == 0) {
      *shift = s;
      *arrived = 0u;  // ready for the next launch on this workspace
    }
  }
}

template <typename T>
int launch(const T* sums, const T* counts, int k, int f, const float* C, int64_t ldc, float* newC, double* shift,
           void* ws, hipStream_t s) {
  const int64_t kf = (int64_t)k * f;
  int64_t blocks = (kf + 256 * 4 - 1) / (256 * 4);
  if (blocks > FIN_MAX_BLOCKS) blocks = FIN_MAX_BLOCKS;
  if (blocks < 1) blocks = 1;
  double* part = reinterpret_cast<double*>(ws);
  unsigned* arrived = reinterpret_cast<unsigned*>(part + FIN_MAX_BLOCKS);
  hipLaunchKernelGGL(km_finalize<T>, dim3((unsigned)blocks), dim3(256), 0, s, sums, counts, k, f, C, ldc, newC,
                     shift, part, arrived);
  return ha_launch_status();
}

}  // namespace

// bytes of the workspace (zero-initialised once by the caller, reused by every launch on one stream)
HA_EXPORT int64_t ha_km_finalize_workspace() { return FIN_MAX_BLOCKS * sizeof(double) + 64; }

// packed = [sums (k x f) | counts (k)], fp64
HA_EXPORT int ha_km_finalize(const double* packed, int k, int f, const float* C, int64_t ldc, float* newC,
                             double* shift, void* ws, void* stream) {
  if (k <= 0 || f <= 0 || ldc < f || (int64_t)k * f >= ((int64_t)1 << 31)) return HA_BAD_ARG;
  const int64_t kf = (int64_t)k * f;
  return launch<double>(packed, packed + kf, k, f, C, ldc, newC, shift, ws, (hipStream_t)stream);
}

// sums (k x f) and counts (k) as fp32 (single-process step)
HA_EXPORT int ha_km_finalize_f32(const float* sums, const float* counts, int k, int f, const float* C, int64_t ldc,
                                 float* newC, double* shift, void* ws, void* stream) {
  if (k <= 0 || f <= 0 || ldc < f || (int64_t)k * f >= ((int64_t)1 << 31)) return HA_BAD_ARG;
  return launch<float>(sums, counts, k, f, C, ldc, newC, shift, ws, (hipStream_t)stream);
}
