// Lloyd-step epilogue in ONE launch: new centroids from the (all-reduced) fp64 sums and counts,
// empty clusters keep their centroid, and the squared centroid shift. Replaces ~12 small torch
// kernels (casts, cat, clamp, divide, where, difference, square, sum) whose launch gaps cost
// ~0.1 ms per 5 ms k-means step.
//   packed = [sums (k x f, fp64) | counts (k, fp64)]
//   newC[c, j] = counts[c] > 0 ? (float)(sums[c, j] / counts[c]) : C[c, j]
//   shift     += (C[c, j] - newC[c, j])^2      (fp64, zeroed here)
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void km_finalize(const double* __restrict__ packed, int k, int f,
                                                   const float* __restrict__ C, int64_t ldc,
                                                   float* __restrict__ newC, double* __restrict__ shift) {
  const int64_t kf = (int64_t)k * f;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < kf; i += (int64_t)gridDim.x * 256) {
    const int64_t c = i / f, j = i - c * f;
    const double cnt = packed[kf + c];
    const float old = C[c * ldc + j];
    const float nv = cnt > 0.0 ? (float)(packed[i] / cnt) : old;
    newC[i] = nv;
    const double d = (double)old - (double)nv;
    acc = fma(d, d, acc);
  }
  acc = ha_wave_sum_d(acc);
  __shared__ double part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(shift, part[0] + part[1] + part[2] + part[3]);
}

}  // namespace

HA_EXPORT int ha_km_finalize(const double* packed, int k, int f, const float* C, int64_t ldc, float* newC,
                             double* shift, void* stream) {
  if (k <= 0 || f <= 0 || ldc < f) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(shift, 0, sizeof(double), s);
  const int64_t kf = (int64_t)k * f;
  int64_t blocks = (kf + 256 * 8 - 1) / (256 * 8);
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(km_finalize, dim3((unsigned)blocks), dim3(256), 0, s, packed, k, f, C, ldc, newC, shift);
  return ha_launch_status();
}
