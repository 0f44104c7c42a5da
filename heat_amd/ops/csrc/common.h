// Shared helpers for the heat_amd CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define HA_EXPORT extern "C" __attribute__((visibility("default")))

// status codes returned to Python
enum { HA_OK = 0, HA_BAD_ARG = 1, HA_UNSUPPORTED = 2, HA_LAUNCH = 3 };

static inline int ha_launch_status() { return hipGetLastError() == hipSuccess ? HA_OK : HA_LAUNCH; }

__device__ __forceinline__ float ha_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double ha_wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
