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

// Inter-workgroup hand-off inside one launch without a per-block release fence (the
// "write-through stores + counter" form of the CDNA4 visibility rules): every handed-off word is
// stored sc1 (relaxed agent-scope atomic store on a GLOBAL pointer), every storing wave drains
// (s_waitcnt vmcnt(0)) before the workgroup barrier, one lane then takes a ticket with an
// agent-scope atomic add; the workgroup whose add came last does ONE agent acquire (L1
// invalidate) and reads. A release fence per block (buffer_wbl2) serialises per CU: ~9 us per
// block at 8 blocks per CU, measured as +70 us on a 0.64 ms moments pass with 2048 blocks.
typedef __attribute__((address_space(1))) unsigned long long ha_gu64;
typedef __attribute__((address_space(1))) unsigned ha_gu32;

__device__ __forceinline__ void ha_store_wt(double* p, double v) {
  __hip_atomic_store((ha_gu64*)(p), (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
