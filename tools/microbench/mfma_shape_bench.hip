// Sustained fp16 MFMA throughput under full-chip load: v_mfma_f32_32x32x16_f16 vs
// v_mfma_f32_16x16x32_f16 (same FLOP per instruction-cycle on paper), random operands, 8 waves
// per CU, 4 independent accumulator chains per wave. Prints TFLOP/s per shape (hipEvent timing).
//   hipcc --offload-arch=gfx950 -O3 mfma_shape_bench.hip -o /tmp/mfma_shape && /tmp/mfma_shape
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mm32(const halfx8* __restrict__ in, float* __restrict__ out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  halfx8 a = in[t & 4095], b = in[(t * 7 + 3) & 4095], c = in[(t * 13 + 5) & 4095], d = in[(t * 31 + 1) & 4095];
  floatx16 acc0 = (floatx16)(0.f), acc1 = acc0, acc2 = acc0, acc3 = acc0;
  for (int i = 0; i < iters; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c, d, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, d, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c, b, acc3, 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r] + acc2[r] + acc3[r];
  out[t] = s;
}

__global__ __launch_bounds__(256) void mm16(const halfx8* __restrict__ in, float* __restrict__ out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  halfx8 a = in[t & 4095], b = in[(t * 7 + 3) & 4095], c = in[(t * 13 + 5) & 4095], d = in[(t * 31 + 1) & 4095];
  floatx4 acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = (floatx4)(0.f);
  for (int i = 0; i < iters; ++i) {
    // 4 x 16x16x32 = the FLOP of one 32x32x16; 16 accumulators keep the same register footprint
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16((j & 1) ? a : c, (j & 2) ? b : d, acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[t] = s;
}

int main() {
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = ncu * 2, threads = blocks * 256, iters = 20000;
  halfx8* in;
  float* out;
  hipMalloc(&in, 4096 * sizeof(halfx8));
  hipMalloc(&out, threads * sizeof(float));
  _Float16 h[4096 * 8];
  unsigned s = 12345;
  for (int i = 0; i < 4096 * 8; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = (_Float16)(((s >> 8) & 0xFFFF) / 65536.0f - 0.5f);
  }
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int shape = 0; shape < 2; ++shape) {
      hipEventRecord(e0);
      if (shape == 0) hipLaunchKernelGGL(mm32, dim3(blocks), dim3(256), 0, 0, in, out, iters);
      else hipLaunchKernelGGL(mm16, dim3(blocks), dim3(256), 0, 0, in, out, iters / 4);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      // per wave per iteration (32x32x16 form): 4 MFMAs x 2*32*32*16 flops
      const double flops = (double)(threads / 64) * iters * 4.0 * 2 * 32 * 32 * 16;
      printf("{\"shape\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", shape ? "16x16x32" : "32x32x16", rep,
             ms, flops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
