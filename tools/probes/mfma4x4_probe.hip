// Operand / result layout of v_mfma_f32_4x4x1_16b_f32 on gfx950 (not in the guides): one MFMA
// with A = a marker per lane and B = 1, then B = marker and A = 1; prints which lanes' A / B
// values land in each (lane, register) of D.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out) {
  const int l = threadIdx.x;
  floatx4 z = {0.f, 0.f, 0.f, 0.f};
  // A marker: 2^(l % 16) * (1 + l / 16) / 1000 would collide; use distinct lane ids with B = 1
  floatx4 d1 = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.f, z, 0, 0, 0);
  floatx4 d2 = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, (float)(l + 1), z, 0, 0, 0);
  for (int i = 0; i < 4; ++i) {
    out[l * 4 + i] = d1[i];
    out[256 + l * 4 + i] = d2[i];
  }
}

int main() {
  float* d;
  hipMalloc(&d, 512 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[512];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane reg : A-lane+1 (B=1) | B-lane+1 (A=1)\n");
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) printf("%2d %d : %4.0f | %4.0f\n", l, i, h[l * 4 + i], h[256 + l * 4 + i]);
  hipFree(d);
  return 0;
}
