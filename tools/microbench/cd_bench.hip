// Ablation timing of the fp16x3 cdist kernel on one 65536 x 65536 tile, f = 128 (and f = 18).
#include "../../heat_amd/ops/csrc/cdist_f16x3.hip"
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int ABL>
float run(const _Float16* P, const float2* A, int64_t n, int f, float* C) {
  const int fpad = ha_cdist_h3_fpad(f);
  const int64_t tiles = ((n + TM - 1) / TM) * ((n + TN - 1) / TN);
  const int64_t per_xcd = (tiles + 7) / 8;
  const size_t lds = 2 * IMG_H * 2 + 512 * 4;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((cdist_h3<0, ABL>), dim3((unsigned)(per_xcd * 8)), dim3(256), lds, 0, P, A, n, P, A, n, fpad, C, n, 1.f);
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 5; ++w)
    hipLaunchKernelGGL((cdist_h3<0, ABL>), dim3((unsigned)(per_xcd * 8)), dim3(256), lds, 0, P, A, n, P, A, n, fpad, C, n, 1.f);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 5;
}

int main() {
  const int64_t n = 65536;
  for (int f : {128, 18}) {
    float *X, *C; _Float16* P; float2* A;
    const int fpad = ha_cdist_h3_fpad(f);
    CHECK(hipMalloc(&X, n * f * 4)); CHECK(hipMalloc(&C, n * n * 4));
    CHECK(hipMalloc(&P, n * 2 * fpad * 2)); CHECK(hipMalloc(&A, n * 8));
    float* h = (float*)malloc(n * f * 4);
    uint32_t st = 7;
    for (int64_t i = 0; i < n * f; ++i) { st = st * 1664525u + 1013904223u; h[i] = (st >> 8) * (1.f / 16777216.f); }
    CHECK(hipMemcpy(X, h, n * f * 4, hipMemcpyHostToDevice));
    if (ha_cdist_h3_pack(X, n, f, f, P, A, nullptr) != 0) { printf("pack failed\n"); return 1; }
    const double gb = n * n * 4 / 1e9;
    float t;
    t = run<0>(P, A, n, f, C); printf("f=%d full      %.3f ms  %.0f GB/s out\n", f, t, gb / t * 1e3);
    t = run<1>(P, A, n, f, C); printf("f=%d no-store  %.3f ms\n", f, t);
    t = run<2>(P, A, n, f, C); printf("f=%d no-mfma   %.3f ms  %.0f GB/s out\n", f, t, gb / t * 1e3);
    CHECK(hipFree(X)); CHECK(hipFree(C)); CHECK(hipFree(P)); CHECK(hipFree(A)); free(h);
  }
  return 0;
}
