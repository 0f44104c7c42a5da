// Ablation timing of the fp16x3 k-means assign kernel (n=12.5M, k=1024, f=64).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../heat_amd/ops/csrc -o h3_bench h3_bench.hip
#include "../../heat_amd/ops/csrc/kmeans_f16x3.hip"
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int NPB, bool EPI>
float time_variant(const _Float16* planes, const float* sx, int64_t n, const _Float16* image, const float* u,
                   const float* meta, int nch, int* labels) {
  using KC = H3Cfg<64, NPB>;
  const size_t lds = 2 * ((size_t)KC::CHUNK_H * 2 + KC::CB * 4);
  CHECK(hipFuncSetAttribute((const void*)h3_assign<64, NPB, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((h3_assign<64, NPB, EPI>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 10; ++w)
    hipLaunchKernelGGL((h3_assign<64, NPB, EPI>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int NPB, bool EPI, int MINB = 3>
float time_glds(const _Float16* planes, const float* sx, int64_t n, const _Float16* image, const float* u,
                const float* meta, int nch, int* labels) {
  using KC = H3Cfg<64, NPB>;
  const size_t lds = (size_t)KC::CHUNK_H * 2 + KC::CB * 4;
  const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((h3_assign_g<64, NPB, EPI, MINB>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 10; ++w)
    hipLaunchKernelGGL((h3_assign_g<64, NPB, EPI, MINB>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int NPB, int MINB = 2>
float time_pipe(const _Float16* planes, const float* sx, int64_t n, const _Float16* image, const float* u,
                const float* meta, int nch, int* labels) {
  using KC = H3Cfg<64, NPB>;
  const size_t lds = (size_t)KC::CHUNK_H * 2 + KC::CB * 4;
  const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((h3_assign_p<64, NPB, true, MINB>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 10; ++w)
    hipLaunchKernelGGL((h3_assign_p<64, NPB, true, MINB>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

int main() {
  const int64_t n = 12500000; const int f = 64, k = 1024;
  float *X, *C, *sx; _Float16* planes; int* labels; void* ws;
  CHECK(hipMalloc(&X, n * f * 4)); CHECK(hipMalloc(&C, k * f * 4)); CHECK(hipMalloc(&sx, n * 4));
  CHECK(hipMalloc(&planes, n * 128 * 2)); CHECK(hipMalloc(&labels, n * 4));
  CHECK(hipMalloc(&ws, ha_h3_workspace_bytes(k, f)));
  // pseudo-random data on the host (cheap LCG)
  float* h = (float*)malloc(n * f * 4);
  uint32_t st = 12345;
  for (int64_t i = 0; i < n * f; ++i) { st = st * 1664525u + 1013904223u; h[i] = ((st >> 8) * (1.f / 16777216.f)) - 0.5f; }
  CHECK(hipMemcpy(X, h, n * f * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(C, h + 777 * f, k * f * 4, hipMemcpyHostToDevice));
  CHECK((hipError_t)(ha_h3_pack_points(X, n, f, f, planes, sx, nullptr) == 0 ? hipSuccess : hipErrorUnknown));
  CHECK((hipError_t)(ha_h3_assign(planes, sx, n, f, C, k, f, ws, labels, nullptr, nullptr) == 0 ? hipSuccess : hipErrorUnknown));
  CHECK(hipDeviceSynchronize());
  const _Float16* image = (const _Float16*)ws;
  const float* u = (const float*)((char*)ws + (int64_t)1024 * 64 * 4);
  const float* meta = u + 1024;
  const int nch = 1024 / 128;
  const double flop = 2.0 * n * k * f;
  float t;
  t = time_variant<2, true>(planes, sx, n, image, u, meta, nch, labels);  printf("NPB2 full     %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_variant<2, false>(planes, sx, n, image, u, meta, nch, labels); printf("NPB2 mfma-only %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_variant<1, true>(planes, sx, n, image, u, meta, nch, labels);  printf("NPB1 full     %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_variant<4, true>(planes, sx, n, image, u, meta, nch, labels);  printf("NPB4 full     %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_variant<4, false>(planes, sx, n, image, u, meta, nch, labels); printf("NPB4 mfma-only %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  // correctness of the glds variant against the double-buffered one
  int* lab2; CHECK(hipMalloc(&lab2, n * 4));
  time_variant<2, true>(planes, sx, n, image, u, meta, nch, labels);
  time_pipe<2>(planes, sx, n, image, u, meta, nch, lab2);
  {
    int* h1 = (int*)malloc(n * 4); int* h2 = (int*)malloc(n * 4);
    CHECK(hipMemcpy(h1, labels, n * 4, hipMemcpyDeviceToHost)); CHECK(hipMemcpy(h2, lab2, n * 4, hipMemcpyDeviceToHost));
    int64_t diff = 0; for (int64_t i = 0; i < n; ++i) diff += h1[i] != h2[i];
    printf("pipelined labels differing: %lld\n", (long long)diff);
  }
  t = time_glds<2, true>(planes, sx, n, image, u, meta, nch, labels);  printf("GLDS NPB2 full     %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_glds<2, false>(planes, sx, n, image, u, meta, nch, labels); printf("GLDS NPB2 mfma-only %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_glds<1, true>(planes, sx, n, image, u, meta, nch, labels);  printf("GLDS NPB1 full     %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_glds<1, true, 4>(planes, sx, n, image, u, meta, nch, labels);  printf("GLDS NPB1 4wg full %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_glds<2, true, 2>(planes, sx, n, image, u, meta, nch, labels);  printf("GLDS NPB2 2wg full %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_pipe<2, 2>(planes, sx, n, image, u, meta, nch, labels);  printf("PIPE NPB2 2wg full %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_pipe<1, 3>(planes, sx, n, image, u, meta, nch, labels);  printf("PIPE NPB1 3wg full %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  t = time_pipe<1, 4>(planes, sx, n, image, u, meta, nch, labels);  printf("PIPE NPB1 4wg full %.3f ms  %.0f TF\n", t, flop / t / 1e9);
  return 0;
}
