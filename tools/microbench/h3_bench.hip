// Timing of fp16x3 k-means assign configurations (NPB point blocks per wave, workgroups per CU)
// at k=1024: f=64 (n=12.5M) and f=100 (padded to 128, n=6.25M).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../heat_amd/ops/csrc -o h3_bench h3_bench.hip
#include "../../heat_amd/ops/csrc/kmeans_f16x3.hip"
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int NPB, int MINB = 2, int FP = 64>
float time_pipe(const _Float16* planes, const float* sx, int64_t n, const _Float16* image, const float* u,
                const float* meta, int nch, int* labels) {
  using KC = H3Cfg<FP, NPB>;
  const size_t lds = (size_t)KC::CHUNK_H * 2 + KC::CB * 4;
  const unsigned blocks = (unsigned)((n + KC::PTS_PER_WG - 1) / KC::PTS_PER_WG);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((h3_assign_p<FP, NPB, true, MINB>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 10; ++w)
    hipLaunchKernelGGL((h3_assign_p<FP, NPB, true, MINB>), dim3(blocks), dim3(256), lds, 0, planes, sx, n, image, u, meta, nch, labels, (float*)nullptr);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int FP>
void suite(int f) {
  const int64_t n = 12500000 / (FP / 64 > 0 ? FP / 64 : 1); const int k = 1024;
  float *X, *C, *sx; _Float16* planes; int *labels, *lab2; void* ws;
  CHECK(hipMalloc(&X, n * f * 4)); CHECK(hipMalloc(&C, k * f * 4)); CHECK(hipMalloc(&sx, n * 4));
  CHECK(hipMalloc(&planes, n * 2 * FP * 2)); CHECK(hipMalloc(&labels, n * 4)); CHECK(hipMalloc(&lab2, n * 4));
  CHECK(hipMalloc(&ws, ha_h3_workspace_bytes(k, f)));
  float* h = (float*)malloc(n * f * 4);
  uint32_t st = 12345;
  for (int64_t i = 0; i < n * f; ++i) { st = st * 1664525u + 1013904223u; h[i] = ((st >> 8) * (1.f / 16777216.f)) - 0.5f; }
  CHECK(hipMemcpy(X, h, n * f * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(C, h + 777 * f, k * f * 4, hipMemcpyHostToDevice));
  CHECK((hipError_t)(ha_h3_pack_points(X, n, f, f, planes, sx, nullptr) == 0 ? hipSuccess : hipErrorUnknown));
  CHECK((hipError_t)(ha_h3_assign(planes, sx, n, f, C, k, f, ws, labels, nullptr, nullptr) == 0 ? hipSuccess : hipErrorUnknown));
  CHECK(hipDeviceSynchronize());
  using KC = H3Cfg<FP>;
  const _Float16* image = (const _Float16*)ws;
  const float* u = (const float*)((char*)ws + (int64_t)1024 * FP * 4);
  const float* meta = u + 1024;
  const int nch = 1024 / KC::CB;
  const double flop = 2.0 * n * k * f;
  int* h1 = (int*)malloc(n * 4); int* h2 = (int*)malloc(n * 4);
  CHECK(hipMemcpy(h1, labels, n * 4, hipMemcpyDeviceToHost));
  auto cmp = [&](const char* name, float t) {
    CHECK(hipMemcpy(h2, lab2, n * 4, hipMemcpyDeviceToHost));
    int64_t diff = 0; for (int64_t i = 0; i < n; ++i) diff += h1[i] != h2[i];
    printf("f=%d n=%lld %-16s %.3f ms  %.0f TF (fp32-equivalent)  labels differing from ha_h3_assign: %lld\n", f,
           (long long)n, name, t, flop / t / 1e9, (long long)diff);
  };
  cmp("NPB2 2wg", time_pipe<2, 2, FP>(planes, sx, n, image, u, meta, nch, lab2));
  cmp("NPB1 3wg", time_pipe<1, 3, FP>(planes, sx, n, image, u, meta, nch, lab2));
  cmp("NPB1 4wg", time_pipe<1, 4, FP>(planes, sx, n, image, u, meta, nch, lab2));
  CHECK(hipFree(X)); CHECK(hipFree(C)); CHECK(hipFree(sx)); CHECK(hipFree(planes)); CHECK(hipFree(labels));
  CHECK(hipFree(lab2)); CHECK(hipFree(ws)); free(h); free(h1); free(h2);
}

int main() {
  suite<64>(64);
  suite<128>(100);
  return 0;
}
