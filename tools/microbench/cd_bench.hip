// Timing of the fp16x3 cdist kernels on one 65536 x 65536 tile (f = 128, 64, 18): the panel-resident
// cdist_p (production for fpad <= 128), the LDS-staged cdist_t (production for larger fpad) and
// cdist_p without output stores (ablation). Sampled outputs are checked against fp64 on the host.
#include "../../heat_amd/ops/csrc/cdist_f16x3.hip"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <typename F>
float timeit(F&& launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) launch();
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 5; ++w) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 5;
}

static double check(const float* C, const float* h, int64_t n, int f) {
  double worst = 0;
  for (int i = 0; i < 2048; ++i) {
    const int64_t r = (int64_t)i * 7919 % n, c = (int64_t)i * 104729 % n;
    float v; CHECK(hipMemcpy(&v, C + r * n + c, 4, hipMemcpyDeviceToHost));
    double d = 0;
    for (int k = 0; k < f; ++k) { const double t = (double)h[r * f + k] - h[c * f + k]; d += t * t; }
    worst = fmax(worst, fabs(v - sqrt(d)) / (1.0 + sqrt(d)));
  }
  return worst;
}

template <int KS>
void run_p(const _Float16* P, const float2* A, int64_t n, float* C, const float* h, int f) {
  const double gb = n * n * 4 / 1e9, tf = 2.0 * n * n * f * 3 / 1e12;
  CHECK(hipMemset(C, 0, n * n * 4));
  float t = timeit([&] { launch_p<0, KS>(P, A, n, P, A, n, C, n, 1.f, 0); });
  printf("f=%d cdist_p          %.3f ms  %5.0f GB/s out  %4.0f TF fp16  relerr %.1e\n", f, t, gb / t * 1e3,
         tf / t * 1e3, check(C, h, n, f));
  const int run = cdist_run(n, n);
  const int64_t per_xcd = ((n / TM) * ((n / TN + run - 1) / run) + 7) / 8;
  const size_t lds = 4 * KS * 2 * FRAG_H * 2 + 256 * 4;
  CHECK(hipFuncSetAttribute((const void*)cdist_p<0, KS, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  t = timeit([&] {
    hipLaunchKernelGGL((cdist_p<0, KS, 1>), dim3((unsigned)(per_xcd * 8)), dim3(256), lds, 0, P, A, n, P, A, n, C, n,
                       1.f, run);
  });
  printf("f=%d cdist_p no-store %.3f ms  %4.0f TF fp16\n", f, t, tf / t * 1e3);
}

int main() {
  const int64_t n = 65536;
  for (int f : {128, 64, 18}) {
    float *X, *C; _Float16* P; float2* A;
    const int fpad = ha_cdist_h3_fpad(f);
    CHECK(hipMalloc(&X, n * f * 4)); CHECK(hipMalloc(&C, n * n * 4));
    CHECK(hipMalloc(&P, n * 2 * fpad * 2)); CHECK(hipMalloc(&A, n * 8));
    float* h = (float*)malloc(n * f * 4);
    uint32_t st = 7;
    for (int64_t i = 0; i < n * f; ++i) { st = st * 1664525u + 1013904223u; h[i] = (st >> 8) * (1.f / 16777216.f); }
    CHECK(hipMemcpy(X, h, n * f * 4, hipMemcpyHostToDevice));
    if (ha_cdist_h3_pack(X, n, f, f, P, A, nullptr) != 0) { printf("pack failed\n"); return 1; }
    CHECK(hipDeviceSynchronize());
    const double gb = n * n * 4 / 1e9;
    CHECK(hipMemset(C, 0, n * n * 4));
    float t = timeit([&] { launch_t<0>(P, A, n, P, A, n, fpad, C, n, 1.f, 0); });
    printf("f=%d cdist_t          %.3f ms  %5.0f GB/s out  relerr %.1e\n", f, t, gb / t * 1e3, check(C, h, n, f));
    if (fpad == 128) run_p<8>(P, A, n, C, h, f);
    if (fpad == 64) run_p<4>(P, A, n, C, h, f);
    if (fpad == 32) run_p<2>(P, A, n, C, h, f);
    CHECK(hipFree(X)); CHECK(hipFree(C)); CHECK(hipFree(P)); CHECK(hipFree(A)); free(h);
  }
  return 0;
}
