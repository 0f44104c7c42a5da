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

// write-bandwidth references: a sequential 16-byte non-temporal fill of the same bytes, and the
// same bytes written in cdist_p's pattern (128 x 128 tiles, 8 rows x 128 B per store instruction)
__global__ __launch_bounds__(256) void fill_seq(floatx4* C, int64_t n4) {
  const floatx4 v = {1.f, 2.f, 3.f, 4.f};
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    __builtin_nontemporal_store(v, C + i);
}
__global__ __launch_bounds__(256) void fill_tiles(float* C, int64_t n, int run) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31, t = j & 3;
  const int64_t panels = n / 128, tiles_n = n / 128, runs = (tiles_n + run - 1) / run;
  const int64_t total = panels * runs, per_xcd = (total + 7) / 8, b = blockIdx.x;
  const int64_t tt = (b % 8) * per_xcd + b / 8;
  if (tt >= total) return;
  const int64_t rp = tt % panels, cr = tt / panels, row0 = rp * 128;
  const floatx4 v = {1.f, 2.f, 3.f, 4.f};
  for (int64_t c = cr * run; c < (cr + 1) * run && c < tiles_n; ++c) {
    float* p = C + (row0 + 4 * h + t) * n + c * 128 + wave * 32 + (j >> 2) * 4;
    for (int k = 0; k < 16; ++k) __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p + (int64_t)8 * k * n));
  }
}

void run_fill(float* C, int64_t n) {
  const double gb = n * n * 4 / 1e9;
  float t = timeit([&] { hipLaunchKernelGGL(fill_seq, dim3(256 * 8), dim3(256), 0, 0, (floatx4*)C, n * n / 4); });
  printf("fill sequential     %.3f ms  %5.0f GB/s\n", t, gb / t * 1e3);
  const int run = cdist_run(n, n);
  const int64_t per_xcd = ((n / TM) * ((n / TN + run - 1) / run) + 7) / 8;
  t = timeit([&] { hipLaunchKernelGGL(fill_tiles, dim3((unsigned)(per_xcd * 8)), dim3(256), 0, 0, C, n, run); });
  printf("fill cdist pattern  %.3f ms  %5.0f GB/s\n", t, gb / t * 1e3);
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
    if (f == 128) run_fill(C, n);
    CHECK(hipFree(X)); CHECK(hipFree(C)); CHECK(hipFree(P)); CHECK(hipFree(A)); free(h);
  }
  return 0;
}
