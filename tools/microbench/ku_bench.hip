// Microbenchmark: k-means update (per-cluster sums) variants on MI355X.
// hipcc --offload-arch=gfx950 -O3 -o ku_bench ku_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int T = 1024;
constexpr int U = 8;

// MODE 0: LDS atomics (current); 1: plain LDS stores; 2: register sum only; 3: LDS atomics on a
// per-wave-offset layout (k-major with +1 padding)
template <int FC, int MODE>
__global__ __launch_bounds__(T) void ku(const float* __restrict__ X, long n, int f, const int* __restrict__ labels,
                                        int k, long rows_per_wg, float* __restrict__ out) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  for (int e = tid; e < k * FC + k; e += T) lds[e] = 0.f;
  __syncthreads();
  const int c0 = blockIdx.y * FC;
  const long r0 = (long)blockIdx.x * rows_per_wg;
  const long r1 = r0 + rows_per_wg < n ? r0 + rows_per_wg : n;
  constexpr int RP = T / FC;
  const int c = tid % FC, rs = tid / FC;
  float acc = 0.f;
  long i = r0 + rs;
  for (; i + (U - 1) * RP < r1; i += U * RP) {
    int lab[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lab[u] = labels[i + u * RP];
      v[u] = X[(i + u * RP) * f + c0 + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE == 0) atomicAdd(&lds[lab[u] * FC + c], v[u]);
      else if (MODE == 1) lds[lab[u] * FC + c] = v[u];
      else if (MODE == 2) acc += v[u] * (float)lab[u];
    }
  }
  __syncthreads();
  float s = acc;
  for (int e = tid; e < k * FC; e += T) s += lds[e];
  out[(blockIdx.y * gridDim.x + blockIdx.x) * T + tid] = s;
}

// MODE 4: float4 loads, 8 lanes per 32-col half row, 4 LDS atomics per lane
template <int FC>
__global__ __launch_bounds__(T) void ku4(const float* __restrict__ X, long n, int f, const int* __restrict__ labels,
                                         int k, long rows_per_wg, float* __restrict__ out) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  for (int e = tid; e < k * FC + k; e += T) lds[e] = 0.f;
  __syncthreads();
  const int c0 = blockIdx.y * FC;
  const long r0 = (long)blockIdx.x * rows_per_wg;
  const long r1 = r0 + rows_per_wg < n ? r0 + rows_per_wg : n;
  constexpr int LPR = FC / 4;   // lanes per row
  constexpr int RP = T / LPR;
  const int c = (tid % LPR) * 4, rs = tid / LPR;
  long i = r0 + rs;
  for (; i + (U - 1) * RP < r1; i += U * RP) {
    int lab[U];
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lab[u] = labels[i + u * RP];
      v[u] = *(const float4*)&X[(i + u * RP) * f + c0 + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float* p = &lds[lab[u] * FC + c];
      atomicAdd(p + 0, v[u].x);
      atomicAdd(p + 1, v[u].y);
      atomicAdd(p + 2, v[u].z);
      atomicAdd(p + 3, v[u].w);
    }
  }
  __syncthreads();
  float s = 0.f;
  for (int e = tid; e < k * FC; e += T) s += lds[e];
  out[(blockIdx.y * gridDim.x + blockIdx.x) * T + tid] = s;
}

template <typename K>
float run(K kern, int fc, const float* X, long n, int f, const int* lab, int k, float* out, int wgs_per_cb) {
  int ncb = f / fc;
  size_t lds = ((size_t)k * fc + k) * 4;
  CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long rows = (n + wgs_per_cb - 1) / wgs_per_cb;
  dim3 grid(wgs_per_cb, ncb);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, grid, dim3(T), lds, 0, X, n, f, lab, k, rows, out);
  CHECK(hipEventRecord(a));
  for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kern, grid, dim3(T), lds, 0, X, n, f, lab, k, rows, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return ms / 5;
}

int main() {
  const long n = 12500000; const int f = 64, k = 1024;
  float* X; int* lab; float* out;
  CHECK(hipMalloc(&X, n * f * 4)); CHECK(hipMalloc(&lab, n * 4)); CHECK(hipMalloc(&out, 64L * 1024 * 1024 * 4));
  std::vector<int> h(n);
  srand(1);
  for (long i = 0; i < n; ++i) h[i] = rand() % k;
  CHECK(hipMemcpy(lab, h.data(), n * 4, hipMemcpyHostToDevice));
  CHECK(hipMemset(X, 0, n * f * 4));
  double gb = n * f * 4 / 1e9;
  for (int wg : {128, 256, 512}) {
    float t;
    t = run(ku<32, 0>, 32, X, n, f, lab, k, out, wg); printf("wg/cb %d  FC32 atomics      %.3f ms  %.0f GB/s\n", wg, t, gb / t * 1e3);
    t = run(ku<32, 1>, 32, X, n, f, lab, k, out, wg); printf("wg/cb %d  FC32 lds stores   %.3f ms  %.0f GB/s\n", wg, t, gb / t * 1e3);
    t = run(ku<32, 2>, 32, X, n, f, lab, k, out, wg); printf("wg/cb %d  FC32 regs only    %.3f ms  %.0f GB/s\n", wg, t, gb / t * 1e3);
    t = run(ku<16, 0>, 16, X, n, f, lab, k, out, wg); printf("wg/cb %d  FC16 atomics      %.3f ms  %.0f GB/s\n", wg, t, gb / t * 1e3);
    t = run(ku4<32>, 32, X, n, f, lab, k, out, wg); printf("wg/cb %d  FC32 float4 atom  %.3f ms  %.0f GB/s\n", wg, t, gb / t * 1e3);
  }
  // skewed labels: everything in 8 clusters
  for (long i = 0; i < n; ++i) h[i] = rand() % 8;
  CHECK(hipMemcpy(lab, h.data(), n * 4, hipMemcpyHostToDevice));
  float t = run(ku<32, 0>, 32, X, n, f, lab, k, out, 128); printf("skew8 FC32 atomics %.3f ms\n", t);
  for (long i = 0; i < n; ++i) h[i] = 0;
  CHECK(hipMemcpy(lab, h.data(), n * 4, hipMemcpyHostToDevice));
  t = run(ku<32, 0>, 32, X, n, f, lab, k, out, 128); printf("all-one-label FC32 atomics %.3f ms\n", t);
  return 0;
}
