// Microbenchmark: counting-sort based k-means update vs LDS-atomic update.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// K1: per-block histograms hist[b][k] (LDS int atomics)
__global__ __launch_bounds__(1024) void k_hist(const int* __restrict__ lab, long n, int k, long rows_per_blk,
                                               int* __restrict__ hist) {
  extern __shared__ int h[];
  for (int e = threadIdx.x; e < k; e += 1024) h[e] = 0;
  __syncthreads();
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(n, r0 + rows_per_blk);
  for (long i = r0 + threadIdx.x; i < r1; i += 1024) atomicAdd(&h[lab[i]], 1);
  __syncthreads();
  for (int e = threadIdx.x; e < k; e += 1024) hist[(long)blockIdx.x * k + e] = h[e];
}

// K2a: per cluster exclusive prefix over blocks (in place) + totals
__global__ void k_scan_blocks(int* __restrict__ hist, int nblk, int k, int* __restrict__ total) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= k) return;
  int run = 0;
  for (int b = 0; b < nblk; ++b) {
    const int v = hist[(long)b * k + c];
    hist[(long)b * k + c] = run;
    run += v;
  }
  total[c] = run;
}

// K2b: exclusive scan of totals (one block of 1024 threads, k <= 1024*ITEMS)
__global__ __launch_bounds__(1024) void k_scan_total(const int* __restrict__ total, int k, int* __restrict__ cstart) {
  __shared__ int s[1024];
  const int per = (k + 1023) / 1024;
  const int t = threadIdx.x;
  int loc = 0;
  for (int j = 0; j < per; ++j) { int c = t * per + j; if (c < k) loc += total[c]; }
  s[t] = loc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int v = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  int run = s[t] - loc;
  for (int j = 0; j < per; ++j) { int c = t * per + j; if (c < k) { cstart[c] = run; run += total[c]; } }
  if (t == 1023) cstart[k] = s[1023];
}

// K3: scatter row ids into cluster order
__global__ __launch_bounds__(1024) void k_scatter(const int* __restrict__ lab, long n, int k, long rows_per_blk,
                                                  const int* __restrict__ hist, const int* __restrict__ cstart,
                                                  int* __restrict__ order) {
  extern __shared__ int h[];
  for (int e = threadIdx.x; e < k; e += 1024) h[e] = cstart[e] + hist[(long)blockIdx.x * k + e];
  __syncthreads();
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(n, r0 + rows_per_blk);
  for (long i = r0 + threadIdx.x; i < r1; i += 1024) {
    const int p = atomicAdd(&h[lab[i]], 1);
    order[p] = (int)i;
  }
}

// K4: gather-reduce. WG of 256 threads: FW = 64 columns x 4 row lanes; chunk of CH positions.
constexpr int CH = 2048;
constexpr int RU = 8;
__global__ __launch_bounds__(256) void k_gather(const float* __restrict__ X, int f, long ldx,
                                                const int* __restrict__ order, const int* __restrict__ cstart, int k,
                                                long n, float* __restrict__ sums) {
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const long p0 = (long)blockIdx.x * CH;
  const long p1 = min(n, p0 + CH);
  // first cluster with cstart[cl+1] > p
  long p = p0 + rl;
  if (p >= p1) return;
  int lo = 0, hi = k - 1;
  while (lo < hi) { int mid = (lo + hi) >> 1; if (cstart[mid + 1] > p) hi = mid; else lo = mid + 1; }
  int cur = lo;
  int nextb = cstart[cur + 1];
  for (int cb = 0; cb < f; cb += 64) {
    const int col = cb + c;
    const bool ok = col < f;
    int curc = cur, nb = nextb;
    float acc = 0.f;
    long q = p;
    for (; q + (RU - 1) * 4 < p1; q += RU * 4) {
      int idx[RU];
      float v[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) idx[u] = order[q + u * 4];
#pragma unroll
      for (int u = 0; u < RU; ++u) v[u] = ok ? X[(long)idx[u] * ldx + col] : 0.f;
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const long qq = q + u * 4;
        while (qq >= nb) {
          if (ok && acc != 0.f) atomicAdd(&sums[(long)curc * f + col], acc);
          acc = 0.f;
          ++curc;
          nb = cstart[curc + 1];
        }
        acc += v[u];
      }
    }
    for (; q < p1; q += 4) {
      const float v = ok ? X[(long)order[q] * ldx + col] : 0.f;
      while (q >= nb) {
        if (ok && acc != 0.f) atomicAdd(&sums[(long)curc * f + col], acc);
        acc = 0.f;
        ++curc;
        nb = cstart[curc + 1];
      }
      acc += v;
    }
    if (ok && acc != 0.f) atomicAdd(&sums[(long)curc * f + col], acc);
  }
}

int main() {
  const long n = 12500000; const int f = 64, k = 1024;
  float *X, *sums; int *lab, *hist, *total, *cstart, *order;
  const int nblk = 1024;
  const long rpb = (n + nblk - 1) / nblk;
  CHECK(hipMalloc(&X, n * f * 4)); CHECK(hipMalloc(&lab, n * 4)); CHECK(hipMalloc(&order, n * 4));
  CHECK(hipMalloc(&hist, (long)nblk * k * 4)); CHECK(hipMalloc(&total, k * 4)); CHECK(hipMalloc(&cstart, (k + 1) * 4));
  CHECK(hipMalloc(&sums, (long)k * f * 4));
  std::vector<int> h(n);
  std::vector<float> hx(n * f);
  srand(1);
  for (long i = 0; i < n; ++i) h[i] = rand() % k;
  for (long i = 0; i < n * f; ++i) hx[i] = (float)((rand() % 2001) - 1000) / 1000.f;
  CHECK(hipMemcpy(lab, h.data(), n * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(X, hx.data(), n * f * 4, hipMemcpyHostToDevice));
  auto pipeline = [&]() {
    hipMemsetAsync(sums, 0, (long)k * f * 4, 0);
    hipLaunchKernelGGL(k_hist, dim3(nblk), dim3(1024), k * 4, 0, lab, n, k, rpb, hist);
    hipLaunchKernelGGL(k_scan_blocks, dim3((k + 255) / 256), dim3(256), 0, 0, hist, nblk, k, total);
    hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1024), 0, 0, total, k, cstart);
    hipLaunchKernelGGL(k_scatter, dim3(nblk), dim3(1024), k * 4, 0, lab, n, k, rpb, hist, cstart, order);
    hipLaunchKernelGGL(k_gather, dim3((n + CH - 1) / CH), dim3(256), 0, 0, X, f, (long)f, order, cstart, k, n, sums);
  };
  pipeline();
  CHECK(hipDeviceSynchronize());
  std::vector<float> gs(k * f);
  CHECK(hipMemcpy(gs.data(), sums, k * f * 4, hipMemcpyDeviceToHost));
  std::vector<double> ref(k * f, 0.0);
  for (long i = 0; i < n; ++i) for (int j = 0; j < f; ++j) ref[h[i] * f + j] += hx[i * f + j];
  double maxerr = 0;
  for (int e = 0; e < k * f; ++e) maxerr = fmax(maxerr, fabs(ref[e] - gs[e]));
  printf("max abs err %.3e\n", maxerr);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int stage : {0, 1, 5}) {
    if (stage == 5) pipeline();
    CHECK(hipEventRecord(a));
    for (int w = 0; w < 10; ++w) {
      if (stage == 0) pipeline();
      // stages 2-4 rewrite hist in place: re-running them alone would scatter out of bounds
      if (stage == 1) hipLaunchKernelGGL(k_hist, dim3(nblk), dim3(1024), k * 4, 0, lab, n, k, rpb, hist);
      if (stage == 5) hipLaunchKernelGGL(k_gather, dim3((n + CH - 1) / CH), dim3(256), 0, 0, X, f, (long)f, order, cstart, k, n, sums);
    }
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    const char* names[] = {"pipeline", "hist", "scan_blocks", "scan_total", "scatter", "gather"};
    printf("%-12s %.3f ms\n", names[stage], ms / 10);
  }
  return 0;
}
