// Host-side AddressSanitizer check of the native library's C ABI (sanitizer builds
// of the native extension). Built by tests/test_asan_host.py against an ASan-instrumented copy of
// the library (-fsanitize=address on the HOST code only: GPU ASan is not available here). Calls
// every host-only entry point (workspace / capacity calculators) over many shapes and the launch
// wrappers with arguments they must reject before touching the GPU, so ASan sees all host paths
// that run without a device. Prints "asan host check ok" and exits 0 on success.
#include <dlfcn.h>
#include <initializer_list>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

extern "C" {
int64_t ha_h3_amb_rows(int64_t n);
int ha_h3_amb_shards();
int ha_h3_fpad(int f);
int64_t ha_h3_workspace_bytes(int k, int f);
void ha_moments_rows_workspace(int64_t nrows, int nchunks, int64_t* part_doubles, int64_t* counters);
void ha_moments_cols_workspace(int64_t ncols, int nchunks, int64_t* part_doubles, int64_t* counters);
int64_t ha_lasso_prepare_scratch(int64_t m, int n);
int64_t ha_lasso_partial_floats(int num_cus);
int64_t ha_hh_part_len(int64_t m);
int ha_hh_counters();
int ha_hh_nb();
int ha_hh_slen();
int64_t ha_km_update_workspace(int64_t n, int k, int f, int num_cus);
int ha_km_workspace_floats(int k, int f, int* fpad_out, int* kpad_out);
int64_t ha_gemm_tiled_slices(int64_t K, int64_t slices);
int ha_moments_rows(const float* x, int64_t nrows, int64_t len, int64_t ld, int nchunks, double* part, void* out,
                    int kind, double ddof, unsigned* cnt, void* stream);
int ha_moments_cols(const float* x, int64_t len, int64_t ncols, int64_t ld, int nchunks, double* part, void* out,
                    int kind, double ddof, unsigned* cnt, void* stream);
int ha_gemm_f32t(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                 int64_t ldc, int a_kmajor, int b_kmajor, float alpha, int beta, int upper, int64_t slices,
                 int64_t cslice, void* stream);
int ha_gemm_h3t(const void* Ahi, const void* Alo, const void* Bhi, const void* Blo, const int* eA, const int* eB,
                float* C, int64_t M, int64_t N, int64_t Kp, int64_t Mp, int64_t Np, int64_t ldc, float alpha, int beta,
                int upper, int64_t slices, int64_t cslice, void* stream);
int ha_hh_colsums(const void* A, int dtype, int64_t m, int64_t lda, int64_t g0, int64_t k0, int ncols, int64_t d,
                  double* S, double* part, unsigned* cnt, void* stream);
int ha_hh_step(void* A, int dtype, int64_t m, int64_t lda, int64_t g0, int64_t k0, int64_t coff, int ncols, int j,
               const double* Sin, double* Sout, void* tau, double* Y, double* part, unsigned* cnt, void* stream);
int ha_threefry_fill(void* out, int64_t e0, int64_t n, uint64_t counter_lo, uint64_t counter_hi, uint64_t seed,
                     int bits, int dist, double low, double span, void* stream);
int ha_knn_rescore(const float* Q, int64_t ldq, const float* T, int64_t ldt, int64_t nt, int64_t nq, int f,
                   const void* cand, int idx64, int c, int k, float* dist, int64_t* out_idx, void* stream);
}

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "check failed line %d: %s\n", __LINE__, #c); \
      ++fails;                                                    \
    }                                                             \
  } while (0)

int main() {
  enum { OK = 0, BAD = 1, UNSUP = 2 };
  const int64_t sizes[] = {0, 1, 3, 255, 256, 257, 4096, 12500000, 100000007};
  for (int64_t n : sizes) {
    const int64_t r = ha_h3_amb_rows(n);
    CHECK(r >= n && r % ha_h3_amb_shards() == 0);
    CHECK(ha_hh_part_len(n > 0 ? n : 1) % ha_hh_nb() == 0);
    for (int k : {1, 7, 64, 1024})
      for (int f : {3, 16, 64})
        if (n < ((int64_t)1 << 31)) CHECK(ha_km_update_workspace(n, k, f, 256) >= 0);
  }
  for (int nchunks : {1, 2, 17, 4096, 65536}) {
    int64_t pd = -1, nc = -1;
    ha_moments_rows_workspace(5, nchunks, &pd, &nc);
    CHECK(pd >= 15 && nc >= 0);
    ha_moments_cols_workspace(1000, nchunks, &pd, &nc);
    CHECK(pd >= 3000 && nc >= 4);
  }
  for (int f : {1, 16, 17, 64, 100, 128, 129}) {
    const int fp = ha_h3_fpad(f);
    CHECK(fp == -1 || fp >= f);
    if (fp > 0) CHECK(ha_h3_workspace_bytes(1024, f) > 0);
    int fpad = 0, kpad = 0;
    const int w = ha_km_workspace_floats(1000, f, &fpad, &kpad);
    CHECK(w < 0 || (fpad >= f && kpad >= 1000));
  }
  for (int64_t m : {1, 1000, 10000000}) CHECK(ha_lasso_prepare_scratch(m, 16) >= 16);
  CHECK(ha_lasso_partial_floats(256) >= 4 + 1024);
  CHECK(ha_hh_slen() == ha_hh_counters() * 2 * ha_hh_nb());
  for (int64_t K : {1, 16, 17, 4096, 1250000})
    for (int64_t s : {1, 2, 7, 1000}) {
      const int64_t t = ha_gemm_tiled_slices(K, s);
      CHECK(t >= 1 && t <= s);
    }
  // launch wrappers: invalid arguments are rejected before any device work
  float dummy[16] = {0};
  CHECK(ha_moments_rows(dummy, 4, 100, 100, 0, nullptr, nullptr, 1, 0.0, nullptr, nullptr) == BAD);
  CHECK(ha_moments_rows(dummy, 4, 100, 100, 70000, nullptr, nullptr, 1, 0.0, nullptr, nullptr) == BAD);
  CHECK(ha_moments_rows(dummy, 4, 100, 100, 8, (double*)dummy, dummy, 1, 0.0, nullptr, nullptr) == BAD);
  CHECK(ha_moments_rows(dummy, 0, 100, 100, 8, nullptr, nullptr, 1, 0.0, nullptr, nullptr) == OK);
  CHECK(ha_moments_cols(dummy, 100, 4, 4, 0, nullptr, nullptr, 1, 0.0, nullptr, nullptr) == BAD);
  CHECK(ha_moments_cols(dummy, 100, 0, 4, 4, nullptr, nullptr, 1, 0.0, nullptr, nullptr) == OK);
  CHECK(ha_gemm_f32t(dummy, dummy, dummy, -1, 4, 4, 4, 4, 4, 0, 0, 1.f, 0, 0, 1, 0, nullptr) == BAD);
  CHECK(ha_gemm_f32t(dummy, dummy, dummy, 8, 4, 4, 4, 4, 4, 0, 0, 1.f, 0, 1, 1, 0, nullptr) == BAD);  // upper, M != N
  CHECK(ha_gemm_f32t(dummy, dummy, dummy, 0, 4, 4, 4, 4, 4, 0, 0, 1.f, 0, 0, 1, 0, nullptr) == OK);
  CHECK(ha_gemm_f32t(dummy, dummy, dummy, 4, 4, 2, 4, 4, 4, 0, 0, 1.f, 0, 0, 1, 0, nullptr) == UNSUP);  // K < 4
  CHECK(ha_gemm_h3t(dummy, dummy, dummy, dummy, nullptr, nullptr, dummy, 10, 10, 15, 256, 256, 10, 1.f, 0, 0, 1, 0,
                    nullptr) == BAD);  // Kp % 16
  CHECK(ha_gemm_h3t(dummy, dummy, dummy, dummy, nullptr, nullptr, dummy, 300, 10, 16, 256, 256, 10, 1.f, 0, 0, 1, 0,
                    nullptr) == BAD);  // Mp < M
  CHECK(ha_hh_colsums(dummy, 0, 10, 4, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr) == BAD);
  CHECK(ha_hh_colsums(dummy, 0, 10, 4, 0, 0, 99, 0, nullptr, nullptr, nullptr, nullptr) == BAD);
  CHECK(ha_hh_step(dummy, 0, 10, 4, 0, 0, 0, 4, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) ==
        BAD);  // j >= ncols
  CHECK(ha_hh_step(dummy, 0, 10, 4, 0, 0, -1, 4, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) ==
        BAD);  // coff < 0
  CHECK(ha_threefry_fill(dummy, 0, 0, 0, 0, 1, 32, 0, 0.0, 1.0, nullptr) == OK);
  CHECK(ha_threefry_fill(dummy, 0, 4, 0, 0, 1, 16, 0, 0.0, 1.0, nullptr) == BAD);
  CHECK(ha_knn_rescore(nullptr, 4, nullptr, 4, 10, 5, 4, nullptr, 0, 33, 8, nullptr, nullptr, nullptr) == BAD);  // c > 32
  CHECK(ha_knn_rescore(nullptr, 4, nullptr, 4, 10, 5, 4, nullptr, 0, 16, 17, nullptr, nullptr, nullptr) == BAD);  // k > c
  CHECK(ha_knn_rescore(nullptr, 2, nullptr, 4, 10, 5, 4, nullptr, 0, 16, 8, nullptr, nullptr, nullptr) == BAD);  // ldq < f
  CHECK(ha_knn_rescore(nullptr, 4, nullptr, 4, 10, 0, 4, nullptr, 0, 16, 8, nullptr, nullptr, nullptr) == OK);   // nq = 0
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("asan host check ok\n");
  return 0;
}
