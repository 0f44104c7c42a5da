"""Short, fixed workloads for rocprofv3 --pmc passes (one pass per counter group, see
tools/gpu_pmc_r03.sh): the hot kernels of the benchmark configs, each warmed up and run 3 times.
  kmeans  - 8 Lloyd steps, k = 1024, 1.25e7 x 64 (h3_assign_p + deterministic update)
  moments - mean of 1e9 fp32, axis None / 0 / 1 (moments.hip, one kernel per call)
  gemm    - ht.matmul 8192^3 fp32 at precision highest (gemm_f32t) and high (gemm_h3t)
  cdist   - one 32768 x 32768 x 128 distance tile (cdist_f16x3.hip)
  topk    - 8 nearest of 65536 x 128 queries among 1e6 points (spatial.cdist_topk -> h3_topk)
  knn     - the bench.py knn step: 8 nearest of all 1e6 x 128 rows among themselves (certified h1_topk)
  randn   - 8e8 standard normals and 8e8 uniforms, fp32 (threefry.hip: tf_fill32, 3.2 GB each)
  smallk  - 10 fused small-k passes, k = 8, 1.25e7 x 64 (kmeans_smallk.hip: ks_step64, the reference protocol)
  cdist_exact - exact (difference) cdist, SUSY size 40k x 18, 3 calls (cdist.hip: cdist_vx)
  gemm_small - 1024^3 and 2048^3 exact fp32 through fgemm's plan (gemm_small.hip / gemm_tiled.hip split-K)
  gemm_f32s_big - gemm_f32s alone at 6144^3 and 8192^3 (one K slice)
  gram    - ht.matmul(A.T, A) at 400000 x 2048 (upper-triangle Gram tiles + fp64 slice sums)
  tri     - CholeskyQR2's A R^-1 at 1.25e6 x 4096 (upper-triangular B: K clipped per column tile),
            2 calls, then the same product as a full GEMM, 1 call
  libvsmid - 6144^3 exact fp32: hipBLASLt (torch.mm at precision highest) and gemm_f32m 128-tile, 2 calls each
  mid     - the LDS-DMA 128-tile gemm_f32m: 3072^3 (3 K slices), 6144^3 (1 slice) and the
            Householder update C[4e5, 3840] -= V[4e5, 256] X[256, 3840], 2 calls each"""
import sys

import torch

import heat_amd as ht
from heat_amd import ops


def main():
    which = sys.argv[1]
    ht.use_device("gpu")
    ht.random.seed(11)
    if which == "kmeans":
        x = ht.random.randn(12_500_000, 64, split=0)
        km = ht.cluster.KMeans(n_clusters=1024, init="random", max_iter=1, tol=None, random_state=3)
        for _ in range(8):  # the first steps probe the certified filter, then the full kernel runs
            km.step(x)
    elif which == "moments":
        x = ht.random.rand(1_000_000, 1000, split=0)
        for axis in (None, 0, 1):
            for _ in range(3):
                ht.mean(x, axis=axis)
    elif which == "gemm":
        a = torch.randn(8192, 8192, device="cuda")
        b = torch.randn(8192, 8192, device="cuda")
        A, B = ht.array(a, split=0), ht.array(b)
        for prec in ("highest", "high"):
            torch.set_float32_matmul_precision(prec)
            for _ in range(3):
                ht.matmul(A, B)
    elif which == "cdist":
        x = torch.rand(32768, 128, device="cuda")
        for _ in range(3):
            ops.cdist(x, x)
    elif which == "topk":
        q = ht.random.rand(65536, 128, split=0)
        y = ht.random.rand(1_000_000, 128, split=0)
        for _ in range(3):
            ht.spatial.cdist_topk(q, y, 8)
    elif which == "knn":
        x = ht.random.rand(1_000_000, 128, split=0)
        ht.spatial.cdist_topk(x, x, 8)
    elif which == "libvsmid":
        torch.set_float32_matmul_precision("highest")
        a = torch.randn(6144, 6144, device="cuda")
        b = torch.randn(6144, 6144, device="cuda")
        for _ in range(2):
            torch.mm(a, b)
        for _ in range(2):
            ops.gemm_f32_small(a, b, slices=1, kernel="mid128")
    elif which == "mid":
        torch.set_float32_matmul_precision("highest")
        for n, sl in ((3072, 3), (6144, 1)):
            a = torch.randn(n, n, device="cuda")
            b = torch.randn(n, n, device="cuda")
            for _ in range(2):
                ops.gemm_f32_small(a, b, slices=sl, kernel="mid256")
        A = torch.randn(400_000, 4096, device="cuda")
        V = torch.randn(400_000, 256, device="cuda")
        X = torch.randn(256, 3840, device="cuda") * 1e-3
        for _ in range(2):
            ops.gemm_f32_small(V, X, out=A[:, 256:], alpha=-1.0, accumulate=True, kernel="mid256")
    elif which == "tri":
        a = torch.randn(1_250_000, 4096, device="cuda")
        r = torch.triu(torch.randn(4096, 4096, device="cuda")) + 4 * torch.eye(4096, device="cuda")
        for _ in range(2):
            ops.gemm_f32(a, r, b_upper=True)
        ops.gemm_f32(a, r)
    elif which == "randn":
        for _ in range(3):
            ht.random.randn(1_000_000, 800, split=0)
            ht.random.rand(1_000_000, 800, split=0)
    elif which == "smallk":
        x = torch.randn(12_500_000, 64, device="cuda")
        c = torch.randn(8, 64, device="cuda")
        for _ in range(10):
            ops.kmeans_step_small(x, c)
    elif which == "cdist_exact":
        x = torch.rand(40_000, 18, device="cuda")
        for _ in range(3):
            ops.cdist(x, x, exact=True)
    elif which == "gemm_small":
        from heat_amd.core.linalg import basics

        for n in (1024, 2048):
            a = torch.randn(n, n, device="cuda")
            b = torch.randn(n, n, device="cuda")
            for _ in range(5):
                basics.fgemm(a, b)
    elif which == "gemm_f32s_big":
        # the 128-tile kernel alone on large products (6144^3, 8192^3, one K slice)
        from heat_amd.ops import kernels as K

        for n in (6144, 8192):
            a = torch.randn(n, n, device="cuda")
            b = torch.randn(n, n, device="cuda")
            for _ in range(3):
                K.gemm_f32_small(a, b, slices=1)
    elif which == "gram":
        A = ht.random.randn(400_000, 2048, split=0)
        for _ in range(3):
            ht.matmul(A.T, A)
    elif which == "hh":
        # round 4: two-level Householder QR pieces (panel steps, sliced V^T C, library update)
        a = torch.randn(400_000, 1024, device="cuda")
        ops.householder_qr(a, 0, a.shape[0], True)
    torch.cuda.synchronize()
    print("done", which)


if __name__ == "__main__":
    main()
