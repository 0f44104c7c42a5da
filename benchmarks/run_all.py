"""
Run the benchmark suite at several GPU counts (one node) and collect the JSON lines:

    python -m benchmarks.run_all --gpus 1,2,4,8 --out results.jsonl [--quick]

Each (benchmark, N) runs as ``torch.distributed.run --nproc-per-node N`` (rendezvous on
127.0.0.1) in a child process with its own time limit.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name -> (module, extra arguments)
SUITE = {
    "kmeans": ("benchmarks.kmeans.run", []),
    "kmeans_reference": ("benchmarks.kmeans.run", ["--case", "reference"]),   # k = 8, 30 iterations
    "distance_matrix": ("benchmarks.distance_matrix.run", []),
    "knn": ("benchmarks.distance_matrix.run", ["--case", "knn"]),               # 1e6 x 1e6 x 128, k = 8
    "statistical_moments": ("benchmarks.statistical_moments.run", []),
    "lasso": ("benchmarks.lasso.run", []),
    "linalg": ("benchmarks.linalg.run", []),
    "linalg_high": ("benchmarks.linalg.run", ["--precision", "high"]),       # fp16x3 split GEMM
}
QUICK = {
    "kmeans": ["--rows-per-gpu", "200000", "--trials", "2"],
    "kmeans_reference": ["--rows-per-gpu", "200000", "--trials", "2"],
    "distance_matrix": ["--rows", "8000", "--trials", "2"],
    "knn": ["--rows", "8000", "--trials", "2"],
    "statistical_moments": ["--rows-per-gpu", "10000", "--cols", "100", "--trials", "2"],
    "lasso": ["--rows", "100000", "--trials", "2"],
    "linalg": ["--rows-per-gpu", "20000", "--cols", "256", "--trials", "2"],
    "linalg_high": ["--rows-per-gpu", "20000", "--cols", "256", "--trials", "2"],
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", default="1")
    p.add_argument("--only", default=",".join(SUITE))
    p.add_argument("--out", default="benchmark_results.jsonl")
    p.add_argument("--quick", action="store_true")
    p.add_argument("--timeout", type=int, default=900)
    a = p.parse_args()
    port = 29611
    with open(a.out, "a") as out:
        for n in [int(x) for x in a.gpus.split(",")]:
            for name in a.only.split(","):
                port += 1
                cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                       "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", SUITE[name][0]]
                cmd += SUITE[name][1]
                cmd += QUICK[name] if a.quick else []
                print("#", " ".join(cmd), flush=True)
                res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=a.timeout)
                for line in res.stdout.splitlines():
                    if line.startswith("{"):
                        out.write(line + "\n")
                        print(line, flush=True)
                if res.returncode != 0:
                    print(res.stderr[-3000:], file=sys.stderr)
                    return res.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
