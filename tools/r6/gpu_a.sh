#!/bin/bash
# round 6, call a: 1-GPU bench + 8-rank shared-GPU rehearsal of the four bench workloads
set -o pipefail
mkdir -p gpurun_out/r6a
export HEAT_BENCH_AB_TIMEOUT=120
timeout -k 10 300 python bench.py > gpurun_out/r6a/bench1.json 2> gpurun_out/r6a/bench1.err || exit 1
echo "bench1 done"
export HEAT_BENCH_SHARED_GPU=1
timeout -k 10 400 python bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r6a/shared8_kmeans.json 2> gpurun_out/r6a/shared8_kmeans.err || exit 2
echo "kmeans8 done"
timeout -k 10 300 python bench.py --gpus 8 --workload moments --steps 3 --warmup 1 --comm-ab 0 > gpurun_out/r6a/shared8_moments.json 2> gpurun_out/r6a/shared8_moments.err || exit 3
echo "moments8 done"
timeout -k 10 400 python bench.py --gpus 8 --workload knn --steps 1 --warmup 1 --comm-ab 0 > gpurun_out/r6a/shared8_knn.json 2> gpurun_out/r6a/shared8_knn.err || exit 4
echo "knn8 done"
timeout -k 10 400 python bench.py --gpus 8 --workload cdist --steps 1 --warmup 1 --comm-ab 0 > gpurun_out/r6a/shared8_cdist.json 2> gpurun_out/r6a/shared8_cdist.err || exit 5
echo "cdist8 done"
