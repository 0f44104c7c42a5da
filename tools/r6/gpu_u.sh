#!/bin/bash
# round 6: 8- and 4-rank shared-GPU rehearsal of the distributed QR workload (CholeskyQR2 over the
# world: Gram all-reduce, replicated fp64 Cholesky, local triangular products)
set -o pipefail
OUT=gpurun_out/r6u; mkdir -p $OUT
export HEAT_BENCH_SHARED_GPU=1
timeout -k 10 400 python bench.py --gpus 8 --workload qr --steps 2 --warmup 0 --n-per-gpu 131072 --f 1024 --comm-ab 0 > $OUT/shared8_qr.json 2> $OUT/shared8_qr.err || exit 1
echo "qr8 done"
timeout -k 10 400 python bench.py --gpus 4 --workload qr --steps 2 --warmup 1 --n-per-gpu 262144 --f 2048 --comm-ab 0 > $OUT/shared4_qr.json 2> $OUT/shared4_qr.err || exit 2
echo "qr4 done"
