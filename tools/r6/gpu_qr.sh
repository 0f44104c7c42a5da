#!/bin/bash
# round 6: bench.py --workload qr on one GPU, a 2-rank shared-GPU rehearsal of it, and a kernel trace
# of the Householder QR (no library GEMM expected)
set -o pipefail
OUT=gpurun_out/r6qr; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u bench.py --workload qr --steps 3 --warmup 1 > $OUT/qr1.json 2> $OUT/qr1.err || exit 1
echo qr1 ok
HEAT_BENCH_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --workload qr --gpus 2 --steps 2 --warmup 1 --n-per-gpu 625000 > $OUT/qr2_shared.json 2> $OUT/qr2_shared.err || exit 2
echo qr2 ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/hhtrace -o hh -- python3 $ROOT/tools/microbench/hh_profile.py > $ROOT/$OUT/hhtrace.log 2>&1 || exit 3
echo trace ok
