# Lasso covariance-solver GPU check: kernel tests, gram-pass unroll/occupancy sweep, solver comparison.
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_framework.py -x -v --timeout 120 --timeout-method thread -k "lasso" > gpurun_out/lasso_tests.log 2>&1
for u in 1 2 4; do for b in 1 2; do
HEAT_GRAM_UNROLL=$u HEAT_GRAM_BLOCKS_PER_CU=$b HEAT_LASSO_SOLVER=gram timeout -k 10 120 python -u -m benchmarks.lasso.run --iterations 1 --trials 7 2>&1 | grep median | sed "s/^/u=$u b=$b /" >> gpurun_out/lasso_bench.log
done; done
for s in sweep gram; do
HEAT_LASSO_SOLVER=$s timeout -k 10 120 python -u -m benchmarks.lasso.run --iterations 100 --trials 5 2>&1 | grep median >> gpurun_out/lasso_bench.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HEAT_LASSO_SOLVER=gram timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lasso_gram -o run -- python3 -m benchmarks.lasso.run --iterations 100 --trials 3 > gpurun_out/lasso_prof.log 2>&1
tail -3 gpurun_out/lasso_tests.log
cat gpurun_out/lasso_bench.log
