set -e
export PYTHONUNBUFFERED=1
: timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_framework.py -x -v --timeout 120 --timeout-method thread -k "lasso" > gpurun_out/lasso_tests.log 2>&1
for s in sweep gram; do for it in 1 100; do
HEAT_LASSO_SOLVER=$s timeout -k 10 120 python -u -m benchmarks.lasso.run --iterations $it --trials 5 >> gpurun_out/lasso_bench.log 2>&1
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HEAT_LASSO_SOLVER=gram timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lasso_gram -o run -- python3 -m benchmarks.lasso.run --iterations 100 --trials 3 > gpurun_out/lasso_prof.log 2>&1
cat gpurun_out/lasso_bench.log | grep -v "^$" | tail -8
