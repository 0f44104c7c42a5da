# Lasso covariance-solver GPU check: kernel tests, then the solvers at wide n.
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_framework.py -x -q --timeout 120 --timeout-method thread -k "lasso" > gpurun_out/lasso_tests.log 2>&1
for f in 256 1024; do for s in gram; do for it in 1 20; do
HEAT_LASSO_SOLVER=$s timeout -k 10 150 python -u -m benchmarks.lasso.run --rows 4000000 --features $f --iterations $it --trials 3 >> gpurun_out/lasso_bench.log 2>&1
done; done; done
tail -2 gpurun_out/lasso_tests.log
grep median gpurun_out/lasso_bench.log | cut -c1-220
