# Lasso covariance-solver GPU check: solver comparison at wide n.
set -e
export PYTHONUNBUFFERED=1
for f in 1024; do for s in gram sweep; do for it in 1 20; do
HEAT_LASSO_SOLVER=$s timeout -k 10 150 python -u -m benchmarks.lasso.run --rows 4000000 --features $f --iterations $it --trials 3 >> gpurun_out/lasso_bench.log 2>&1
done; done; done
grep median gpurun_out/lasso_bench.log | cut -c1-220
