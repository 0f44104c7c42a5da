# round-3 GPU chain d: kernel tests, bench.py, moments whole-call timing + rocprof, linalg rocprof
mkdir -p gpurun_out/prof_mom gpurun_out/prof_lin gpurun_out/prof_bench && export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_kernels.py -k "matmul_split_precision or kmeans or moments" > gpurun_out/t_kernels.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_1gpu.json 2> gpurun_out/bench_1gpu.err && \
timeout -k 10 200 python -u tools/microbench/moments_prof.py > gpurun_out/moments_wall.jsonl 2> gpurun_out/moments_wall.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mom -o mom -- python3 tools/microbench/moments_prof.py > gpurun_out/prof_mom.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_bench.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lin -o lin -- python3 tools/microbench/linalg_bench.py > gpurun_out/prof_lin.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/pmc_gemm -o gemm -- python3 tools/microbench/gemm_bench.py 8192x8192x8192 --only=f32t,blas_f32,h3t,blas_f16x3 --quick > gpurun_out/pmc_gemm.log 2>&1
