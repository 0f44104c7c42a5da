# round-3 GPU chain b: IPC + v-collective tests, GEMM and linalg benchmarks
mkdir -p gpurun_out && export PYTHONPATH=$PWD
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_ipc.py tests/test_gpu_native_comm.py > gpurun_out/t_ipc.txt 2>&1 && \
timeout -k 10 400 $T tests/test_gpu_dist.py -k vcoll > gpurun_out/t_vcoll.txt 2>&1 && \
timeout -k 10 500 python -u tools/microbench/gemm_bench.py 8192x8192x8192 1250000x4096x4096 gram:1250000:4096 > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py > gpurun_out/linalg_bench.jsonl 2> gpurun_out/linalg_bench.err
