# round-3 GPU validation chain: each step time-limited, stop at the first failure
mkdir -p gpurun_out && export PYTHONPATH=$PWD
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "moments" > gpurun_out/t_moments.txt 2>&1 && \
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "kmeans_update or bit_reproducible" > gpurun_out/t_kmeans.txt 2>&1 && \
timeout -k 10 300 $T tests/test_gpu_gemm.py > gpurun_out/t_gemm.txt 2>&1 && \
timeout -k 10 300 $T tests/test_gpu_qr.py > gpurun_out/t_qr.txt 2>&1 && \
timeout -k 10 300 $T tests/test_gpu_ipc.py tests/test_gpu_native_comm.py > gpurun_out/t_ipc.txt 2>&1 && \
timeout -k 10 500 python -u tools/microbench/gemm_bench.py 8192x8192x8192 1250000x4096x4096 gram:1250000:4096 > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err
