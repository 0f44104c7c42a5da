# round-3 GPU chain c: QR / GEMM tests (split-K Gram, vtc64, two-level Householder), linalg bench
mkdir -p gpurun_out && export PYTHONPATH=$PWD
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_qr.py tests/test_gpu_gemm.py > gpurun_out/t_qr.txt 2>&1 && \
timeout -k 10 500 python -u tools/microbench/linalg_bench.py --householder > gpurun_out/linalg_bench.jsonl 2> gpurun_out/linalg_bench.err
