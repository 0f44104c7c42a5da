# round-3 GPU chain c: QR / GEMM tests (split-K Gram, vtc64, two-level Householder), linalg bench
mkdir -p gpurun_out && export PYTHONPATH=$PWD
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_qr.py -k cholqr_native > gpurun_out/t_qr.txt 2>&1 && \
timeout -k 10 500 python -u tools/microbench/linalg_bench.py --householder > gpurun_out/linalg_bench.jsonl 2> gpurun_out/linalg_bench.err && \
timeout -k 10 300 python -u tools/microbench/gemm_bench.py 8192x8192x8192 1250000x4096x4096 gram:1250000:4096 --only=f32t,blas_f32 --quick > gpurun_out/gemm_sp1.jsonl 2>&1 && \
HEAT_GEMM_F32_SPREAD=0 timeout -k 10 300 python -u tools/microbench/gemm_bench.py 8192x8192x8192 1250000x4096x4096 gram:1250000:4096 --only=f32t,blas_f32 --quick > gpurun_out/gemm_sp0.jsonl 2>&1
