set -u
mkdir -p gpurun_out/r6j
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py tests/test_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6j/t.txt 2>&1 || exit $?
