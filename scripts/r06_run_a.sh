set -u
mkdir -p gpurun_out/r6t
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_loop.py -m gpu -x -q --timeout 120 --timeout-method thread -k "w1_gemm or wide_classes or confusion" > gpurun_out/r6t/new.txt 2>&1 || exit $?
bash scripts/r06_epoch_trace.sh
