# mode-SINGLE GPU check: the single-layer / MPNetm parity tests, then the C3 single bench
set -e
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_score.py tests/test_loop.py -k "single or custom or mpnetm or adam or golden or squeeze or score or loop" > gpurun_out/single_tests.log 2>&1
timeout -k 10 200 python bench.py --mode single --no-cpu-baseline > gpurun_out/bench_single_bf3.json
echo ok
