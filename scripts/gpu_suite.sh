# full GPU suite + smoke + the C3 bench lines (mode all, mode single); outputs under gpurun_out/suite
set -e
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/suite
MPGNN_PARITY_REPORT=$PWD/gpurun_out/suite/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/suite/bench_c3.json 2> gpurun_out/suite/bench_c3.err
timeout -k 10 300 python bench.py --mode single > gpurun_out/suite/bench_c3_single.json 2> gpurun_out/suite/bench_c3_single.err
echo ok
