set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/final5
mkdir -p $O
MPGNN_PARITY_REPORT=$PWD/$O/parity_report.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
echo suite done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_single -o run --output-format csv -- python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof_single.json 2> $O/bench_prof_single.err || exit $?
echo prof done
OUT=$O/pmc_fwd bash scripts/pmc.sh > $O/pmc_fwd.log 2>&1 || exit $?
OUT=$O/pmc_bwd ARGS="--iters 10 --backward" bash scripts/pmc.sh > $O/pmc_bwd.log 2>&1 || exit $?
echo pmc done
