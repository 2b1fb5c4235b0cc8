#!/bin/bash
# Round-5 closing evidence in one GPU call (each step under its own limit; the first failure ends
# the call): GPU suite + smoke, rocprofv3 kernel stats of the C3 bench commands (mode ALL, mode
# SINGLE), the PMC passes of the C3 forward / backward layer, then the C3 / C2 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/final5}
mkdir -p $O
if [[ ${SKIP_SUITE:-0} != 1 ]]; then
MPGNN_PARITY_REPORT=$PWD/$O/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
echo suite done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_single -o run --output-format csv -- \
    python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof_single.json 2> $O/bench_prof_single.err || exit $?
echo prof done
OUT=$O/pmc_fwd bash scripts/pmc.sh > $O/pmc_fwd.log 2>&1 || exit $?
OUT=$O/pmc_bwd ARGS="--iters 10 --backward" bash scripts/pmc.sh > $O/pmc_bwd.log 2>&1 || exit $?
echo pmc done
OUT=$O bash scripts/bench_all.sh ${BENCH_SET:-full} || exit $?
echo all done
