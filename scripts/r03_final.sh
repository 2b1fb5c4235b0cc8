#!/bin/bash
# Round-3 closing evidence in one GPU call (each step under its own limit; the first failure
# ends the call): grad-stash A/B on one box (AB=1), the GPU suite + smoke, rocprofv3 kernel stats of the C3 bench commands
# (mode ALL, mode SINGLE), then the bench lines of C3 / C3 single / C2 / C2 single.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
if [[ ${AB:-0} == 1 ]]; then
for i in 1 2; do
    MPGNN_GRAD_STASH=0 timeout -k 10 200 python bench.py --no-cpu-baseline --epoch-steps 100 > $O/ab_off_$i.json 2> $O/ab_off_$i.err || exit $?
    MPGNN_GRAD_STASH=1 timeout -k 10 200 python bench.py --no-cpu-baseline --epoch-steps 100 > $O/ab_on_$i.json 2> $O/ab_on_$i.err || exit $?
done
echo ab done
fi
MPGNN_PARITY_REPORT=$PWD/$O/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_single -o run --output-format csv -- \
    python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof_single.json 2> $O/bench_prof_single.err || exit $?
echo prof done
OUT=$O bash scripts/bench_all.sh quick
