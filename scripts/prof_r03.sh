#!/bin/bash
# Round-3 profiles of the C3 headline (outputs under gpurun_out/r03, summaries copied to
# profiles/r03_* on the CPU side): rocprofv3 kernel-trace stats of the mode-ALL and mode-SINGLE
# bench commands, then the PMC passes of scripts/pmc.sh (forward layer; forward + backward).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/stats -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > gpurun_out/r03/bench_prof.json 2> gpurun_out/r03/bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/stats_single -o run --output-format csv -- \
    python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > gpurun_out/r03/bench_prof_single.json 2> gpurun_out/r03/bench_prof_single.err || exit $?
OUT=gpurun_out/r03/pmc_fwd bash scripts/pmc.sh > gpurun_out/r03/pmc_fwd.log 2>&1 || exit $?
OUT=gpurun_out/r03/pmc_bwd ARGS="--iters 10 --backward" bash scripts/pmc.sh > gpurun_out/r03/pmc_bwd.log 2>&1 || exit $?
echo done
