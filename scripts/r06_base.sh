#!/bin/bash
# Round-6 baseline on one box: the driver's exact bench command, then a kernel trace of the C3
# forward steps alone (no epoch / loop legs) for the per-boundary gap analysis.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6base}
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
echo driver-bench done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 0 > $O/bench_trace.json 2> $O/bench_trace.err || exit $?
echo trace done
