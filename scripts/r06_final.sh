#!/bin/bash
# Round-6 closing evidence in one GPU call (each step under its own limit; the first failure ends
# the call): GPU suite + parity report + smoke, the driver's exact bench command, rocprofv3 kernel
# stats + trace of the C3 bench (timed region isolated by scripts/step_gaps.py), the epoch's
# kernels, the PMC passes of one C3 layer forward / training step, every bench line, and the
# per-rank shard compute. PART=suite|prof|pmc|bench|shard runs one part (default: all).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6f}
P=${PART:-all}
mkdir -p $O
if [[ $P == all || $P == suite ]]; then
MPGNN_PARITY_REPORT=$PWD/$O/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
echo suite done
fi
if [[ $P == all || $P == prof ]]; then
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
echo prof done
fi
if [[ $P == all || $P == pmc ]]; then
OUT=$O/pmc_fwd bash scripts/pmc.sh > $O/pmc_fwd.log 2>&1 || exit $?
OUT=$O/pmc_bwd ARGS="--iters 10 --backward" bash scripts/pmc.sh > $O/pmc_bwd.log 2>&1 || exit $?
echo pmc done
fi
if [[ $P == all || $P == bench ]]; then
OUT=$O bash scripts/bench_all.sh ${BENCH_SET:-full} > $O/bench_all.log 2>&1 || exit $?
echo bench done
fi
if [[ $P == all || $P == shard ]]; then
timeout -k 10 300 python3 scripts/shard_compute.py gathered > $O/shard_gathered.json 2> $O/shard_gathered.err || exit $?
timeout -k 10 300 python3 scripts/shard_compute.py rows > $O/shard_rows.json 2> $O/shard_rows.err || exit $?
echo shard done
fi
echo all done
