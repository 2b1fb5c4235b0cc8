#!/bin/bash
# Kernel trace of the C3 bench's epoch leg (no loop leg, no CPU baseline) for scripts/epoch_kernels.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6ep}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench.json 2> $O/bench.err || exit $?
echo trace done
