#!/bin/bash
# The narrow heads' forward at four rows per wave: GPU suite, the eager C3 epoch A/B against
# torch's addmm for those heads (mode ALL), and its kernel time in a short bench trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/smallhead2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
echo suite done
timeout -k 10 200 python -u scripts/epoch_host_profile.py --mode all --ab-small-fwd --epochs 30 > $O/ab_all.json 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench.json 2> $O/bench.err || exit $?
echo done
