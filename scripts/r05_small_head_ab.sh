#!/bin/bash
# The narrow Linear heads' forward (O <= 8) on the C ABI (float64 sums): GPU suite, then the
# eager C3 epoch A/B against torch's addmm for those heads (both modes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/smallhead}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
echo suite done
timeout -k 10 200 python -u scripts/epoch_host_profile.py --mode single --ab-small-fwd --epochs 30 > $O/ab_single.json 2>&1 || exit $?
timeout -k 10 200 python -u scripts/epoch_host_profile.py --mode all --ab-small-fwd --epochs 30 > $O/ab_all.json 2>&1 || exit $?
echo ab done
