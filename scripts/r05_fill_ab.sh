#!/bin/bash
# The grad_x split-counter memset as one fill launch and the fused training loss: GPU suite, the
# kernel trace of the C3 bench (launches per epoch), the C3 library A/B against
# libmpgnn_rgcn_prev.so (fill change only), the loss A/B (both modes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/fill}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
echo suite done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
echo prof done
timeout -k 10 200 python -u scripts/epoch_host_profile.py --mode all --ab-loss --epochs 30 > $O/ab_loss_all.json 2>&1 || exit $?
timeout -k 10 200 python -u scripts/epoch_host_profile.py --mode single --ab-loss --epochs 30 > $O/ab_loss_single.json 2>&1 || exit $?
echo loss ab done
OUT=$O bash scripts/r05_ab_lib_c3.sh || exit $?
