#!/bin/bash
# rel_gemm_w1_kernel (MPGNN_OPT_GEMM_W1 = 35) against rel_gemm_bf3_kernel: bit-equality of one C3
# layer's forward and gradients, per-kernel times alternated, then the forward step both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/r6w1}
mkdir -p $O
timeout -k 10 200 python3 scripts/ab_opt_layer.py --opt 35 --values 0,1 --iters 30 --rounds 3 > $O/ab_layer.json 2> $O/ab_layer.err || exit $?
echo ab done
timeout -k 10 200 python3 scripts/step_probe.py --opt 35=0 --json $O/step0.json > $O/step0.out 2>&1 || exit $?
timeout -k 10 200 python3 scripts/step_probe.py --opt 35=1 --json $O/step1.json > $O/step1.out 2>&1 || exit $?
echo step done
