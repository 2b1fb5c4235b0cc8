# fused backward: parity subset, then the C3 epoch A/B (MPGNN_OPT_BWD_FUSED 1 / 0), mode ALL and SINGLE
set -e
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fused_backward or backward or bwd or graph or net_forward or rel_gemm or width or shards or adam or chunk or single or squeeze or fast or golden or deterministic or multirank" > gpurun_out/bwd_tests.log 2>&1
OPTS="f1:--bwd-fused 1;f0:--bwd-fused 0" ARGS="--epoch-steps 30" bash scripts/ab_opts.sh
OPTS="g1:--bwd-fused 1 --mode single;g0:--bwd-fused 0 --mode single" ARGS="--epoch-steps 30" bash scripts/ab_opts.sh
