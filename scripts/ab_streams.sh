# GPU parity of the backward (two-stream default) + the streams A/B on the C3 bench
set -e
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "backward or bwd or graph or net_forward or rel_gemm or width or shards or adam or chunk or single or linear" > gpurun_out/streams_tests.log 2>&1
OPTS="s1:--bwd-streams 1;s0:--bwd-streams 0" ARGS="--epoch-steps 30" bash scripts/ab_opts.sh
