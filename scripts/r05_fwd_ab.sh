#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/fwdab
mkdir -p $out
PREV=mpgnn-metapath-graph-neural-network_amd/libmpgnn_rgcn_prev.so
for rep in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then export MPGNN_LIB_PATH=$PREV; else unset MPGNN_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --loop-epochs 0 --steps 50 > $out/bench_${v}_${rep}.json 2>> $out/bench.err || exit 1
  done
done
echo done
