#!/bin/bash
# A/B of two library builds on one box (the tree's and libmpgnn_rgcn_prev.so), alternated 3x:
# per-kernel times of a C3 layer (ab_opt_layer, identity switch) and the C3 bench (step + epoch).
set -o pipefail
out=${OUT:-gpurun_out/r5u}
mkdir -p $out
PREV=mpgnn-metapath-graph-neural-network_amd/libmpgnn_rgcn_prev.so
for rep in 1 2 3; do
  for v in cur prev; do
    if [ $v = prev ]; then export MPGNN_LIB_PATH=$PREV; else unset MPGNN_LIB_PATH; fi
    timeout -k 10 120 python -u scripts/ab_opt_layer.py --opt 33 --values 1,1 --iters 20 --rounds 1 \
      > $out/ab_${v}_${rep}.json 2>> $out/ab.err || exit 1
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --loop-epochs 0 --steps 20 \
      > $out/bench_${v}_${rep}.json 2>> $out/bench.err || exit 1
  done
done
unset MPGNN_LIB_PATH
echo done
