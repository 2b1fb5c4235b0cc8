#!/bin/bash
# A/B of two library builds on one box (the tree's and libmpgnn_rgcn_prev.so), alternated:
# per-kernel times of a C5 layer (ab_opt_layer, identity switch) and the C5 mode-SINGLE step.
set -o pipefail
out=${OUT:-gpurun_out/r5q}
mkdir -p $out
PREV=mpgnn-metapath-graph-neural-network_amd/libmpgnn_rgcn_prev.so
for rep in 1 2; do
  for v in cur prev; do
    if [ $v = prev ]; then export MPGNN_LIB_PATH=$PREV; else unset MPGNN_LIB_PATH; fi
    timeout -k 10 200 python -u scripts/ab_opt_layer.py --opt 33 --values 1,1 --workload C5 --iters 3 --rounds 1 \
      > $out/ab_${v}_${rep}.json 2>> $out/ab.err || exit 1
    timeout -k 10 200 python -u bench.py --workload C5 --mode single --no-cpu-baseline --loop-epochs 0 --epoch-steps 0 --steps 10 \
      > $out/single_${v}_${rep}.json 2>> $out/bench.err || exit 1
  done
done
unset MPGNN_LIB_PATH
echo done
