#!/bin/bash
# Reduction-chunk length A/B under the round-5 weight-gradient kernel: per-kernel times of one
# C3 layer (forward + training backward) and the bench epoch, alternated, one process each.
set -o pipefail
out=gpurun_out/r5p
mkdir -p $out
for rep in 1 2; do
  for cr in 256 128 192 96; do
    MPGNN_OPTS=20=$cr timeout -k 10 120 python -u scripts/ab_opt_layer.py --opt 33 --values 1,1 --iters 20 --rounds 1 \
      > $out/ab_cr${cr}_r${rep}.json 2>> $out/ab.err || exit 1
  done
done
for cr in 256 128 256 128; do
  timeout -k 10 200 python -u bench.py --chunk-rows $cr --no-cpu-baseline --loop-epochs 0 --steps 20 \
    >> $out/bench_cr${cr}.jsonl 2>> $out/bench.err || exit 1
done
echo done
