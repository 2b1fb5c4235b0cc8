#!/bin/bash
# bench.py's C3 headline line with and without the clock pre-warm (MPGNN_BENCH_PREWARM_S), three
# alternations, each a fresh process with the driver's --steps 20 --warmup 5; then the driver's
# exact command once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/r6pw}
mkdir -p $O
for r in 1 2 3; do
  for pw in 0 0.3; do
    MPGNN_BENCH_PREWARM_S=$pw timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 0 > $O/pw${pw}_$r.json 2> $O/pw${pw}_$r.err || exit $?
  done
done
echo ab done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
echo driver done
