# switch cost 120 / 150 / 190 (forward GEMM), then the epoch at 150 vs 250, alternated 3x
set -u
O=${O:-gpurun_out/r6af}
mkdir -p $O
for i in 1 2 3; do
  for v in 120 150 190; do
    MPGNN_BENCH_SET_OPT=29=$v timeout -k 10 150 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 0 > $O/sc_${v}_$i.json 2> $O/sc_${v}_$i.err || exit $?
  done
done
for i in 1 2 3; do
  for v in 150 250; do
    MPGNN_BENCH_SET_OPT=29=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 > $O/ep_${v}_$i.json 2> $O/ep_${v}_$i.err || exit $?
  done
done
