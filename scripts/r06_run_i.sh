set -u
mkdir -p gpurun_out/r6fold
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "single_fold" > gpurun_out/r6fold/t.txt 2>&1 || exit $?
for r in 1 2 3; do
  for v in 0 1; do
    MPGNN_BENCH_SET_OPT=39=$v timeout -k 10 150 python3 bench.py --mode single --steps 50 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 30 > gpurun_out/r6fold/c3_${v}_$r.json 2> gpurun_out/r6fold/c3_${v}_$r.err || exit $?
  done
done
for v in 0 1; do
  MPGNN_BENCH_SET_OPT=39=$v timeout -k 10 150 python3 bench.py --mode single --workload C2 --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > gpurun_out/r6fold/c2_${v}.json 2> gpurun_out/r6fold/c2_${v}.err || exit $?
done
