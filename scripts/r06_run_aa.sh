# GEMM prologue records (option 42): bit-identity tests, then the C3 step and epoch with 42=1 vs 0,
# fresh processes alternated 3x
set -u
O=${O:-gpurun_out/r6aa}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "variants_bit_identical" > $O/t.txt 2>&1 || exit $?
for i in 1 2 3; do
  for v in 1 0; do
    MPGNN_BENCH_SET_OPT=42=$v timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 > $O/ab42_${v}_$i.json 2> $O/ab42_${v}_$i.err || exit $?
  done
done
