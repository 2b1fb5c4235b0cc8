# side-stream slab reduce (option 41): its bit-identity tests, then the C3 epoch with 41=1 vs 0,
# alternated 3x, and a trace with it on
set -u
O=${O:-gpurun_out/r6y}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "variants_bit_identical or shared_conv2 or net_forward_backward" > $O/t.txt 2>&1 || exit $?
for i in 1 2 3; do
  for v in 1 0; do
    MPGNN_BENCH_SET_OPT=41=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 > $O/ep_side${v}_$i.json 2> $O/ep_side${v}_$i.err || exit $?
  done
done
MPGNN_BENCH_SET_OPT=41=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
