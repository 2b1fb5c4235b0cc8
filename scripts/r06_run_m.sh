# HIP Adam v2 (LDS tensor table, 4 slots in flight, no per-workgroup fence): its bit-identity
# test, then the C3 epoch with it against torch's pair, fresh processes alternated
set -u
O=${O:-gpurun_out/r6m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "adam or lean" -s > $O/t_adam.txt 2>&1 || exit $?
for i in 1 2 3; do
  for a in 1 0; do
    MPGNN_HIP_ADAM=$a timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 > $O/ep_adam${a}_$i.json 2> $O/ep_adam${a}_$i.err || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
