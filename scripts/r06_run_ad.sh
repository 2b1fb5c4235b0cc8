# 16-byte lanes in the ordered slab reduce: the GPU suite, the epoch (3 runs) and its trace
set -u
O=${O:-gpurun_out/r6ad}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 > $O/ep_$i.json 2> $O/ep_$i.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
