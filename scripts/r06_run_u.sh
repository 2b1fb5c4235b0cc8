# weighted NLL rows + register-count confusion counts: GPU suite, then the drop-in loop leg
# (3 fresh processes) and its kernel trace
set -u
O=${O:-gpurun_out/r6u}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 120 --epoch-steps 30 > $O/loop_$i.json 2> $O/loop_$i.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/looptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 20 --epoch-steps 0 > $O/bench_loop.json 2> $O/bench_loop.err || exit $?
