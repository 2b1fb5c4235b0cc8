# one-pass confusion counts, class weights from LDS: their tests, then the loop trace
set -u
O=${O:-gpurun_out/r6v}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nll or confusion or loop" > $O/t.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/looptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 20 --epoch-steps 0 > $O/bench_loop.json 2> $O/bench_loop.err || exit $?
