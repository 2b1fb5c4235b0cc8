# kernel trace of the C3 mode-SINGLE epoch legs (MPNetm)
set -u
O=${O:-gpurun_out/r6w}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --mode single --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
