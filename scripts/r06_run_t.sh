# kernel trace of the drop-in training loop leg alone (main_rgcn.mpgnn_parallel_multiple, C3)
set -u
O=${O:-gpurun_out/r6t}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/looptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 20 --epoch-steps 0 > $O/bench_loop.json 2> $O/bench_loop.err || exit $?
