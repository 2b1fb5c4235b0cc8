# MPNetm: dropout + ReLU backward fused: the new test and the MPNetm tests, the GPU suite, then
# the C3 mode-SINGLE epoch with the fusion on / off, alternated 3x, and its trace
set -u
O=${O:-gpurun_out/r6x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mpnetm or dropout or graph_captured or single" > $O/t_new.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
for i in 1 2 3; do
  for a in 1 0; do
    MPGNN_RELU_FUSE=$a timeout -k 10 200 python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 40 --epoch-steps 60 > $O/single_fuse${a}_$i.json 2> $O/single_fuse${a}_$i.err || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --mode single --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
