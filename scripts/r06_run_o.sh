# head log_softmax fusion + the earlier epoch fusions: new tests, GPU suite, then the C3 epoch
# with every epoch fusion on (1) against all off (0: torch's Adam pair, separate ReLU backwards,
# F.linear + F.log_softmax), fresh processes alternated 3x; a kernel trace of the epoch legs
set -u
O=${O:-gpurun_out/r6o}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "head_log_softmax or relu_backward_fused or net_forward_backward or adam or shared_conv2 or nll_loss_rows" > $O/t_new.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
for i in 1 2 3; do
  for a in 1 0; do
    MPGNN_HIP_ADAM=$a MPGNN_RELU_FUSE=$a MPGNN_HEAD_FUSE=$a MPGNN_NLL_DENSE=$a timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 > $O/ep_fuse${a}_$i.json 2> $O/ep_fuse${a}_$i.err || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/eptrace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 > $O/bench_ep.json 2> $O/bench_ep.err || exit $?
