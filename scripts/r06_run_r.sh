# MPNetm's head on the fused log-softmax path: GPU suite, then the C3 mode-SINGLE epoch with the
# round-6 epoch fusions on / off, alternated 3x
set -u
O=${O:-gpurun_out/r6r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
for i in 1 2 3; do
  for a in 1 0; do
    MPGNN_HIP_ADAM=$a MPGNN_RELU_FUSE=$a MPGNN_HEAD_FUSE=$a MPGNN_NLL_DENSE=$a timeout -k 10 200 python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 40 --epoch-steps 60 > $O/single_fuse${a}_$i.json 2> $O/single_fuse${a}_$i.err || exit $?
  done
done
