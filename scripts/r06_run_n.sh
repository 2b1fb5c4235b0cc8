set -u
O=${O:-gpurun_out/r6n}
mkdir -p $O
for nb in 256 512 1024 2048 4096; do
  MPGNN_ADAM_BLOCKS=$nb timeout -k 10 120 python3 scripts/adam_probe.py > $O/adam_$nb.json 2> $O/adam_$nb.err || exit $?
done
