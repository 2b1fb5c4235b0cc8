set -u
O=${O:-gpurun_out/r6s}
mkdir -p $O
for v in 4,0,1024 2,0,2048 8,0,512 8,0,1024 4,1,1024 8,1,512 4,0,2048; do
  MPGNN_ADAM_VARIANT=$v MPGNN_ADAM_BLOCKS=$v timeout -k 10 120 python3 scripts/adam_probe.py > $O/adam_${v//,/_}.json 2> $O/adam_${v//,/_}.err || exit $?
done
