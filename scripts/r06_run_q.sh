# weight-gradient chunk length (MPGNN_OPT_CHUNK_ROWS: fewer, longer chunks = fewer slabs for the
# ordered reduce, coarser outer-kernel balance): the C3 epoch at 256 / 384 / 512 / 768, alternated 2x
set -u
O=${O:-gpurun_out/r6q}
mkdir -p $O
for i in 1 2; do
  for c in 256 384 512 768; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 60 --chunk-rows $c > $O/ep_c${c}_$i.json 2> $O/ep_c${c}_$i.err || exit $?
  done
done
for c in 256 512; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_c$c -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --loop-epochs 0 --epoch-steps 10 --chunk-rows $c > $O/tr_c$c.json 2> $O/tr_c$c.err || exit $?
done
