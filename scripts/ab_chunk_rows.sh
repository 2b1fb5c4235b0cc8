set -e
mkdir -p gpurun_out/cr
for rep in 1 2; do
for cr in 256 192 384 320; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --loop-epochs 0 --chunk-rows $cr > gpurun_out/cr/b_${cr}_$rep.json 2>/dev/null
done
done
