# re-check the GEMM range balance (MPGNN_OPT_GEMM_SWITCH_COST = 29) with the prologue records on:
# C3 forward GEMM at VALS (150 / 250 / 400, then 30 / 75 / 150), fresh processes alternated 3x
set -u
O=${O:-gpurun_out/r6ae}
mkdir -p $O
for i in 1 2 3; do
  for v in ${VALS:-150 250 400}; do
    MPGNN_BENCH_SET_OPT=29=$v timeout -k 10 150 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 0 > $O/sc_${v}_$i.json 2> $O/sc_${v}_$i.err || exit $?
  done
done
