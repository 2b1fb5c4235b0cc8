# switch cost 150 by default: the GPU suite, then the closing bench lines (driver command, C3 with
# stats trace, the quick bench set)
set -u
O=${O:-gpurun_out/r6ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
O=$O PART=prof bash scripts/r06_final.sh > $O/prof.log 2>&1 || exit $?
OUT=$O bash scripts/bench_all.sh full > $O/bench_all.log 2>&1 || exit $?
