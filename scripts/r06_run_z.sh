# refresh the mode-SINGLE bench lines after the dropout + ReLU backward fusion
set -u
O=${O:-gpurun_out/r6z}
mkdir -p $O
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" python -u bench.py "$@" > "$O/bench_$name.log" 2>&1 || exit $?; grep '^{' "$O/bench_$name.log" > "$O/bench_$name.json"; }
run c3_single 300 --mode single
run c2_single 300 --workload C2 --mode single
run c5_single 600 --workload C5 --mode single --steps 10 --warmup 2
