#!/bin/bash
# Bench lines of every workload on one GPU box (each step under its own time limit; a crash,
# abort or timeout ends the session). Usage: bash scripts/bench_all.sh [quick|full]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
run() {  # name timeout args...
    local name=$1 to=$2; shift 2
    echo "== $name: bench.py $*"
    timeout -k 10 "$to" python -u bench.py "$@" > "$OUT/bench_$name.log" 2>&1
    local rc=$?
    grep '^{' "$OUT/bench_$name.log" > "$OUT/bench_$name.json"
    echo "rc=$rc"; tail -c 600 "$OUT/bench_$name.json"; echo
    case $rc in 0) ;; *) tail -20 "$OUT/bench_$name.log"; exit $rc;; esac
}
MODE=${1:-quick}
run c3 300
run c3_single 300 --mode single
run c2_single 300 --workload C2 --mode single
run c2 300 --workload C2
if [[ $MODE == full ]]; then
    run c3_relcond 300 --workload fb15k237_relcond
    run c5_single 600 --workload C5 --mode single --steps 10 --warmup 2
    run c5 900 --workload C5 --steps 5 --warmup 1
fi
echo done
