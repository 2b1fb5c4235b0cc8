#!/bin/bash
# Round-4 bench lines (each step under its own limit; the first failure ends the call):
# score_bags / score_all / score (C3), C5 mode ALL + SINGLE. Outputs under gpurun_out/r04.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
OUT=$O
run() {  # name timeout args...
    local name=$1 to=$2; shift 2
    echo "== $name: bench.py $*"
    timeout -k 10 "$to" python -u bench.py "$@" > "$OUT/bench_$name.log" 2>&1
    local rc=$?
    grep '^{' "$OUT/bench_$name.log" > "$OUT/bench_$name.json"
    echo "rc=$rc"; tail -c 400 "$OUT/bench_$name.json"; echo
    case $rc in 0) ;; *) tail -20 "$OUT/bench_$name.log"; exit $rc;; esac
}
SPECS=("score_bags:300:--mode score_bags" "score_all:300:--mode score_all" "score:300:--mode score"
       "c5:900:--workload C5 --steps 5 --warmup 1" "c5_single:600:--workload C5 --mode single --steps 10 --warmup 2")
if [[ -n "${ONLY:-}" ]]; then SPECS=("$ONLY"); fi
for spec in "${SPECS[@]}"; do
    IFS=: read -r name to args <<< "$spec"
    run "$name" "$to" $args
done
echo done
