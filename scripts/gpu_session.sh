#!/bin/bash
# Round-2 GPU session: parity suite + smoke, bench lines, rocprofv3 kernel stats of the headline
# bench, PMC passes of one forward layer (traffic + MFMA utilisation) and of the training step.
# Every GPU step runs under its own time limit; a crash / abort / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    mkdir -p "$OUT"; echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
    case $rc in 0|1) ;; *) echo "FATAL in $name, stopping"; exit $rc;; esac
}
for part in ${PARTS:-test bench prof pmc}; do
  case $part in
  test)
    MPGNN_PARITY_REPORT=$OUT/parity.jsonl step pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
    step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    step bench_c3 300 python -u bench.py
    grep '^{' $OUT/bench_c3.log > $OUT/bench_c3.json || true
    step bench_c3_single 300 python -u bench.py --mode single
    grep '^{' $OUT/bench_c3_single.log > $OUT/bench_c3_single.json || true ;;
  prof)
    step rocprof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --epoch-steps 10 ;;
  pmc)
    OUT_PMC=$OUT/pmc
    OUT=$OUT_PMC ARGS="--iters 20" step pmc_fwd 600 bash scripts/pmc.sh
    OUT=$OUT_PMC python3 scripts/pmc_report.py $OUT_PMC fwd > $OUT/pmc_report_fwd.json
    OUT=$OUT/pmc_bwd ARGS="--iters 20 --backward" step pmc_bwd 600 bash scripts/pmc.sh
    python3 scripts/pmc_report.py $OUT/pmc_bwd bwd > $OUT/pmc_report_bwd.json ;;
  esac
done
echo done
