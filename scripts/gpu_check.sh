#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout ends the session there
# (exit 124/134/137/139); ordinary test failures (exit 1) do not stop the later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac; }

step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/session.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/session.log"
    tail -n 5 "$OUT/$name.log"
    if fatal $rc; then echo "FATAL in $name, stopping" | tee -a "$OUT/session.log"; exit $rc; fi
    return 0
}

MODE=${1:-all}
rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
if [[ $MODE == all || $MODE == test ]]; then
    MPGNN_PARITY_REPORT=$OUT/parity.jsonl step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $MODE == all || $MODE == bench ]]; then
    step bench 600 python bench.py --steps 50 --warmup 5
fi
if [[ $MODE == all || $MODE == prof ]]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
fi
echo done
