# Round-5 closing bench lines (every workload; each step under its own limit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final5 bash scripts/bench_all.sh ${BENCH_SET:-full} || exit $?
echo all done
