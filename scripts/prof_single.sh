# rocprofv3 kernel-trace stats of the C3 mode-SINGLE bench (true kernel durations; the bench's
# per-kernel event pass includes host submission gaps for these short kernels)
set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_single
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_single -o run --output-format csv -- \
    python3 bench.py --mode single --steps 20 --warmup 5 --no-cpu-baseline --loop-epochs 0 --epoch-steps 5 > gpurun_out/prof_single/bench.json 2> gpurun_out/prof_single/bench.err
echo ok
